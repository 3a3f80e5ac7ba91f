// pybind11 module _textcpu: the CPU preprocess analyzer (text_cpu.h) over a
// packed batch -- the same bytes + offsets + pattern table the GPU pipeline
// stages (ops/text.py), the same stats / hashes layout it reads back.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "text/text_cpu.h"

namespace py = pybind11;
using llmq::textcpu::Analyzer;
using llmq::textcpu::PatternTable;

static void analyze(py::array_t<uint8_t, py::array::c_style> bytes, py::array_t<int64_t, py::array::c_style> offsets,
                    int B, int L, py::bytes table, py::array_t<int32_t, py::array::c_style> stats,
                    py::array_t<uint32_t, py::array::c_style> hashes) {
  const std::string t = table;
  if (t.size() != sizeof(PatternTable)) throw std::invalid_argument("pattern table size mismatch");
  PatternTable pt;
  std::memcpy(&pt, t.data(), sizeof(pt));
  if (pt.npat < 0 || pt.npat > llmq::textcpu::MAX_PAT) throw std::invalid_argument("npat out of range");
  for (int j = 0; j < pt.npat; ++j)
    if (pt.len[j] < 1 || pt.len[j] > 16 || pt.slot[j] < 0 || pt.slot[j] >= llmq::textcpu::SLOTS)
      throw std::invalid_argument("pattern length / slot out of range");
  if (B < 0 || L < 1) throw std::invalid_argument("bad B / L");
  if (offsets.size() < B + 1 || stats.size() < (py::ssize_t)B * llmq::textcpu::STAT_COLS ||
      hashes.size() < (py::ssize_t)B * L)
    throw std::invalid_argument("output / offsets arrays too small");
  const int64_t* off = offsets.data();
  const int64_t nbytes = (int64_t)bytes.size();
  for (int i = 0; i < B; ++i)
    if (off[i] < 0 || off[i + 1] < off[i] || off[i + 1] > nbytes) throw std::invalid_argument("bad offsets");
  const uint8_t* src = bytes.data();
  int32_t* st = stats.mutable_data();
  uint32_t* h = hashes.mutable_data();
  py::gil_scoped_release nogil;
  const Analyzer an(pt, L);
  auto run = [&](int i0, int i1) {
    for (int i = i0; i < i1; ++i)
      an.analyze(src + off[i], (int)(off[i + 1] - off[i]), st + (int64_t)i * llmq::textcpu::STAT_COLS,
                 h + (int64_t)i * L);
  };
  // large batches (an ingest backlog) split over a few threads; messages are
  // independent and each writes only its own rows
  const int nt = B >= 2048 ? (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 8u) : 1;
  if (nt <= 1) {
    run(0, B);
    return;
  }
  std::vector<std::thread> th;
  const int per = (B + nt - 1) / nt;
  for (int t = 1; t < nt; ++t) th.emplace_back(run, std::min(B, t * per), std::min(B, (t + 1) * per));
  run(0, std::min(B, per));
  for (auto& x : th) x.join();
}

PYBIND11_MODULE(_textcpu, m) {
  m.doc() = "CPU twin of the text_analyze kernel (exact Go preprocessor semantics)";
  m.def("analyze", &analyze, py::arg("bytes"), py::arg("offsets"), py::arg("B"), py::arg("L"), py::arg("table"),
        py::arg("stats"), py::arg("hashes"));
  m.attr("STAT_COLS") = llmq::textcpu::STAT_COLS;
  m.attr("PATTERN_TABLE_BYTES") = (int)sizeof(PatternTable);
}
