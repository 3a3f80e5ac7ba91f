// Python bindings of the process-shared request ring (shm_ring.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "queue/shm_coll.h"
#include "queue/shm_ring.h"

namespace py = pybind11;
using llmq::ShmCollective;
using llmq::ShmRing;

// the last op's payloads of every rank
static py::list gathered(const ShmCollective& c) {
  py::list out;
  for (int r = 0; r < c.world(); ++r) {
    uint64_t n = 0;
    const uint8_t* p = c.payload(r, &n);
    out.append(py::bytes(reinterpret_cast<const char*>(p), n));
  }
  return out;
}

// all_to_all payload: world x u64 part sizes, then the parts back to back
static std::string a2a_pack(const ShmCollective& c, const std::vector<py::bytes>& parts) {
  const int world = c.world();
  if ((int)parts.size() != world) throw std::invalid_argument("all_to_all: one part per rank");
  std::string buf(sizeof(uint64_t) * world, '\0');
  for (int r = 0; r < world; ++r) {
    std::string s = parts[r];
    const uint64_t n = s.size();
    std::memcpy(&buf[sizeof(uint64_t) * r], &n, sizeof(n));
    buf += s;
  }
  return buf;
}

// after an all_to_all op: the part every rank addressed to this one
static py::list a2a_mine(const ShmCollective& c) {
  py::list out;
  const int world = c.world(), me = c.rank();
  for (int r = 0; r < world; ++r) {
    uint64_t total = 0;
    const uint8_t* p = c.payload(r, &total);
    uint64_t off = sizeof(uint64_t) * world, n = 0;
    for (int d = 0; d < world; ++d) {
      uint64_t sz;
      std::memcpy(&sz, p + sizeof(uint64_t) * d, sizeof(sz));
      if (d == me) n = sz;
      if (d < me) off += sz;
    }
    if (off + n > total) throw std::runtime_error("all_to_all: corrupt payload");
    out.append(py::bytes(reinterpret_cast<const char*>(p + off), n));
  }
  return out;
}

PYBIND11_MODULE(_shmring, m) {
  m.doc() = "llm_message_queue_amd process-shared MPMC request ring (POSIX shm + robust mutex + futex)";
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, uint64_t, const std::string&, uint64_t>(), py::arg("name"),
           py::arg("capacity") = 1 << 24, py::arg("mode") = "open", py::arg("gen") = 0)
      .def("push",
           [](ShmRing& r, py::bytes b, uint32_t tag) {
             std::string s = b;
             py::gil_scoped_release nogil;
             return r.push(s, tag);
           },
           py::arg("record"), py::arg("tag") = 0)
      .def("push_many",
           [](ShmRing& r, const std::vector<py::bytes>& bs, uint32_t tag) {
             std::vector<std::string> v;
             v.reserve(bs.size());
             for (auto& b : bs) v.emplace_back(b);
             py::gil_scoped_release nogil;
             return r.push_many(v, tag);
           },
           py::arg("records"), py::arg("tag") = 0)
      .def("pop",
           [](ShmRing& r, size_t max_n, int64_t timeout_ms, uint32_t share, int who) {
             std::vector<std::pair<uint32_t, std::string>> v;
             {
               py::gil_scoped_release nogil;
               v = r.pop(max_n, timeout_ms, share, who);
             }
             py::list out;
             for (auto& p : v) out.append(py::make_tuple(p.first, py::bytes(p.second)));
             return out;
           },
           py::arg("max_n") = 1024, py::arg("timeout_ms") = 0, py::arg("share") = 1, py::arg("who") = -1)
      .def("taken", &ShmRing::taken, py::arg("n"))
      .def("size", &ShmRing::size)
      .def("bytes_used", &ShmRing::bytes_used)
      .def_property_readonly("capacity", &ShmRing::capacity)
      .def_property_readonly("name", &ShmRing::name)
      .def_property_readonly("generation", &ShmRing::generation)
      .def_property_readonly("creator_pid", &ShmRing::creator_pid)
      .def("stats",
           [](ShmRing& r) {
             auto s = r.stats();
             py::dict d;
             d["size"] = s.size; d["pushed"] = s.pushed; d["popped"] = s.popped;
             d["dropped_full"] = s.dropped_full; d["bytes_in"] = s.bytes_in;
             d["bytes_used"] = s.bytes_used; d["capacity"] = s.capacity;
             return d;
           })
      .def("wake_all", &ShmRing::wake_all)
      .def("close", &ShmRing::close)
      .def("unlink", &ShmRing::unlink);
  py::register_exception<llmq::ShmCollTimeout>(m, "ShmCollTimeout", PyExc_TimeoutError);
  py::class_<ShmCollective>(m, "ShmCollective")
      .def(py::init<const std::string&, int, int, uint64_t, bool>(), py::arg("name"), py::arg("world"),
           py::arg("rank"), py::arg("buf_bytes") = 4 << 20, py::arg("create") = false)
      .def("all_gather",
           [](ShmCollective& c, py::bytes b, double timeout_s) {
             std::string s = b;
             {
               py::gil_scoped_release nogil;
               c.exchange(s.data(), s.size(), timeout_s);
             }
             return gathered(c);
           },
           py::arg("data"), py::arg("timeout_s") = 60.0)
      .def("all_to_all",
           [](ShmCollective& c, const std::vector<py::bytes>& parts, double timeout_s) {
             std::string buf = a2a_pack(c, parts);
             {
               py::gil_scoped_release nogil;
               c.exchange(buf.data(), buf.size(), timeout_s);
             }
             return a2a_mine(c);
           },
           py::arg("parts"), py::arg("timeout_s") = 60.0)
      // split phase: post_* publishes and returns; ready() polls; finish_*
      // waits (GIL released) and returns what all_gather / all_to_all would
      .def("post_gather",
           [](ShmCollective& c, py::bytes b, double timeout_s) {
             std::string s = b;
             py::gil_scoped_release nogil;
             c.post(s.data(), s.size(), timeout_s);
           },
           py::arg("data"), py::arg("timeout_s") = 60.0)
      .def("post_a2a",
           [](ShmCollective& c, const std::vector<py::bytes>& parts, double timeout_s) {
             std::string buf = a2a_pack(c, parts);
             py::gil_scoped_release nogil;
             c.post(buf.data(), buf.size(), timeout_s);
           },
           py::arg("parts"), py::arg("timeout_s") = 60.0)
      .def("ready", &ShmCollective::ready)
      .def("finish_gather",
           [](ShmCollective& c, double timeout_s) {
             {
               py::gil_scoped_release nogil;
               c.complete(timeout_s);
             }
             return gathered(c);
           },
           py::arg("timeout_s") = 60.0)
      .def("finish_a2a",
           [](ShmCollective& c, double timeout_s) {
             {
               py::gil_scoped_release nogil;
               c.complete(timeout_s);
             }
             return a2a_mine(c);
           },
           py::arg("timeout_s") = 60.0)
      .def("attached", &ShmCollective::attached)
      .def("arrived_next", &ShmCollective::arrived_next)
      .def("unlink", &ShmCollective::unlink)
      .def_property_readonly("ops", &ShmCollective::ops)
      .def_property_readonly("world", &ShmCollective::world)
      .def_property_readonly("rank", &ShmCollective::rank)
      .def_property_readonly("buf_bytes", &ShmCollective::buf_bytes);
}
