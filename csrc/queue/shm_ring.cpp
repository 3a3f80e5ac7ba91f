// Python bindings of the process-shared request ring (shm_ring.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "queue/shm_ring.h"

namespace py = pybind11;
using llmq::ShmRing;

PYBIND11_MODULE(_shmring, m) {
  m.doc() = "llm_message_queue_amd process-shared MPMC request ring (POSIX shm + robust mutex + futex)";
  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, uint64_t, const std::string&>(), py::arg("name"),
           py::arg("capacity") = 1 << 24, py::arg("mode") = "open")
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
           [](ShmRing& r, size_t max_n, int64_t timeout_ms) {
             std::vector<std::pair<uint32_t, std::string>> v;
             {
               py::gil_scoped_release nogil;
               v = r.pop(max_n, timeout_ms);
             }
             py::list out;
             for (auto& p : v) out.append(py::make_tuple(p.first, py::bytes(p.second)));
             return out;
           },
           py::arg("max_n") = 1024, py::arg("timeout_ms") = 0)
      .def("size", &ShmRing::size)
      .def("bytes_used", &ShmRing::bytes_used)
      .def_property_readonly("capacity", &ShmRing::capacity)
      .def_property_readonly("name", &ShmRing::name)
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
}
