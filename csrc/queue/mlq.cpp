// Python bindings of the native queue core (mlq_core.h).  Every call that
// can wait or touch many items releases the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "queue/mlq_core.h"

namespace py = pybind11;
using namespace llmq;

namespace {

py::object stats_dict(MultiLevelQueue& q, const std::string& name) {
  Stats s;
  if (!q.stats(name, &s)) return py::none();
  py::dict d;
  d["pending"] = s.pending;
  d["processing"] = s.processing;
  d["completed"] = s.completed;
  d["failed"] = s.failed;
  d["total_wait_ns"] = s.total_wait_ns;
  d["total_process_ns"] = s.total_process_ns;
  d["last_update_ns"] = s.last_update_ns;
  d["pushed"] = s.pushed;
  d["popped"] = s.popped;
  d["rejected_full"] = s.rejected_full;
  return d;
}

std::vector<int> push_batch(MultiLevelQueue& q, const std::vector<std::string>& names, py::array_t<int32_t> qidx,
                            py::array_t<int64_t> handles, py::array_t<int32_t> prios) {
  auto qi = qidx.unchecked<1>();
  auto h = handles.unchecked<1>();
  auto p = prios.unchecked<1>();
  const ssize_t n = h.shape(0);
  if (qi.shape(0) != n || p.shape(0) != n) throw std::invalid_argument("length mismatch");
  py::gil_scoped_release nogil;
  return q.push_batch(names, qi.data(0), h.data(0), p.data(0), n);
}

py::tuple pop_tiers(MultiLevelQueue& q, const std::vector<std::string>& tiers, int64_t count,
                    const std::vector<int64_t>& aging_ns, std::vector<int64_t> budget,
                    const std::vector<int64_t>& lifo_ns, py::array_t<int64_t, py::array::c_style | py::array::forcecast> skip) {
  // skip: handles to leave queued (any order; sorted here for the binary search)
  std::vector<int64_t> sk(skip.data(), skip.data() + skip.size());
  std::sort(sk.begin(), sk.end());
  std::vector<int64_t> hs, enq;
  std::vector<int32_t> ti;
  {
    py::gil_scoped_release nogil;
    hs.reserve(count > 0 ? count : 0);
    q.pop_tiers(tiers, count, aging_ns, std::move(budget), hs, ti, enq, lifo_ns, sk);
  }
  py::array_t<int64_t> a_h(hs.size()), a_e(enq.size());
  py::array_t<int32_t> a_t(ti.size());
  std::copy(hs.begin(), hs.end(), a_h.mutable_data());
  std::copy(enq.begin(), enq.end(), a_e.mutable_data());
  std::copy(ti.begin(), ti.end(), a_t.mutable_data());
  return py::make_tuple(a_h, a_t, a_e);
}

}  // namespace

PYBIND11_MODULE(_mlq, m) {
  m.doc() = "llm_message_queue_amd native queue core (MultiLevelQueue, DelayedQueue)";
  m.attr("OK") = (int)OK;
  m.attr("QUEUE_NOT_FOUND") = (int)QUEUE_NOT_FOUND;
  m.attr("QUEUE_FULL") = (int)QUEUE_FULL;
  m.attr("QUEUE_EMPTY") = (int)QUEUE_EMPTY;
  m.def("mono_ns", &llmq::mono_ns);

  py::class_<MultiLevelQueue>(m, "MultiLevelQueue")
      .def(py::init<int64_t>(), py::arg("max_size") = 0)
      .def("add_queue", &MultiLevelQueue::add_queue, py::arg("name"), py::arg("max_size") = -1)
      .def("remove_queue", &MultiLevelQueue::remove_queue)
      .def("has_queue", &MultiLevelQueue::has_queue)
      .def("names", &MultiLevelQueue::names)
      .def("push", &MultiLevelQueue::push)
      .def("push_batch", &push_batch)
      .def("pop", &MultiLevelQueue::pop)
      .def("peek", &MultiLevelQueue::peek)
      .def("pop_batch", &MultiLevelQueue::pop_batch, py::call_guard<py::gil_scoped_release>())
      .def("pop_tiers", &pop_tiers, py::arg("tiers"), py::arg("count"), py::arg("aging_ns"), py::arg("budget"),
           py::arg("lifo_ns") = std::vector<int64_t>{}, py::arg("skip") = py::array_t<int64_t>(0))
      .def("size", &MultiLevelQueue::size)
      .def("total_size", &MultiLevelQueue::total_size)
      .def("stats", &stats_dict)
      .def("complete", &MultiLevelQueue::complete)
      .def("fail", &MultiLevelQueue::fail)
      .def("unprocess", &MultiLevelQueue::unprocess)
      .def("remove", &MultiLevelQueue::remove)
      .def("snapshot", &MultiLevelQueue::snapshot)
      .def("clear", &MultiLevelQueue::clear)
      .def_property_readonly("max_size", &MultiLevelQueue::max_size);

  py::class_<DelayedQueue>(m, "DelayedQueue")
      .def(py::init<>())
      .def("schedule", &DelayedQueue::schedule)
      .def("remove", &DelayedQueue::remove)
      .def("wait_ready", &DelayedQueue::wait_ready, py::call_guard<py::gil_scoped_release>())
      .def("size", &DelayedQueue::size)
      .def("ready_size", &DelayedQueue::ready_size)
      .def("peek", &DelayedQueue::peek)
      .def("clear", &DelayedQueue::clear)
      .def("shutdown", &DelayedQueue::shutdown, py::call_guard<py::gil_scoped_release>());
}
