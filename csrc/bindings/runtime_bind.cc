// pybind11 bindings of the native engine runtime (scheduler, block allocator).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime/scheduler.h"

namespace py = pybind11;
using namespace p2p;

void bind_runtime(py::module_& m) {
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int, int>(), py::arg("num_pages"), py::arg("reserved") = 1)
      .def("alloc", &BlockAllocator::alloc)
      .def("free", &BlockAllocator::free)
      .def("can_alloc", &BlockAllocator::can_alloc)
      .def_property_readonly("free_pages", &BlockAllocator::free_count)
      .def_property_readonly("num_pages", &BlockAllocator::num_pages);

  py::class_<SchedRequest>(m, "SchedRequest")
      .def_readonly("id", &SchedRequest::id)
      .def_readonly("prompt_len", &SchedRequest::prompt_len)
      .def_readonly("max_new", &SchedRequest::max_new)
      .def_readonly("state", &SchedRequest::state)
      .def_readonly("pages", &SchedRequest::pages)
      .def_readonly("tokens", &SchedRequest::tokens)
      .def_readonly("pos", &SchedRequest::pos)
      .def_readonly("finish_reason", &SchedRequest::finish_reason);

  py::class_<SchedPlan>(m, "SchedPlan")
      .def_readonly("prefill", &SchedPlan::prefill)
      .def_readonly("decode", &SchedPlan::decode);

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int>(), py::arg("num_pages"), py::arg("page_size"),
           py::arg("max_batch"), py::arg("max_prefill_tokens"), py::arg("max_ctx"))
      .def("add", &Scheduler::add, py::arg("prompt_len"), py::arg("max_new"),
           py::arg("stop_on_eos") = true, py::arg("eos") = std::vector<int>{})
      .def("cancel", &Scheduler::cancel)
      .def("schedule", &Scheduler::schedule)
      .def("on_first_token", &Scheduler::on_first_token)
      .def("on_decode_tokens", &Scheduler::on_decode_tokens)
      .def("take_finished", &Scheduler::take_finished)
      .def("get", &Scheduler::get, py::return_value_policy::copy)
      .def("release", &Scheduler::release)
      .def_property_readonly("n_waiting", &Scheduler::n_waiting)
      .def_property_readonly("n_running", &Scheduler::n_running)
      .def_property_readonly("free_pages", &Scheduler::free_pages)
      .def_property_readonly("page_size", &Scheduler::page_size);
}
