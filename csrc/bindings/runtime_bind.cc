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

// ---------------------------------------------------------------- native engine loop
#include <pybind11/functional.h>

#include "runtime/engine_loop.h"
#include "runtime/hip_dyn.h"
#include "runtime/loop_capi.h"
#include "runtime/mirror.h"

namespace {

template <class T>
T* ptr_of(const py::dict& d, const char* k) {
  return d.contains(k) ? reinterpret_cast<T*>(py::cast<uintptr_t>(d[k])) : nullptr;
}

template <class T>
T val_of(const py::dict& d, const char* k, T def) {
  return d.contains(k) ? py::cast<T>(d[k]) : def;
}

LoopConfig loop_cfg(const py::dict& d) {
  LoopConfig c;
  c.num_pages = val_of<int>(d, "num_pages", 0);
  c.page_size = val_of<int>(d, "page_size", 64);
  c.max_batch = val_of<int>(d, "max_batch", 16);
  c.max_prefill_tokens = val_of<int>(d, "max_prefill_tokens", 1024);
  c.max_ctx = val_of<int>(d, "max_ctx", 4096);
  c.eos = val_of<std::vector<int>>(d, "eos", {});
  c.decode_chunk = val_of<int>(d, "decode_chunk", 8);
  c.admit_wait_us = val_of<double>(d, "admit_wait_us", 500.0);
  c.prefill_first = val_of<bool>(d, "prefill_first", true);
  c.mixed = val_of<bool>(d, "mixed", true);
  c.riders_all = val_of<bool>(d, "riders_all", false);
  c.pipeline = val_of<bool>(d, "pipeline", true);
  c.device = val_of<int>(d, "device", 0);
  if (d.contains("batch_buckets")) c.batch_buckets = py::cast<std::vector<int>>(d["batch_buckets"]);
  if (d.contains("ctx_buckets")) c.ctx_buckets = py::cast<std::vector<int>>(d["ctx_buckets"]);
  if (d.contains("row_buckets")) c.row_buckets = py::cast<std::vector<int>>(d["row_buckets"]);
  c.prefill_max_pages = val_of<int>(d, "prefill_max_pages", 64);
  c.prefill_graph_after = val_of<int>(d, "prefill_graph_after", 2);
  c.pipeline_free_slots = val_of<bool>(d, "pipeline_free_slots", false);
  c.dp_world = val_of<int>(d, "dp_world", 1);
  return c;
}

DecodeGraphDesc decode_desc(const py::dict& d) {
  DecodeGraphDesc g;
  g.B = val_of<int>(d, "B", 0);
  g.max_pages = val_of<int>(d, "max_pages", 0);
  g.ctx = val_of<int>(d, "ctx", 0);
  g.greedy = val_of<bool>(d, "greedy", true);
  g.exec = ptr_of<void>(d, "exec");
  g.meta = ptr_of<int32_t>(d, "meta");
  g.hist = ptr_of<int32_t>(d, "hist");
  g.max_steps = val_of<int>(d, "max_steps", 0);
  g.step = ptr_of<int32_t>(d, "step");
  g.keys = ptr_of<void>(d, "keys");
  g.keys_bytes = val_of<size_t>(d, "keys_bytes", 0);
  g.temp = ptr_of<float>(d, "temp");
  g.topk = ptr_of<int32_t>(d, "topk");
  g.topp = ptr_of<float>(d, "topp");
  g.seeds = ptr_of<int64_t>(d, "seeds");
  g.err = ptr_of<int32_t>(d, "err");
  g.exec_k = ptr_of<void>(d, "exec_k");
  g.k_steps = val_of<int>(d, "k_steps", 0);
  if (!g.exec || !g.meta || !g.hist || !g.step || g.B <= 0 || g.max_steps <= 0 ||
      (!g.greedy && !(g.temp && g.topk && g.topp && g.seeds)))
    throw std::runtime_error("add_decode_graph: incomplete description");
  return g;
}

PrefillGraphDesc prefill_desc(const py::dict& d) {
  PrefillGraphDesc g;
  g.rows = val_of<int>(d, "rows", 0);
  g.n_seq = val_of<int>(d, "n_seq", 0);
  g.max_pages = val_of<int>(d, "max_pages", 0);
  g.qtile = val_of<int>(d, "qtile", 16);
  g.max_tiles = val_of<int>(d, "max_tiles", 0);
  g.greedy = val_of<bool>(d, "greedy", true);
  g.exec = ptr_of<void>(d, "exec");
  g.meta = ptr_of<int32_t>(d, "meta");
  g.meta_len = val_of<size_t>(d, "meta_len", 0);
  g.off_bt = val_of<size_t>(d, "off_bt", 0);
  g.off_seq = val_of<size_t>(d, "off_seq", 0);
  g.off_pos = val_of<size_t>(d, "off_pos", 0);
  g.off_ids = val_of<size_t>(d, "off_ids", 0);
  g.off_slots = val_of<size_t>(d, "off_slots", 0);
  g.off_ctx = val_of<size_t>(d, "off_ctx", 0);
  g.off_out = val_of<size_t>(d, "off_out", 0);
  g.off_spos = val_of<size_t>(d, "off_spos", 0);
  g.off_tiles = val_of<size_t>(d, "off_tiles", 0);
  g.first = ptr_of<int32_t>(d, "first");
  g.temp = ptr_of<float>(d, "temp");
  g.topk = ptr_of<int32_t>(d, "topk");
  g.topp = ptr_of<float>(d, "topp");
  g.seeds = ptr_of<int64_t>(d, "seeds");
  g.err = ptr_of<int32_t>(d, "err");
  if (!g.exec || !g.meta || !g.first || g.rows <= 0 || g.n_seq <= 0 || !g.meta_len ||
      (!g.greedy && !(g.temp && g.topk && g.topp && g.seeds)))
    throw std::runtime_error("add_prefill_graph: incomplete description");
  return g;
}

EngineLoop::GraphProvider py_provider(py::function f) {
  auto fn = std::make_shared<py::function>(std::move(f));
  return [fn](const std::string& kind, int a, int b, bool greedy) {
    py::gil_scoped_acquire gil;
    try {
      (*fn)(kind, a, b, greedy);
    } catch (py::error_already_set& e) {  // formatted here, with the GIL held
      throw std::runtime_error(std::string("graph provider raised: ") + e.what());
    }
  };
}

EngineLoop::EagerPrefill py_eager(py::function f) {
  auto fn = std::make_shared<py::function>(std::move(f));
  return [fn](const std::vector<std::vector<int>>& prompts, const std::vector<std::vector<int>>& pages,
              const std::vector<int>& starts, const std::vector<LoopSampling>& samp, int pad_rows) {
    py::gil_scoped_acquire gil;
    try {
      py::list sp;
      for (auto& s : samp) sp.append(py::make_tuple(s.temperature, s.top_k, s.top_p, s.seed));
      if (pad_rows > 0)  // EP a2a groups (LoopConfig::dp_world): exactly this many rows
        return py::cast<std::vector<int>>((*fn)(prompts, pages, starts, sp, pad_rows));
      return py::cast<std::vector<int>>((*fn)(prompts, pages, starts, sp));
    } catch (py::error_already_set& e) {
      throw std::runtime_error(std::string("eager prefill raised: ") + e.what());
    }
  };
}

}  // namespace

void bind_engine_loop(py::module_& m) {
  m.def("loop_use_host_fake_hip", &hip_api_use_host_fake,
        "tests: run the native engine loop on host memory with host-function 'graphs'");
  py::class_<EngineLoop>(m, "EngineLoop")
      .def(py::init([](py::dict d) { return new EngineLoop(loop_cfg(d)); }))
      .def("add_decode_graph", [](EngineLoop& L, py::dict d) { L.add_decode_graph(decode_desc(d)); })
      .def("add_prefill_graph", [](EngineLoop& L, py::dict d) { L.add_prefill_graph(prefill_desc(d)); })
      .def("set_provider", [](EngineLoop& L, py::function f) { L.set_provider(py_provider(f)); })
      .def("set_eager_prefill",
           [](EngineLoop& L, py::function f) { L.set_eager_prefill(py_eager(f)); })
      // TP / EP group leader: record every device operation for the followers (mirror.h)
      .def("set_mirror", &EngineLoop::set_mirror)
      .def("set_aux_fault", &EngineLoop::set_aux_fault, py::arg("word"))
      .def("set_coll_fault", &EngineLoop::set_coll_fault, py::arg("word"))
      .def("serve", &EngineLoop::serve, py::arg("name"))
      .def("mirror_provide", &EngineLoop::mirror_provide, py::call_guard<py::gil_scoped_release>())
      .def("start", &EngineLoop::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &EngineLoop::stop, py::call_guard<py::gil_scoped_release>())
      .def("shutdown", &EngineLoop::shutdown, py::call_guard<py::gil_scoped_release>())
      .def("submit",
           [](EngineLoop& L, const std::vector<int>& prompt, int max_new, bool stop_on_eos,
              float temperature, int top_k, float top_p, int64_t seed) {
             LoopSampling s;
             s.temperature = temperature;
             s.top_k = top_k;
             s.top_p = top_p;
             s.seed = seed;
             py::gil_scoped_release rel;
             return L.submit(prompt, max_new, stop_on_eos, s);
           },
           py::arg("prompt"), py::arg("max_new"), py::arg("stop_on_eos") = true,
           py::arg("temperature") = 0.f, py::arg("top_k") = 40, py::arg("top_p") = 0.9f,
           py::arg("seed") = 0)
      .def("cancel", &EngineLoop::cancel, py::call_guard<py::gil_scoped_release>())
      .def("release", &EngineLoop::release, py::call_guard<py::gil_scoped_release>())
      .def("stall", &EngineLoop::stall, py::call_guard<py::gil_scoped_release>())
      .def("wait",
           [](EngineLoop& L, int64_t id, double timeout_s) {
             LoopResult r;
             {
               py::gil_scoped_release rel;
               L.wait(id, timeout_s, &r);
             }
             py::dict d;
             d["tokens"] = r.tokens;
             d["done"] = r.done;
             d["done_reason"] = r.done_reason;
             d["error"] = r.error;
             d["prompt_eval_count"] = r.prompt_eval_count;
             d["prompt_eval_duration"] = r.prompt_eval_ns;
             d["eval_count"] = (int)r.tokens.size();
             d["eval_duration"] = r.eval_ns;
             d["total_duration"] = r.total_ns;
             d["ttft_ns"] = r.ttft_ns;
             return d;
           })
      .def("wait_tokens",
           [](EngineLoop& L, int64_t id, size_t have, double timeout_s) {
             bool done = false;
             std::vector<int> t;
             {
               py::gil_scoped_release rel;
               t = L.wait_tokens(id, have, timeout_s, &done);
             }
             return py::make_tuple(t, done);
           })
      .def("metrics", &EngineLoop::metrics, py::call_guard<py::gil_scoped_release>())
      .def("dead", &EngineLoop::dead, py::call_guard<py::gil_scoped_release>())
      // the loop's address, for native front ends driving it through p2p_loop_api()
      .def("handle", [](EngineLoop& L) { return (uintptr_t)&L; });
  // address of the plain-C table (runtime/loop_capi.h) of the loop code in THIS module
  m.def("loop_api", []() { return (uintptr_t)p2p_loop_api(); });
  // TP / EP group follower: applies the leader loop's device operations (mirror.h)
  py::class_<EngineMirror>(m, "EngineMirror")
      .def(py::init<int, int>(), py::arg("fd"), py::arg("device"))
      .def("add_decode_graph", [](EngineMirror& M, py::dict d) { M.add_decode_graph(decode_desc(d)); })
      .def("add_prefill_graph", [](EngineMirror& M, py::dict d) { M.add_prefill_graph(prefill_desc(d)); })
      .def("set_provider", [](EngineMirror& M, py::function f) { M.set_provider(py_provider(f)); })
      .def("set_eager_prefill", [](EngineMirror& M, py::function f) { M.set_eager_prefill(py_eager(f)); })
      .def("set_aux_fault", &EngineMirror::set_aux_fault, py::arg("word"))
      .def("set_coll_fault", &EngineMirror::set_coll_fault, py::arg("word"))
      .def("run", &EngineMirror::run, py::call_guard<py::gil_scoped_release>())
      .def("metrics", &EngineMirror::metrics)
      .def("shutdown", &EngineMirror::shutdown, py::call_guard<py::gil_scoped_release>());
}
