// Engine C ABI -- see engine_capi.h.
//
// Python builds the engine once (p2p_engine_create: weights, autotune, graph captures, the
// native step loop).  When the server runs on the native loop (engine/native_loop.py) the
// requests never enter the interpreter: the Ollama JSON is parsed here, the prompt is
// tokenised by the native tokenizer (engine/native_tok.h), EngineLoop::submit / wait /
// wait_tokens run through the loop's plain-C table (runtime/loop_capi.h), and the reply is
// detokenised and serialised here.  Python is entered per request only for what the
// native side does not implement (a real BPE tokenizer, non-ASCII text, the metrics
// endpoint, or the Python loop of a TP/EP group); `capi_gil_entries` in the metrics
// counts those entries.
#include "engine_capi.h"

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <cmath>

#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "engine/native_tok.h"
#include "net/json.h"
#include "runtime/loop_capi.h"
#include "runtime/loop_remote.h"

using p2p::Json;

namespace {

// the native request path of a server on the native loop
struct Front {
  const P2PLoopApi* api = nullptr;
  void* loop = nullptr;
  bool remote = false;  // loop is a RemoteLoops over the replicas' sockets (loop_remote.h)
  p2p::NativeTok tok;
  std::string model;
  int default_max = 128;
  double timeout_s = 60.0;
  std::atomic<long> requests{0}, native_requests{0}, python_tokenize{0}, python_decode{0};
};

std::atomic<long> g_gil_entries{0};  // PyGILState_Ensure calls after create (per request)

}  // namespace

struct p2p_engine {
  PyObject* server = nullptr;  // engine.server.EngineServer / NativeEngineServer / cluster
  std::unique_ptr<Front> front;
};

namespace {

thread_local std::string t_err;
std::once_flag g_init;
bool g_init_ok = false;

// The package root: two levels above this library (p2p_llm_chat_go_amd/_lib/).
std::string package_root() {
  Dl_info info{};
  if (!dladdr((void*)&package_root, &info) || !info.dli_fname) return "";
  std::string p = info.dli_fname;
  for (int i = 0; i < 3; ++i) {
    const size_t s = p.rfind('/');
    if (s == std::string::npos) return "";
    p.resize(s);
  }
  return p;
}

std::string py_error() {
  PyObject *t = nullptr, *v = nullptr, *tb = nullptr;
  PyErr_Fetch(&t, &v, &tb);
  PyErr_NormalizeException(&t, &v, &tb);
  std::string msg = "python error";
  if (v) {
    PyObject* s = PyObject_Str(v);
    if (s) {
      const char* c = PyUnicode_AsUTF8(s);
      if (c) msg = c;
      Py_DECREF(s);
    }
  }
  Py_XDECREF(t);
  Py_XDECREF(v);
  Py_XDECREF(tb);
  return msg;
}

void init_python() {
  // extension modules (torch, the pybind module) resolve libpython symbols globally
  dlopen("libpython3.10.so.1.0", RTLD_NOW | RTLD_GLOBAL);
  const bool own = !Py_IsInitialized();
  if (own) Py_InitializeEx(0);
  PyGILState_STATE g = PyGILState_Ensure();
  const std::string root = package_root();
  if (!root.empty()) {
    PyObject* path = PySys_GetObject("path");  // borrowed
    PyObject* r = PyUnicode_FromString(root.c_str());
    if (path && r) PyList_Insert(path, 0, r);
    Py_XDECREF(r);
  }
  g_init_ok = true;
  PyGILState_Release(g);
  if (own) PyEval_SaveThread();  // other threads take the GIL through PyGILState_Ensure
}

char* dup_utf8(PyObject* s) {
  const char* c = s ? PyUnicode_AsUTF8(s) : nullptr;
  return c ? strdup(c) : nullptr;
}

struct EmitCtx {
  p2p_engine_emit_fn fn;
  void* ctx;
};

// Python-callable emit(chunk_text) -> bool, wrapping the C callback (GIL released around it:
// the callback writes to a socket)
PyObject* py_emit(PyObject* self, PyObject* arg) {
  auto* ec = (EmitCtx*)PyCapsule_GetPointer(self, "p2p_emit");
  const char* chunk = PyUnicode_AsUTF8(arg);
  if (!ec || !chunk) return nullptr;
  int ok;
  Py_BEGIN_ALLOW_THREADS ok = ec->fn(chunk, ec->ctx);
  Py_END_ALLOW_THREADS return PyBool_FromLong(ok != 0);
}

PyMethodDef g_emit_def = {"emit", (PyCFunction)py_emit, METH_O, nullptr};

}  // namespace

// ------------------------------------------------------------------ native request path
namespace {

struct Gil {  // a counted PyGILState_Ensure (every entry after create shows in the metrics)
  PyGILState_STATE g;
  Gil() : g(PyGILState_Ensure()) { g_gil_entries++; }
  ~Gil() { PyGILState_Release(g); }
};

std::string now_rfc3339() {  // the Python servers' created_at: seconds, ".000000Z"
  char buf[64];
  const time_t t = time(nullptr);
  struct tm tm;
  gmtime_r(&t, &tm);
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm);
  return std::string(buf) + ".000000Z";
}

std::string fmt_g(double v) {
  char b[64];
  snprintf(b, sizeof b, "%g", v);
  return b;
}

bool truthy(const Json& v) {
  switch (v.type()) {
    case Json::Null: return false;
    case Json::Bool: return v.boolean();
    case Json::Number: return v.num() != 0.0;
    case Json::String: return !v.str().empty();
    case Json::Array: return v.size() > 0;
    default: return !v.fields().empty();
  }
}

// Python float(x) / int(x) of a JSON number or bool; false for anything else (the request
// then takes the Python path, which raises the same error Python would)
bool as_double(const Json& v, double* out) {
  if (v.is_number()) return *out = v.num(), true;
  if (v.is_bool()) return *out = v.boolean() ? 1.0 : 0.0, true;
  return false;
}

struct Params {
  int max_new = 128;
  bool stop_on_eos = true;
  float temperature = 0.f, top_p = 0.9f;
  int top_k = 40;
  int64_t seed = 0;
};

// SamplingParams.from_ollama + resolved_seed
bool parse_params(const Json& req, int default_max, Params* p) {
  const Json& o = req.get("options");
  if (!o.is_null() && !o.is_object()) return false;
  double v;
  int64_t n = default_max;
  if (o.has("num_predict")) {
    if (!as_double(o.get("num_predict"), &v)) return false;
    n = (int64_t)v;  // int() truncates
  }
  if (n < 0) n = default_max;
  p->max_new = (int)std::max<int64_t>(1, std::min<int64_t>(n, 1 << 30));
  p->temperature = 0.f;
  if (o.has("temperature")) {
    if (!as_double(o.get("temperature"), &v)) return false;
    p->temperature = (float)v;
  }
  if (o.has("top_k")) {
    if (!as_double(o.get("top_k"), &v)) return false;
    p->top_k = (int)v;
  }
  if (o.has("top_p")) {
    if (!as_double(o.get("top_p"), &v)) return false;
    p->top_p = (float)v;
  }
  p->stop_on_eos = !truthy(o.get("ignore_eos"));
  p->seed = 0;
  if (p->temperature > 0.f) {  // greedy requests carry seed 0 (NativeEngineServer._submit)
    const Json& sd = o.get("seed");
    if (sd.is_null()) {
      static thread_local std::mt19937_64 rng{std::random_device{}()};
      p->seed = (int64_t)(rng() >> 2);  // random.getrandbits(62)
    } else {
      // int(seed) & (2**63 - 1) exactly: beyond 2**53 a JSON number has lost its low bits
      // in the double, so those seeds (and non-numbers) take the Python path
      if (!as_double(sd, &v) || !(std::fabs(v) < 9007199254740992.0)) return false;
      p->seed = (int64_t)v & INT64_MAX;
    }
  }
  return true;
}

// prompt ids natively; false = ask Python (encode_request)
bool native_ids(const Front& f, const Json& req, std::vector<int>* ids) {
  if (!f.tok.ok) return false;
  if (req.get_string("endpoint") == "chat") return f.tok.messages_ids(req.get("messages"), ids);
  // a missing prompt is ""; an explicit null (or any non-string) goes to Python, which
  // raises on it as it always did
  const Json& pr = req.get("prompt");
  if (req.has("prompt") && !pr.is_string()) return false;
  const std::string prompt = pr.is_string() ? pr.str() : "";
  if (truthy(req.get("raw"))) {
    ids->push_back(f.tok.bos);
    return f.tok.encode(prompt, ids);
  }
  return f.tok.chat_ids(prompt, ids);
}

std::vector<int> py_int_list(PyObject* r) {
  std::vector<int> out;
  PyObject* seq = r ? PySequence_Fast(r, "ids") : nullptr;
  if (!seq) return out;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t i = 0; i < n; ++i)
    out.push_back((int)PyLong_AsLong(PySequence_Fast_GET_ITEM(seq, i)));
  Py_DECREF(seq);
  return out;
}

bool request_ids(p2p_engine* e, const Json& req, const char* req_text, std::vector<int>* ids) {
  if (native_ids(*e->front, req, ids)) return true;
  ids->clear();
  e->front->python_tokenize++;
  Gil g;
  PyObject* r = PyObject_CallMethod(e->server, "encode_request", "s", req_text);
  if (!r) {
    t_err = py_error();
    return false;
  }
  *ids = py_int_list(r);
  Py_DECREF(r);
  return true;
}

std::string decode_text(p2p_engine* e, const std::vector<int>& toks) {
  if (e->front->tok.ok) return e->front->tok.decode(toks);
  e->front->python_decode++;
  Gil g;
  PyObject* lst = PyList_New((Py_ssize_t)toks.size());
  for (size_t i = 0; i < toks.size(); ++i) PyList_SET_ITEM(lst, i, PyLong_FromLong(toks[i]));
  PyObject* r = PyObject_CallMethod(e->server, "decode_ids", "O", lst);
  Py_DECREF(lst);
  std::string out;
  if (r && PyUnicode_AsUTF8(r)) out = PyUnicode_AsUTF8(r);
  if (!r) PyErr_Clear();
  Py_XDECREF(r);
  return out;
}

Json final_object(const Json& model, const P2PLoopResult& r, bool chat, const std::string& text) {
  Json out = Json::object();
  out.set("model", model);
  out.set("created_at", now_rfc3339());
  out.set("done", true);
  out.set("done_reason", std::string(r.done_reason));
  out.set("total_duration", (long long)r.total_ns);
  out.set("load_duration", 0);
  out.set("prompt_eval_count", r.prompt_eval_count);
  out.set("prompt_eval_duration", (long long)r.prompt_eval_ns);
  out.set("eval_count", r.n_tokens);
  out.set("eval_duration", (long long)r.eval_ns);
  if (chat) {
    Json m = Json::object();
    m.set("role", "assistant");
    m.set("content", text);
    out.set("message", m);
  } else {
    out.set("response", text);
    out.set("context", Json::array());
  }
  return out;
}

struct ReqCtx {
  Json req;
  Json model;
  bool chat = false;
  Params p;
  std::vector<int> ids;
};

// 1: native (ctx filled), 0: take the Python path, -1: failed (t_err set)
int prepare(p2p_engine* e, const char* req_text, ReqCtx* c) {
  try {
    c->req = Json::parse(req_text);
  } catch (const std::exception&) {
    return 0;  // Python reports the parse error
  }
  if (!c->req.is_object()) return 0;
  const std::string ep = c->req.get_string("endpoint");
  if (!ep.empty() && ep != "chat" && ep != "generate") return 0;  // metrics, ...
  c->chat = ep == "chat";
  if (!parse_params(c->req, e->front->default_max, &c->p)) return 0;
  c->model = c->req.has("model") ? c->req.get("model") : Json(e->front->model);
  if (!request_ids(e, c->req, req_text, &c->ids)) return -1;
  return 1;
}

int64_t submit(p2p_engine* e, const ReqCtx& c) {
  Front& f = *e->front;
  char err[512] = {0};
  std::vector<int32_t> ids(c.ids.begin(), c.ids.end());
  const int64_t id = f.api->submit(f.loop, ids.data(), (int)ids.size(), c.p.max_new,
                                   c.p.stop_on_eos ? 1 : 0, c.p.temperature, c.p.top_k,
                                   c.p.top_p, c.p.seed, err, sizeof err);
  if (id < 0) t_err = err[0] ? err : "engine refused the request";
  f.requests++;
  return id;
}

std::string timeout_msg(double t) {
  return "engine did not answer within " + fmt_g(t) + "s (request cancelled)";
}

char* native_generate(p2p_engine* e, const ReqCtx& c) {
  Front& f = *e->front;
  const int64_t id = submit(e, c);
  if (id < 0) return nullptr;
  P2PLoopResult r;
  f.api->wait(f.loop, id, f.timeout_s > 0 ? f.timeout_s : -1.0, &r);
  f.api->release(f.loop, id);  // done: forgotten; else cancelled, dropped when it ends
  std::vector<int> toks(r.tokens, r.tokens + r.n_tokens);
  char* out = nullptr;
  if (r.error) {
    t_err = r.error;
  } else if (!r.done) {
    t_err = timeout_msg(f.timeout_s);
  } else {
    out = strdup(final_object(c.model, r, c.chat, decode_text(e, toks)).dump().c_str());
    f.native_requests++;
  }
  f.api->free_mem(r.tokens);
  f.api->free_mem(r.error);
  return out;
}

char* native_stream(p2p_engine* e, const ReqCtx& c, p2p_engine_emit_fn emit, void* ctx) {
  Front& f = *e->front;
  const int64_t id = submit(e, c);
  if (id < 0) return nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<int> toks;
  std::string sent;
  bool alive = true;
  auto flush = [&](bool final) {
    const std::string text = decode_text(e, toks);
    if (!final && text.size() >= 3 && text.compare(text.size() - 3, 3, "\xef\xbf\xbd") == 0)
      return;  // incomplete UTF-8 sequence: wait for the next token
    const std::string delta =
        text.compare(0, sent.size(), sent) == 0 ? text.substr(sent.size()) : text;
    sent = text;
    if (delta.empty() || !alive) return;
    Json ch = Json::object();
    ch.set("model", c.model);
    ch.set("created_at", now_rfc3339());
    ch.set("done", false);
    if (c.chat) {
      Json m = Json::object();
      m.set("role", "assistant");
      m.set("content", delta);
      ch.set("message", m);
    } else {
      ch.set("response", delta);
    }
    alive = emit(ch.dump().c_str(), ctx) != 0;
    if (!alive) f.api->cancel(f.loop, id);  // the client went away: stop generating for it
  };
  while (true) {
    int32_t* nt = nullptr;
    int n = 0, done = 0;
    f.api->wait_tokens(f.loop, id, toks.size(), 0.05, &nt, &n, &done);
    toks.insert(toks.end(), nt, nt + n);
    f.api->free_mem(nt);
    if (n) flush(false);
    if (done) break;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (f.timeout_s > 0 && el > f.timeout_s) {
      f.api->release(f.loop, id);
      t_err = timeout_msg(f.timeout_s);
      return nullptr;
    }
  }
  P2PLoopResult r;
  f.api->wait(f.loop, id, 0.0, &r);
  f.api->release(f.loop, id);
  char* out = nullptr;
  if (r.error) {
    t_err = r.error;
  } else {
    toks.assign(r.tokens, r.tokens + r.n_tokens);
    flush(true);
    out = strdup(final_object(c.model, r, c.chat, "").dump().c_str());
    f.native_requests++;
  }
  f.api->free_mem(r.tokens);
  f.api->free_mem(r.error);
  return out;
}

// the server's native_front() (NativeEngineServer), if it has one
void attach_front(p2p_engine* e) {
  if (!PyObject_HasAttrString(e->server, "native_front")) return;
  PyObject* d = PyObject_CallMethod(e->server, "native_front", nullptr);
  if (!d || !PyDict_Check(d)) {
    PyErr_Clear();
    Py_XDECREF(d);
    return;
  }
  auto f = std::make_unique<Front>();
  auto item = [&](const char* k) { return PyDict_GetItemString(d, k); };  // borrowed
  if (PyObject* v = item("api")) f->api = (const P2PLoopApi*)PyLong_AsVoidPtr(v);
  if (PyObject* v = item("loop")) f->loop = PyLong_AsVoidPtr(v);
  if (PyObject* v = item("cluster")) {  // multi-GPU node: the replica leaders' loop sockets
    std::vector<std::string> names;
    const Py_ssize_t n = PyList_Check(v) ? PyList_Size(v) : 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
      const char* c = PyUnicode_AsUTF8(PyList_GetItem(v, i));
      if (c) names.push_back(c);
    }
    if (!names.empty() && (Py_ssize_t)names.size() == n) {
      f->api = p2p::remote_loop_api();
      f->loop = p2p::remote_loops_create(names);
      f->remote = true;
    }
  }
  if (PyObject* v = item("model")) f->model = PyUnicode_AsUTF8(v) ? PyUnicode_AsUTF8(v) : "";
  if (PyObject* v = item("default_max_tokens")) f->default_max = (int)PyLong_AsLong(v);
  if (PyObject* v = item("timeout_s")) f->timeout_s = PyFloat_AsDouble(v);
  if (PyObject* v = item("tokenizer")) {
    const char* spec = PyUnicode_AsUTF8(v);
    try {
      if (spec) f->tok.load(spec);
    } catch (const std::exception&) {
      f->tok = p2p::NativeTok();
    }
  }
  PyErr_Clear();
  Py_DECREF(d);
  if (f->api && f->api->version == P2P_LOOP_API_VERSION && f->loop) e->front = std::move(f);
}

char* python_call(p2p_engine* e, const char* method, const char* req, PyObject* extra) {
  Gil g;
  PyObject* r = extra ? PyObject_CallMethod(e->server, method, "sO", req, extra)
                      : PyObject_CallMethod(e->server, method, "s", req);
  char* out = dup_utf8(r);
  if (!out) t_err = py_error();
  Py_XDECREF(r);
  return out;
}

}  // namespace

extern "C" {

p2p_engine* p2p_engine_create(const char* model, const char* device) {
  std::call_once(g_init, init_python);
  if (!g_init_ok) {
    t_err = "python interpreter failed to start";
    return nullptr;
  }
  PyGILState_STATE g = PyGILState_Ensure();
  p2p_engine* e = nullptr;
  PyObject* mod = PyImport_ImportModule("p2p_llm_chat_go_amd.net.node");
  if (mod) {
    PyObject* srv = PyObject_CallMethod(mod, "build_engine_server", "zz",
                                        (model && *model) ? model : nullptr,
                                        (device && *device) ? device : nullptr);
    if (srv) {
      e = new p2p_engine;
      e->server = srv;
      attach_front(e);
    }
    Py_DECREF(mod);
  }
  if (!e) t_err = py_error();
  PyGILState_Release(g);
  return e;
}

char* p2p_engine_generate(p2p_engine* e, const char* request_json) {
  if (!e || !request_json) return nullptr;
  if (e->front) {
    ReqCtx c;
    const int k = prepare(e, request_json, &c);
    if (k < 0) return nullptr;
    if (k > 0) return native_generate(e, c);
    try {  // the metrics endpoint: Python's, plus this library's counters
      Json req = Json::parse(request_json);
      if (req.is_object() && req.get_string("endpoint") == "metrics") {
        char* py = python_call(e, "handle_json", request_json, nullptr);
        if (!py) return nullptr;
        Json m = Json::parse(py);
        free(py);
        Front& f = *e->front;
        m.set("capi_requests", (long long)f.requests.load());
        m.set("capi_native_requests", (long long)f.native_requests.load());
        m.set("capi_python_tokenize", (long long)f.python_tokenize.load());
        m.set("capi_python_decode", (long long)f.python_decode.load());
        m.set("capi_gil_entries", (long long)g_gil_entries.load());
        m.set("capi_native_tokenizer", f.tok.ok ? 1 : 0);
        if (f.remote) {  // requests the C ABI routed to each replica's loop socket
          Json per = Json::array();
          long tot = 0;
          for (long r : p2p::remote_loops_routed(f.loop)) per.push(Json(r)), tot += r;
          m.set("capi_remote_routed", per);
          m.set("capi_remote_requests", (long long)tot);
        }
        return strdup(m.dump().c_str());
      }
    } catch (const std::exception&) {
    }
  }
  return python_call(e, "handle_json", request_json, nullptr);
}

char* p2p_engine_generate_stream(p2p_engine* e, const char* request_json, p2p_engine_emit_fn emit,
                                 void* ctx) {
  if (!e || !request_json || !emit) return nullptr;
  if (e->front) {
    ReqCtx c;
    const int k = prepare(e, request_json, &c);
    if (k < 0) return nullptr;
    if (k > 0) return native_stream(e, c, emit, ctx);
  }
  EmitCtx ec{emit, ctx};
  Gil g;
  char* out = nullptr;
  PyObject* cap = PyCapsule_New(&ec, "p2p_emit", nullptr);
  PyObject* fn = cap ? PyCFunction_New(&g_emit_def, cap) : nullptr;
  if (fn) {
    PyObject* r = PyObject_CallMethod(e->server, "handle_json_stream", "sO", request_json, fn);
    out = dup_utf8(r);
    Py_XDECREF(r);
  }
  if (!out) t_err = py_error();
  Py_XDECREF(fn);
  Py_XDECREF(cap);
  return out;
}

void p2p_engine_free(char* s) { free(s); }

const char* p2p_engine_error(void) { return t_err.c_str(); }

void p2p_engine_destroy(p2p_engine* e) {
  if (!e) return;
  if (e->front && e->front->remote) p2p::remote_loops_destroy(e->front->loop);
  PyGILState_STATE g = PyGILState_Ensure();
  PyObject* r = PyObject_CallMethod(e->server, "close", nullptr);
  if (!r) PyErr_Clear();
  Py_XDECREF(r);
  Py_DECREF(e->server);
  PyGILState_Release(g);
  delete e;
}

// Test hook (CPU tier): the native tokenizer of `spec_json` (SyntheticTokenizer.native_spec)
// on an Ollama request and an id list -> {"native": bool, "ids": [...], "text": "..."}.
char* p2p_engine_tok_probe(const char* spec_json, const char* request_json, const char* ids_json) {
  try {
    Front f;
    try {
      f.tok.load(spec_json);
    } catch (const std::exception&) {  // a tokenizer.json the native side does not cover
      f.tok = p2p::NativeTok();
    }
    Json out = Json::object();
    std::vector<int> ids;
    const bool ok = native_ids(f, Json::parse(request_json), &ids);
    out.set("native", ok);
    out.set("ids", Json::array_of(ids));
    std::vector<int> dec;
    const Json dj = Json::parse(ids_json);
    for (auto& v : dj.items()) dec.push_back((int)v.integer());
    out.set("text", f.tok.decode(dec));
    return strdup(out.dump().c_str());
  } catch (const std::exception& ex) {
    t_err = ex.what();
    return nullptr;
  }
}

}  // extern "C"
