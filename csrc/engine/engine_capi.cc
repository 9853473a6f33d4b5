// Engine C ABI over an embedded CPython interpreter -- see engine_capi.h.
#include "engine_capi.h"

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>

struct p2p_engine {
  PyObject* server = nullptr;  // engine.server.EngineServer
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
    }
    Py_DECREF(mod);
  }
  if (!e) t_err = py_error();
  PyGILState_Release(g);
  return e;
}

char* p2p_engine_generate(p2p_engine* e, const char* request_json) {
  if (!e || !request_json) return nullptr;
  PyGILState_STATE g = PyGILState_Ensure();
  PyObject* r = PyObject_CallMethod(e->server, "handle_json", "s", request_json);
  char* out = dup_utf8(r);
  if (!out) t_err = py_error();
  Py_XDECREF(r);
  PyGILState_Release(g);
  return out;
}

char* p2p_engine_generate_stream(p2p_engine* e, const char* request_json, p2p_engine_emit_fn emit,
                                 void* ctx) {
  if (!e || !request_json || !emit) return nullptr;
  EmitCtx ec{emit, ctx};
  PyGILState_STATE g = PyGILState_Ensure();
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
  PyGILState_Release(g);
  return out;
}

void p2p_engine_free(char* s) { free(s); }

const char* p2p_engine_error(void) { return t_err.c_str(); }

void p2p_engine_destroy(p2p_engine* e) {
  if (!e) return;
  PyGILState_STATE g = PyGILState_Ensure();
  PyObject* r = PyObject_CallMethod(e->server, "close", nullptr);
  if (!r) PyErr_Clear();
  Py_XDECREF(r);
  Py_DECREF(e->server);
  PyGILState_Release(g);
  delete e;
}

}  // extern "C"
