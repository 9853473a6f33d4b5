// C ABI of the in-process suggest-reply engine (SURVEY §7.1 "engine.h:
// create/submit/poll/destroy"; BASELINE north star: the node links the engine in
// process instead of calling Ollama over HTTP, `web/streamlit_app.py:91`).
//
// Any native front-end -- the C++ p2p-node daemon here (ENGINE=inproc), or a cgo
// node -- hosts the engine in its own process through these calls.  The engine
// itself is the Python/HIP stack (EngineServer: continuous batching, hipGraph
// decode, gfx950 kernels); this library embeds the interpreter that drives it and
// serialises nothing but the Ollama request/response JSON.
#pragma once

#ifdef __cplusplus
extern "C" {
#endif

typedef struct p2p_engine p2p_engine;

// model: preset ("llama3.1-8b", "tiny-llama", ...) or NULL/"" for the default of the
// device; device: "cuda:N" / "cpu" or NULL/"" (cuda:0 when available).  Other knobs
// come from the environment (ENGINE_CHECKPOINT, ENGINE_MAX_BATCH, TOKENIZER_PATH, ...).
// Returns NULL on failure (p2p_engine_error()).
p2p_engine* p2p_engine_create(const char* model, const char* device);

// Ollama /api/generate (or {"endpoint": "chat", ...} for /api/chat) request JSON ->
// response JSON.  Blocking; safe to call from many threads at once (requests batch
// in the engine loop).  The result is malloc'd: release it with p2p_engine_free.
char* p2p_engine_generate(p2p_engine* e, const char* request_json);

// Streaming variant: emit(chunk_json, ctx) per token batch (return 0 to stop, e.g. the
// client went away); returns the final `done: true` object (malloc'd).
typedef int (*p2p_engine_emit_fn)(const char* chunk_json, void* ctx);
char* p2p_engine_generate_stream(p2p_engine* e, const char* request_json, p2p_engine_emit_fn emit,
                                 void* ctx);

void p2p_engine_free(char* s);
// Last error of the calling thread ("" if none).
const char* p2p_engine_error(void);
// Stops the engine loop and releases it (the embedded interpreter stays up).
void p2p_engine_destroy(p2p_engine* e);

#ifdef __cplusplus
}
#endif
