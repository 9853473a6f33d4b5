"""Chat node with the in-process suggest-reply engine.

    python -m p2p_llm_chat_go_amd.net.node

Same environment as the reference node (`go/cmd/node/main.go:131-134`):
MYNAMEIS, HTTP_ADDR, DIRECTORY_URL, BOOTSTRAP_ADDRS -- plus opt-in extras
(RELAY_ADDRS, KEY_TYPE, IDENTITY_FILE, INBOX_FILE, REGISTER_INTERVAL,
STRICT_SENDER, UI_FILE) and the engine knobs:

  ENGINE          1 (default) / 0: attach the in-process engine
  ENGINE_MODEL    preset name (default: llama3.1-8b on a GPU, tiny-llama on CPU)
  ENGINE_DEVICE   cuda:N / cpu (default: cuda:0 if available)
  ENGINE_CHECKPOINT  HF checkpoint dir (safetensors + config.json); default random-init
  ENGINE_MAX_BATCH   concurrent sequences (default 16)
  ENGINE_MAX_TOKENS  default num_predict (default 128)
  ENGINE_WARMUP   1 (default on GPUs): autotune GEMMs + capture decode graphs at start
  TOKENIZER_PATH  tokenizer.json (default: synthetic offline tokenizer)
  ENGINE_GPUS     GPUs to serve on (default 1): ENGINE_GPUS / (ENGINE_TP * ENGINE_EP)
                  data-parallel replicas, least-loaded routing (engine.cluster)
  ENGINE_TP       tensor-parallel ranks per replica (default 1; 8 for 70B over xGMI)
  ENGINE_EP       expert-parallel ranks per replica (MoE models, default 1)
  ENGINE_WEIGHTS  bf16 (default) / fp8 (weight-only e4m3 projections)
  ENGINE_NATIVE_LOOP  1 (default) / 0: single-GPU replicas run the C++ step loop
                  (engine.native_loop) instead of the Python one
  ENGINE_TIMEOUT  per-request deadline in seconds (default 60, the reference UI's bound)

The libp2p host, HTTP API and Directory client are the C++ ``Node``; this
process only adds the GPU engine behind the node's /api/generate, /api/chat
and /suggest routes (no Ollama process boundary).
"""
from __future__ import annotations

import os
import signal
import sys
import threading


def build_engine_server(model: str | None = None, device: str | None = None):
    gpus = int(os.environ.get("ENGINE_GPUS", "1"))
    tp = int(os.environ.get("ENGINE_TP", "1"))
    ep = int(os.environ.get("ENGINE_EP", "1"))
    if gpus > 1 or tp > 1 or ep > 1 or os.environ.get("ENGINE_CLUSTER", "0") == "1":
        # one process per GPU, started before this process touches any GPU
        from ..engine import cluster

        if model:
            os.environ["ENGINE_MODEL"] = model
        return cluster.from_env(device)
    import torch

    from ..engine import Engine
    from ..engine.native_loop import make_server
    from ..engine.tokenizer import get_tokenizer
    from ..models.config import get_config
    from ..models.weights import (EngineWeights, config_from_hf, load_safetensors_dir)

    dev = device or os.environ.get("ENGINE_DEVICE") or ("cuda:0" if torch.cuda.is_available()
                                                        else "cpu")
    ckpt = os.environ.get("ENGINE_CHECKPOINT", "")
    max_batch = int(os.environ.get("ENGINE_MAX_BATCH", "16"))
    if ckpt:
        cfg = config_from_hf(ckpt)
        weights = EngineWeights.from_state_dict(load_safetensors_dir(ckpt, dev), cfg, dev)
    else:
        name = model or os.environ.get("ENGINE_MODEL") or (
            "llama3.1-8b" if str(dev).startswith("cuda") else "tiny-llama")
        cfg = get_config(name)
        weights = None
    kv_pages = None if str(dev).startswith("cuda") else 256
    eng = Engine(cfg, weights=weights, device=dev, kv_pages=kv_pages, max_batch=max_batch)
    if str(dev).startswith("cuda") and os.environ.get("ENGINE_WARMUP", "1") != "0":
        # autotuned GEMM launch codes + decode graphs of the common batch buckets, before
        # the first request (ENGINE_WARMUP=0 skips: faster start, untuned first replies)
        eng.warmup(tuple(b for b in (1, 2, 4, 8, 16) if b <= max_batch), ctx=256)
    tok = get_tokenizer(cfg, os.environ.get("TOKENIZER_PATH") or (ckpt or None))
    # single-GPU replica: the continuous-batching loop runs natively (engine.native_loop);
    # CPU engines keep the Python loop
    return make_server(eng, tok, model_name=os.environ.get("LLM_MODEL", "llama3.1"),
                       default_max_tokens=int(os.environ.get("ENGINE_MAX_TOKENS", "128")))


# CLI flags mirror the environment (SURVEY §5 "Config / flag system"): a flag wins
# over the variable of the same meaning.
FLAGS = [
    ("--username", "MYNAMEIS"), ("--http-addr", "HTTP_ADDR"), ("--directory-url", "DIRECTORY_URL"),
    ("--bootstrap", "BOOTSTRAP_ADDRS"), ("--relays", "RELAY_ADDRS"), ("--listen", "LISTEN_ADDRS"),
    ("--key-type", "KEY_TYPE"), ("--identity-file", "IDENTITY_FILE"), ("--inbox-file", "INBOX_FILE"),
    ("--register-interval", "REGISTER_INTERVAL"), ("--dht-mode", "DHT_MODE"),
    ("--llm-model", "LLM_MODEL"), ("--ui-file", "UI_FILE"), ("--engine", "ENGINE"),
    ("--engine-model", "ENGINE_MODEL"), ("--engine-device", "ENGINE_DEVICE"),
    ("--engine-checkpoint", "ENGINE_CHECKPOINT"), ("--engine-max-batch", "ENGINE_MAX_BATCH"),
    ("--engine-max-tokens", "ENGINE_MAX_TOKENS"), ("--tokenizer", "TOKENIZER_PATH"),
    ("--engine-url", "ENGINE_URL"), ("--security", "SECURITY"), ("--nat-pmp", "NAT_PMP"), ("--upnp", "UPNP"),
    ("--engine-gpus", "ENGINE_GPUS"), ("--engine-tp", "ENGINE_TP"), ("--engine-ep", "ENGINE_EP"),
    ("--engine-weights", "ENGINE_WEIGHTS"),
]


def parse_flags(argv=None):
    import argparse

    ap = argparse.ArgumentParser(prog="python -m p2p_llm_chat_go_amd.net.node",
                                 description="P2P chat node with the in-process engine")
    for flag, env in FLAGS:
        ap.add_argument(flag, dest=env, default=None, help="(env %s)" % env)
    a = ap.parse_args(argv)
    for _flag, env in FLAGS:
        v = getattr(a, env)
        if v is not None:
            os.environ[env] = v
    return a


def main(argv=None):
    from ..native import load

    parse_flags(argv)
    N = load()
    cfg = {}
    ui = os.environ.get("UI_FILE") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "web",
        "index.html")
    if os.path.exists(ui):
        cfg["ui_file"] = ui
    node = N.Node(cfg)
    server = None
    if os.environ.get("ENGINE", "1") != "0":
        server = build_engine_server()
        node.set_generate_hook(server.handle_json)
        node.set_generate_stream_hook(server.handle_json_stream)
    try:
        node.start()
    except Exception as e:  # log.Fatal("directory register failed:", err)
        print("directory register failed: %s" % e, file=sys.stderr, flush=True)
        sys.exit(1)
    stop = threading.Event()

    def _sig(*_):
        stop.set()

    signal.signal(signal.SIGTERM, _sig)
    signal.signal(signal.SIGINT, _sig)
    while not stop.wait(0.5):
        pass
    node.stop()
    if server is not None:
        server.close()


if __name__ == "__main__":
    main()
