"""End-to-end suggest-reply through the real chat plane (BASELINE.md "end-to-end suggest
latency"; the reference bounds it only by its 60 s LLM timeout, web/streamlit_app.py:95).

Topology of the reference's manual test (start_all.sh): Directory + node A (no engine)
+ node B whose C++ daemon hosts the engine in-process (ENGINE=inproc, llama3.1-8B
bf16 random-init on cuda:0).  Per iteration, the reference UI's flow:
  A POST /send -> B                      (libp2p stream over TCP+Noise+yamux)
  B POST /suggest {id, send: true}       (prompt template, engine, reply sent to A)
  poll A GET /inbox until the reply lands
Prints one JSON line: p50/p99 of /send, /suggest and the full round trip.
Run on the GPU: python bench/e2e_suggest_bench.py [--iters N] [--new-tokens T]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests"))
from netutil import Procs, free_port, http, wait_http  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(q * len(xs)))], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    procs = Procs()
    try:
        dport = free_port()
        procs.spawn("p2p-directory", {"ADDR": "127.0.0.1:%d" % dport, "GIN_MODE": "quiet"})
        d = "http://127.0.0.1:%d" % dport
        wait_http(d + "/health")
        urls = {}
        for name, extra in (("A", {}), ("B", {"ENGINE": "inproc", "ENGINE_MODEL": a.model,
                                             "ENGINE_DEVICE": a.device, "ENGINE_MAX_BATCH": "4"})):
            port = free_port()
            env = {"MYNAMEIS": name, "HTTP_ADDR": "127.0.0.1:%d" % port, "DIRECTORY_URL": d,
                   "LISTEN_ADDRS": "/ip4/127.0.0.1/tcp/0", "GIN_MODE": "quiet"}
            env.update(extra)
            proc = procs.spawn("p2p-node", env)
            urls[name] = "http://127.0.0.1:%d" % port
            t_start = time.time()
            while True:  # the engine node loads 16 GB of weights + autotunes: allow minutes
                if proc.poll() is not None:
                    raise SystemExit("node %s exited with %s during start-up" % (name, proc.returncode))
                try:
                    if http("GET", urls[name] + "/me")[0] == 200:
                        break
                except Exception:
                    pass
                if time.time() - t_start > 540:
                    raise SystemExit("node %s did not come up" % name)
                time.sleep(0.5)
        A, B = urls["A"], urls["B"]
        opts = {"num_predict": a.new_tokens}
        sends, suggests, totals, toks = [], [], [], []
        for it in range(a.iters + 2):  # 2 warm-up rounds
            t0 = time.perf_counter()
            st, body, _ = http("POST", A + "/send", {"to_username": "B",
                                                     "content": "Hey! How's it going? (%d)" % it})
            t1 = time.perf_counter()
            assert st == 200, body
            mid = json.loads(body)["id"]
            while not any(m["id"] == mid for m in json.loads(http("GET", B + "/inbox")[1])):
                time.sleep(0.001)
            t2 = time.perf_counter()
            st, body, _ = http("POST", B + "/suggest", {"id": mid, "send": True, "options": opts})
            t3 = time.perf_counter()
            assert st == 200, body
            sug = json.loads(body)
            while len(json.loads(http("GET", A + "/inbox")[1])) < it + 1:
                time.sleep(0.001)
            t4 = time.perf_counter()
            if it >= 2:
                sends.append((t1 - t0) * 1e3)
                suggests.append((t3 - t2) * 1e3)
                totals.append((t4 - t0) * 1e3)
                toks.append(sug.get("eval_count", a.new_tokens))
        print(json.dumps({
            "metric": "end-to-end suggest-reply latency (send -> suggest -> reply in sender inbox)",
            "model": a.model, "new_tokens": a.new_tokens, "iters": a.iters,
            "send_ms_p50": pct(sends, 0.5), "suggest_ms_p50": pct(suggests, 0.5),
            "suggest_ms_p99": pct(suggests, 0.99), "round_trip_ms_p50": pct(totals, 0.5),
            "round_trip_ms_p99": pct(totals, 0.99),
            "suggest_tokens_per_s": round(statistics.median(toks) / (pct(suggests, 0.5) / 1e3), 1),
            "stack": "C++ daemons (TCP+Noise+yamux), engine in-process via the C ABI",
            "dtype": "bf16", "data": "synthetic message, random-init weights"}), flush=True)
    finally:
        procs.close()


if __name__ == "__main__":
    main()
