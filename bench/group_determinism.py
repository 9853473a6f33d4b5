"""Run-to-run determinism of a TP group's replies (native loop and Python lockstep loop).

Serves the same four requests (greedy and one seeded sampled) twice through each loop of a
virtual-rank ClusterServer replica and prints, per request, which runs agree.  A loop that
disagrees with ITSELF has a nondeterministic step; two loops that each agree with
themselves but not with each other run different numerics.

  python bench/group_determinism.py [--world 8] [--fused 1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--fused", default="1")
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--sequence", type=int, default=0,
                    help="as the GPU test file runs it: worlds 2 and 4 (both loops) first, then "
                         "world 8 through the native loop this many times and the Python loop once")
    ap.add_argument("--repeat", type=int, default=0,
                    help="instead: ONE group per loop, the sampled request sent this many times "
                         "in a row (run-to-run determinism inside one serving process)")
    a = ap.parse_args()
    os.environ["P2P_TP_FUSED_AR"] = a.fused
    from test_group_native_loop_gpu import _req, _serve
    if a.repeat:
        return repeat_main(a)
    if a.sequence:
        return sequence_main(a)

    reqs = [_req(0), _req(1), _req(2, sampled=True, n=a.n), _req(3, n=40)]
    runs = {}
    for native in (True, False):
        for rep in range(2):
            seq, _conc, _m = _serve(a.world, native, reqs)
            runs["%s%d" % ("native" if native else "python", rep)] = [r["response"] for r in seq]
            print("done", native, rep, flush=True)
    names = list(runs)
    for i in range(len(reqs)):
        groups = {}
        for n in names:
            groups.setdefault(runs[n][i], []).append(n)
        print(json.dumps({"request": i, "distinct_replies": len(groups),
                          "groups": list(groups.values())}), flush=True)


def sequence_main(a):
    from test_group_native_loop_gpu import _req, _serve

    reqs = [_req(0), _req(1), _req(2, sampled=True), _req(3, n=40)]
    for w in (2, 4):
        for native in (True, False):
            _serve(w, native, reqs)
        print("done world", w, flush=True)
    replies = {}
    for i in range(a.sequence):
        seq, _c, _m = _serve(8, True, reqs)
        replies["native%d" % i] = seq[2]["response"]
        print("native", i, repr(seq[2]["response"][:60]), flush=True)
    seq, _c, _m = _serve(8, False, reqs)
    replies["python"] = seq[2]["response"]
    print("python", repr(seq[2]["response"][:60]), flush=True)
    groups = {}
    for k, r in replies.items():
        groups.setdefault(r, []).append(k)
    print(json.dumps({"sequence": a.sequence, "graph_steps": os.environ.get("P2P_GROUP_GRAPH_STEPS"),
                      "distinct_replies": len(groups), "groups": list(groups.values())}), flush=True)


def repeat_main(a):
    from p2p_llm_chat_go_amd.engine.cluster import ClusterServer
    from test_group_native_loop_gpu import _req

    for native in (True, False):
        os.environ.update({"ENGINE_NATIVE_LOOP": "1" if native else "0",
                           "P2P_CAR_TIMEOUT_MS": "30000", "P2P_QA_TIMEOUT_MS": "30000"})
        cs = ClusterServer("tiny-llama-gqa", gpus=a.world, tp=a.world, device="cuda", sd_seed=3,
                           max_batch=2, warmup=False, virtual_ranks=True, start_timeout=600,
                           kv_pages=256)
        try:
            replies = []
            for i in range(a.repeat):
                # a greedy request between the sampled ones, as in the test's sequence
                json.loads(cs.handle_json(_req(1)))
                replies.append(json.loads(cs.handle_json(_req(2, sampled=True, n=a.n)))["response"])
        finally:
            cs.close()
        groups = {}
        for i, r in enumerate(replies):
            groups.setdefault(r, []).append(i)
        print(json.dumps({"loop": "native" if native else "python", "world": a.world,
                          "repeats": a.repeat, "distinct_replies": len(groups),
                          "groups": list(groups.values())}), flush=True)


if __name__ == "__main__":
    main()
