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
    a = ap.parse_args()
    os.environ["P2P_TP_FUSED_AR"] = a.fused
    from test_group_native_loop_gpu import _req, _serve

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


if __name__ == "__main__":
    main()
