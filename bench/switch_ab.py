"""End-to-end A/B of a kernel library switch (a p2p_prefill_* setter in tiled_gemm.hip:
pre_rstd, tile8, deep, phased), set before the engine is built, around bench.py.
Run on the GPU: python bench/switch_ab.py p2p_prefill_tile8 {0|1} [bench.py args]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

if __name__ == "__main__":
    name, val = sys.argv[1], int(sys.argv[2])
    if not name.startswith("p2p_prefill_"):
        raise SystemExit("not a prefill switch: %s" % name)
    getattr(_lib.lib(), name)(val)
    import bench  # noqa: E402  (the repo-root bench.py)

    bench.main(sys.argv[3:])
