"""A/B of the prefill GEMMs' precomputed row rstd (row_rstd_kernel, prefill_gemm.h pre_rstd)
against in-loop sums of squares, end to end: bench.py --peers 8 with the switch set before
the engine is built.  Run on the GPU: python bench/pre_rstd_ab.py {0|1} [bench.py args]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.ops import _lib  # noqa: E402

if __name__ == "__main__":
    _lib.lib().p2p_prefill_pre_rstd(int(sys.argv[1]))
    import bench  # noqa: E402  (the repo-root bench.py)

    bench.main(sys.argv[2:])
