"""End-to-end A/B of one pinned launch code: bench.py with the pinned table's entry KEY
replaced by CODE (in this process only; the table file is not touched).
Run on the GPU: python bench/code_ab.py KEY CODE [bench.py args]
e.g. python bench/code_ab.py lm_head:N128256:K4096:M1 1032 --steps 20 --warmup 5"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from p2p_llm_chat_go_amd.engine import autotune  # noqa: E402

if __name__ == "__main__":
    key, code = sys.argv[1], int(sys.argv[2])
    _load = autotune.load_table

    def load_table(model_name):
        t = dict(_load(model_name))
        if key in t:
            t[key] = code
        return t

    autotune.load_table = load_table
    import bench  # noqa: E402  (the repo-root bench.py)

    bench.main(sys.argv[3:])
