"""bench.py's multi-rank contract on the CPU (gloo): ``--gpus N`` without torchrun
spawns N rank processes itself, every rank joins one process group of N, and
rank 0 prints one JSON line with ``n_gpus == rccl_world == N``."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--steps", "1", "--warmup", "1", "--new-tokens", "4"] + list(args),
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout,
                       env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n,extra,par", [
    (1, ["--model", "tiny-llama"], "dp1"),
    (2, ["--model", "tiny-llama"], "dp2"),
    (8, ["--model", "tiny-llama", "--peers", "2"], "dp8"),
    (8, ["--model", "tiny-llama-gqa", "--tp", "8"], "dp1-tp8"),
    (4, ["--model", "tiny-llama-gqa", "--tp", "2"], "dp2-tp2"),
    (8, ["--model", "tiny-mixtral-8e", "--ep", "8"], "dp1-ep8"),
])
def test_bench_spawns_ranks(n, extra, par):
    out = _bench("--gpus", str(n), *extra)
    assert out["n_gpus"] == n
    assert out["rccl_world"] == n
    assert out["config"]["parallelism"] == par
    assert out["value"] > 0 and out["steps"] == 1 and out["warmup"] == 1
    assert out["config"]["prompt_tokens"] >= 40  # median-length message, not the shortest
    for k in ("metric", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
              "dtype", "data", "ttft_p50_ms", "decode_graph_captured"):
        assert k in out


def test_bench_rejects_world_mismatch():
    e = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--gpus", "2", "--model", "tiny-llama", "--steps", "1"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120,
                       env=e, cwd=ROOT)
    assert r.returncode != 0 and "--gpus 2" in r.stderr
