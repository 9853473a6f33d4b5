"""Launch-configuration autotuning of the skinny MFMA GEMMs for one model.

For every projection of the model (qkv+RoPE, o, gate_up+SiLU, down, LM head
argmax) and every M tile the engine will use, each legal (pipeline depth U,
split-K waves) pair is timed as a hipGraph that runs the projection of every
layer once (cold weights, like the real decode step) and the fastest launch
code is installed in ``ops.gemm._TUNE``.  Measured on MI355X the spread between
configurations is up to ~2x at M=1 (e.g. down_proj 18.7 vs 42.9 us), and the
best choice differs per shape, so a fixed heuristic leaves time on the table.

Determinism.  Several candidates are often within run-to-run noise of each other, and a
pick that flips between boxes moved the bench by a few percent.  So:
  * near-ties are broken by a fixed rule: every candidate within ``TIE_FRAC`` of the
    fastest counts as tied, and the tie goes to the first of them in the fixed candidate
    order (``_configs``), not to whichever was faster on this box;
  * a committed table (``tuned/<model>-<arch>.json``, written by
    ``python -m p2p_llm_chat_go_amd.engine.autotune --model ... --save``) pins the picks:
    with a table present (P2P_AUTOTUNE_TABLE, default on) the recorded code is installed
    and only timed once for the report.  P2P_AUTOTUNE_TABLE=0 re-tunes from scratch.
"""
from __future__ import annotations

import json
import os

import torch

from .. import ops
from ..ops import gemm as G


def _graph_time(fn, reps=3):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    # thread_local, as the engine's captures: in a TP group the RCCL watchdog thread polls
    # its work events meanwhile, which the default global mode turns into a capture error
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    del g
    return best


TIE_FRAC = float(os.environ.get("P2P_AUTOTUNE_TIE", "0.02"))
TABLE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")


def _arch() -> str:
    try:
        return torch.cuda.get_device_properties(0).gcnArchName.split(":")[0]
    except Exception:  # noqa: BLE001
        return "gfx950"


def table_path(model_name: str, arch: str | None = None) -> str:
    return os.path.join(TABLE_DIR, "%s-%s.json" % (model_name, arch or _arch()))


def load_table(model_name: str) -> dict:
    if os.environ.get("P2P_AUTOTUNE_TABLE", "1") == "0":
        return {}
    p = table_path(model_name)
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        return json.load(f).get("codes", {})


def pick(times: dict, order: list) -> int:
    """Fastest candidate, near-ties (within TIE_FRAC) resolved by candidate order."""
    t_min = min(times.values())
    for code in order:
        if code in times and times[code] <= t_min * (1.0 + TIE_FRAC):
            return code
    return min(times, key=times.get)


def _job_key(name, N, K, M, fp8) -> str:
    return "%s:N%d:K%d:M%d%s" % (name, N, K, M, ":fp8" if fp8 else "")


def _configs(K, M=1, tiled=False, midm=False, wide=False):
    """Launch codes: waves | U << 8 | NG << 16 (NG = column groups per block, M > 16);
    G.TILED_FLAG = the split-K LDS-DMA tiled kernel (M > 16, tileable shapes);
    G.MIDM_FLAG = the whole-K LDS-DMA kernel (M > 1, bf16 weights, K % 128 == 0);
    G.WIDE_FLAG = the wide kernel (M > 1, bf16 weights, wide_ok shapes), heuristic K split
    and the two neighbouring powers of two."""
    out = [G.TILED_FLAG] if (tiled and M > 16) else []
    if midm and M > 1 and K % 128 == 0:
        out.append(G.MIDM_FLAG)
    if wide and M > 1:
        for nw in (0, G.WIDE16):
            out += [G.WIDE_FLAG | nw, G.WIDE_FLAG | nw | (4 << 8), G.WIDE_FLAG | nw | (8 << 8)]
    # NG=2 at M <= 16 (twice the weight bytes in flight per wave) is supported by the kernel
    # but was never faster at the 8B decode shapes (two bench runs, w1-w8): not tuned
    for ng in ((1,) if M <= 16 else (1, 2)):
        for u in ((4, 8) if M <= 16 else (2, 4)):
            for w in (1, 2, 4, 8):
                if (K // 32) // w >= 8 and not (ng > 1 and w == 8):
                    out.append(w | (u << 8) | ((ng if ng > 1 else 0) << 16))
    if M <= 16 and (K // 32) // 16 >= 8:
        # 16 waves per block (bf16, not SwiGLU: the kernel falls back to 8 there), 4-deep
        # batches: the stream probe's 16 waves per CU at the 256-column-group projections
        out.append(16 | (4 << 8))
    return out


def describe(code: int) -> str:
    if code & G.PERSIST_FLAG:
        return "persist/x%d" % max(1, (code >> 8) & 0xff)
    if code & G.TILED_FLAG:
        return "tiled"
    if code & G.MIDM_FLAG:
        return "midm"
    if code & G.AFRAG_FLAG:
        return "packed+" + describe(code & ~G.AFRAG_FLAG)
    if code & G.WIDE_FLAG:
        sk = (code >> 8) & 0xff
        return "wide%s/s%s" % ("16" if code & G.WIDE16 else "", sk if sk else "auto")
    ng = (code >> 16) & 0xff
    return "w%d/U%d%s" % (code & 0xff, (code >> 8) & 0xff, "/NG%d" % ng if ng > 1 else "")


def autotune_model(model, batch_sizes=(1,), verbose=False, table: dict | None = None,
                   record: dict | None = None) -> dict:
    """Tune (or, for keys in ``table``, install the recorded pick of) every projection at
    every M of ``batch_sizes``.  ``record`` (if given) receives {job key: code} of every
    pick, for ``--save``."""
    if model.device.type != "cuda":
        return {}
    if table is None:
        tp = getattr(model, "tp", 1)
        table = load_table(model.cfg.name if tp == 1 else "%s-tp%d" % (model.cfg.name, tp))
    cfg, w = model.cfg, model.w
    dev = model.device
    H = cfg.hidden
    nq, nkv = model.nq, model.nkv
    kc, vc = model.kv.layer(0)
    result = {}
    layers = w.layers
    for M in sorted(set(min(b, G.SKINNY_MAX_M) for b in batch_sizes)):
        x = torch.randn(M, H, device=dev).to(torch.bfloat16)
        h = torch.zeros(M, H, device=dev, dtype=torch.bfloat16)
        q = torch.zeros(M, nq * 128, device=dev, dtype=torch.bfloat16)
        pos = torch.zeros(M, device=dev, dtype=torch.int32)
        slots = torch.arange(M, device=dev, dtype=torch.int32) % 64  # null page 0
        keys = ops.new_argmax_keys(M, dev)
        jobs = [("qkv_rope", [lw.qkv for lw in layers], G.EPI_QKV_ROPE,
                 lambda wt, c: ops.qkv_rope_gemm(wt, x, pos, slots, model.rope, nq, nkv, q, kc, vc,
                                                 waves=c)),
                ("o_proj", [lw.o for lw in layers], G.EPI_RESID,
                 lambda wt, c: ops.skinny_gemm(wt, q, ops.EPI_RESID, out=h, waves=c))]
        if not cfg.is_moe:
            F = layers[0].gate_up.shape[0] * 16 // 2
            act = torch.zeros(M, F, device=dev, dtype=torch.bfloat16)
            xf = torch.randn(M, F, device=dev).to(torch.bfloat16)
            jobs += [("gate_up", [lw.gate_up for lw in layers], G.EPI_SILU,
                      lambda wt, c: ops.skinny_gemm(wt, x, ops.EPI_SILU, norm=True, out=act,
                                                    waves=c)),
                     ("down", [lw.down for lw in layers], G.EPI_RESID,
                      lambda wt, c: ops.skinny_gemm(wt, xf, ops.EPI_RESID, out=h, waves=c))]
        jobs.append(("lm_head", [w.lm_head], G.EPI_ARGMAX,
                     lambda wt, c: ops.lm_head_argmax(wt, x, keys, waves=c)))
        for name, wts, epi, fn in jobs:
            N, K = G.tiled_shape(wts[0])
            times = {}
            bf = not G._is_f8(wts[0])
            codes = _configs(K, M, G.tiled_ok(N, K, epi) and bf, midm=bf,
                             wide=bf and G.wide_ok(N, K, epi))
            if bf and epi == G.EPI_ARGMAX and M == 1 and G.wide_ok(N, K, epi):
                # the 1 GB LM head stream: the wide kernel's 8 x 3 chunks of weights in flight
                # per workgroup against the skinny launches
                codes += [G.WIDE_FLAG]
            # (the persistent GEMV, G.PERSIST_FLAG, is not a candidate: 1.3-1.6x slower than
            # the skinny launches on every 8B decode shape, profiles/r4_persist_gemv_negative.jsonl)
            if bf and epi == G.EPI_QKV_ROPE and M > 16:
                # pack the activations fragment-major first (one extra launch, timed with the
                # GEMM): measured to pay on the qkv shape only (profiles/r3_afrag_probe.jsonl)
                codes += [c | G.AFRAG_FLAG for c in _configs(K, M) if (c >> 16) & 0xff]
            jk = _job_key(name, N, K, M, not bf)
            fixed = table.get(jk)
            if fixed is not None and int(fixed) in codes:
                times[int(fixed)] = _graph_time(lambda: [fn(wt, int(fixed)) for wt in wts])
                best = int(fixed)
            else:
                for code in codes:
                    times[code] = _graph_time(lambda: [fn(wt, code) for wt in wts])
                best = pick(times, codes)
            if record is not None:
                record[jk] = best
            norm = epi in (G.EPI_QKV_ROPE, G.EPI_SILU, G.EPI_ARGMAX)
            G.set_tune(G.tune_key(wts[0], M, epi, norm), best)
            if epi == G.EPI_RESID:
                # TP row-parallel projections run the same shape with other epilogues
                # (partial store / fused all-reduce); the weight stream is the same
                for e2 in (G.EPI_STORE, G.EPI_AR):
                    G.set_tune(G.tune_key(wts[0], M, e2, False), best)
            result[(name, M)] = (describe(best), times[best] * 1000 / len(wts))
            if verbose:
                print("autotune %-9s M=%-2d %s  %.2f us" % (
                    name, M, describe(best), times[best] * 1000 / len(wts)), flush=True)
        keys.zero_()
    torch.cuda.synchronize()
    return result


def main(argv=None):
    """Tune a model on this GPU and (``--save``) write the pinned table."""
    import argparse

    from ..models.config import get_config
    from .engine import Engine

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--tp", type=int, default=1, help="tune one rank's shard of a TP group")
    ap.add_argument("--batch", default="1,2,4,8,16,48,64")
    ap.add_argument("--save", action="store_true")
    a = ap.parse_args(argv)
    os.environ["P2P_AUTOTUNE_TABLE"] = "0"
    cfg = get_config(a.model)
    kw = dict(tp_rank=0, tp_size=a.tp) if a.tp > 1 else {}
    eng = Engine(cfg, device="cuda", kv_pages=64, max_batch=16, use_graph=False, **kw)
    rec = {}
    res = autotune_model(eng.model, tuple(int(b) for b in a.batch.split(",")), verbose=True,
                         table={}, record=rec)
    out = {"model": cfg.name, "arch": _arch(), "tp": a.tp, "tie_frac": TIE_FRAC, "codes": rec,
           "us": {"%s@M%d" % k: round(v[1], 2) for k, v in res.items()}}
    print(json.dumps(out), flush=True)
    if a.save:
        name = cfg.name if a.tp == 1 else "%s-tp%d" % (cfg.name, a.tp)
        os.makedirs(TABLE_DIR, exist_ok=True)
        with open(table_path(name), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
