#!/usr/bin/env python3
"""rocprofv3 --pmc passes (scripts/pmc_passes.sh: one SQLite db per pass) -> per kernel
(name, grid) medians of every counter, plus derived quantities:

  hbm_MB      TCC_EA0_RDREQ x 128 B (gfx950 tallies 128-B requests; MI355X_MICROARCH.md)
  wr_MB       TCC_EA0_WRREQ x 64 B
  l2_hit      TCC_HIT / (TCC_HIT + TCC_MISS)
  wait_share  SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  mfma_busy   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
  lat_cyc     TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ (mean L1->L2 read latency, cycles)
  clk_GHz     GRBM_GUI_ACTIVE / 8 / duration

Usage: pmc_summary.py <dir with p1/ p2/ ...> [--match SUBSTR ...] [--json]"""
import argparse
import glob
import json
import os
import re
import sqlite3
import statistics
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", nargs="*", default=[])
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    # (kernel, grid) -> counter -> [values per dispatch]; and durations
    vals = defaultdict(lambda: defaultdict(list))
    for db in sorted(glob.glob(os.path.join(a.dir, "p*", "*.db"))):
        c = sqlite3.connect(db)
        rows = c.execute("select dispatch_id, kernel_name, grid_size, workgroup_size, counter_name, "
                         "value, duration from counters_collection").fetchall()
        per = defaultdict(dict)
        meta = {}
        for did, kn, grid, wg, cn, v, dur in rows:
            per[did][cn] = per[did].get(cn, 0.0) + v
            meta[did] = (short(kn), grid // max(wg, 1), wg, dur)
        for did, cs in per.items():
            kn, blocks, wg, dur = meta[did]
            if a.match and not any(m in kn for m in a.match):
                continue
            key = (kn, blocks, wg)
            for cn, v in cs.items():
                vals[key][cn].append(v)
            vals[key]["_dur_ns"].append(dur)
    out = []
    for (kn, blocks, wg), cs in sorted(vals.items()):
        med = {cn: statistics.median(v) for cn, v in cs.items()}
        d = {"kernel": kn, "blocks": blocks, "threads": wg, "n": len(cs["_dur_ns"]),
             "us": round(med["_dur_ns"] / 1e3, 2)}
        if "TCC_EA0_RDREQ_sum" in med:
            d["hbm_MB"] = round(med["TCC_EA0_RDREQ_sum"] * 128 / 1e6, 1)
        if "TCC_EA0_WRREQ_sum" in med:
            d["wr_MB"] = round(med["TCC_EA0_WRREQ_sum"] * 64 / 1e6, 1)
        if "TCC_HIT_sum" in med and "TCC_MISS_sum" in med:
            d["l2_hit"] = round(med["TCC_HIT_sum"] / max(1, med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 3)
        if "SQ_WAIT_ANY" in med and "SQ_WAVE_CYCLES" in med:
            d["wait_share"] = round(med["SQ_WAIT_ANY"] / max(1, med["SQ_WAVE_CYCLES"]), 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med:
            d["mfma_busy"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, med["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        if "TCP_TCC_READ_REQ_LATENCY_sum" in med and "TCP_TCC_READ_REQ_sum" in med:
            d["lat_cyc"] = round(med["TCP_TCC_READ_REQ_LATENCY_sum"] / max(1, med["TCP_TCC_READ_REQ_sum"]), 1)
            d["l1_l2_MB"] = round(med["TCP_TCC_READ_REQ_sum"] * 128 / 1e6, 1)
        if "GRBM_GUI_ACTIVE" in med:
            d["clk_GHz"] = round(med["GRBM_GUI_ACTIVE"] / 8 / max(1, med["_dur_ns"]), 2)
        for k in ("SQ_WAVES", "SQ_INSTS_VMEM_RD"):
            if k in med:
                d[k] = med[k]
        if "SQ_WAVE_CYCLES" in med and "SQ_WAVES" in med:
            d["wave_us"] = round(med["SQ_WAVE_CYCLES"] * 4 / max(1, med["SQ_WAVES"]) / 2.1e3, 2)
        out.append(d)
    if a.json:
        for d in out:
            print(json.dumps(d))
        return
    cols = ["kernel", "blocks", "threads", "n", "us", "hbm_MB", "wr_MB", "l1_l2_MB", "l2_hit",
            "lat_cyc", "wait_share", "mfma_busy", "wave_us", "clk_GHz"]
    print("| " + " | ".join(cols) + " |")
    print("|" + "---|" * len(cols))
    for d in out:
        print("| " + " | ".join(str(d.get(c, "")) for c in cols) + " |")


if __name__ == "__main__":
    main()
