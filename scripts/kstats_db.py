#!/usr/bin/env python3
"""rocprofv3 SQLite output (``*_results.db``) -> markdown table of the top kernels.

Usage: kstats_db.py <results.db> [N] [--tokens T]  (T: decode tokens in the run, adds
per-token time)."""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:96].replace("|", "/")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("n", nargs="?", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, total_calls, total_duration, average from top_kernels").fetchall()
    tot = sum(r[2] for r in rows)
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for name, calls, t, avg in sorted(rows, key=lambda r: -r[2])[:a.n]:
        # top_kernels reports microseconds
        print("| `%s` | %d | %.2f | %.2f | %.1f |" % (short(name), calls, t / 1e3, avg,
                                                     100 * t / tot))
    calls = sum(r[1] for r in rows)
    print("\ntotal GPU kernel time %.1f ms over %d launches" % (tot / 1e3, calls))
    if a.tokens:
        print("per decode token (all kernels / %d): %.3f ms" % (a.tokens, tot / 1e3 / a.tokens))


if __name__ == "__main__":
    main()
