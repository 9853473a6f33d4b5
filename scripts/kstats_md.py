#!/usr/bin/env python3
"""rocprofv3 kernel_stats.csv -> markdown table (top N kernels by total time)."""
import csv
import sys


def main(path, n=20):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
        t = float(r["TotalDurationNs"])
        print("| %s | %s | %.2f | %.2f | %.1f |" % (r["Name"][:96].replace("|", "/"), r["Calls"],
                                                    t / 1e6, float(r["AverageNs"]) / 1e3,
                                                    100 * t / tot))
    print("\ntotal GPU time %.1f ms over %d kernels" % (tot / 1e6, sum(int(r["Calls"]) for r in rows)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
