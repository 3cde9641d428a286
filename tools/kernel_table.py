#!/usr/bin/env python
"""Condense a rocprofv3 ``*_kernel_stats.csv`` into a readable table (short kernel names, ms, %).

    python tools/kernel_table.py gpurun_out/prof/run_kernel_stats.csv [--top 25] [--steps 5]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel(?:<[^>(]*>)?)", name)
    if m:
        return m.group(1)
    if name.startswith(("Cijk_", "Custom_Cijk_")):  # hipBLASLt / Tensile
        tile = re.search(r"MT(\d+x\d+x\d+)", name)
        kind = name.split("_")[1] if not name.startswith("Custom") else name.split("_")[2]
        return f"hipblaslt[{kind} {tile.group(1) if tile else ''}]"
    return re.sub(r"\(.*", "", name)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many profiled steps")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    agg = {}
    for r in rows:
        k = short(r["Name"])
        t, c = agg.get(k, (0.0, 0))
        agg[k] = (t + float(r["TotalDurationNs"]), c + int(r["Calls"]))
    div = max(a.steps, 1)
    unit = "ms/step" if a.steps else "ms"
    print(f"{'kernel':60s} {'calls':>7s} {unit:>9s} {'avg us':>9s} {'%':>6s}")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{k[:60]:60s} {c // div:7d} {t / 1e6 / div:9.3f} {t / c / 1e3:9.1f} {100 * t / total:6.2f}")
    print(f"{'TOTAL':60s} {'':7s} {total / 1e6 / div:9.3f}")


if __name__ == "__main__":
    main()
