#!/usr/bin/env python
"""Per-kernel table of the LAST K training steps of a rocprofv3 kernel trace (``*_kernel_trace.csv``).

A step ends at its optimizer kernel (``adamw_kernel``), so warm-up and calibration steps (fp8 delayed scaling
switches kernels during its first steps) are left out, unlike ``tools/kernel_table.py`` which averages the
whole run.  Also prints the GPU-busy time and the span of those steps.

    python tools/trace_steps.py gpurun_out/x/prof/run_kernel_trace.csv --last 5 [--top 40]
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_table import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="adamw_kernel")
    ap.add_argument("--gaps", type=int, default=0,
                    help="also list the N largest idle gaps (previous kernel's end -> next kernel's start) of those "
                         "steps, grouped by the kernel pair around them")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(ends) < a.last + 1:
        raise SystemExit(f"only {len(ends)} steps in the trace")
    lo, hi = ends[-a.last - 1] + 1, ends[-1] + 1
    sel = rows[lo:hi]
    agg = {}
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        t, c = agg.get(k, (0.0, 0))
        agg[k] = (t + d, c + 1)
        busy += d
    span = (int(sel[-1]["End_Timestamp"]) - int(rows[lo - 1]["End_Timestamp"])) / 1e3
    n = a.last
    print(f"{'kernel':60s} {'calls':>7s} {'ms/step':>9s} {'avg us':>9s} {'%':>6s}")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{k[:60]:60s} {c // n:7d} {t / 1e3 / n:9.3f} {t / c:9.1f} {100 * t / busy:6.2f}")
    print(f"{'TOTAL (kernel time)':60s} {'':7s} {busy / 1e3 / n:9.3f}")
    print(f"{'SPAN (wall, first to last step end)':60s} {'':7s} {span / 1e3 / n:9.3f}")
    if a.gaps:
        # idle time between consecutive kernels (one stream's view: overlapping kernels give no gap)
        gaps, end = {}, int(rows[lo - 1]["End_Timestamp"])
        prev = short(rows[lo - 1]["Kernel_Name"])
        for r in sel:
            st, k = int(r["Start_Timestamp"]), short(r["Kernel_Name"])
            g = (st - end) / 1e3
            if g > 0:
                t, c = gaps.get((prev, k), (0.0, 0))
                gaps[(prev, k)] = (t + g, c + 1)
            if int(r["End_Timestamp"]) > end:
                end, prev = int(r["End_Timestamp"]), k
        tot = sum(t for t, _ in gaps.values())
        print(f"\nidle gaps: {tot / 1e3 / n:.3f} ms/step; largest (us/step, count/step): previous -> next kernel")
        for (pk, nk), (t, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[: a.gaps]:
            print(f"{t / n:9.1f} {c / n:6.1f}  {pk[:45]} -> {nk[:45]}")


if __name__ == "__main__":
    main()
