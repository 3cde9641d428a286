#!/usr/bin/env python
"""GPU busy/idle accounting from a rocprofv3 ``*_kernel_trace.csv``: over the window between the first and
last kernel, how much time no kernel was running (launch gaps, host syncs), and the largest gaps with the
kernels around them.

    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv [--skip 0.3] [--top 10]
(``--skip`` drops the first fraction of the window: warm-up steps.)
"""
import argparse
import csv
import re


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel(?:<[^>(]*>)?)", name)
    return m.group(1) if m else re.sub(r"\(.*", "", name)[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=float, default=0.3)
    ap.add_argument("--top", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    cut = t0 + a.skip * (t1 - t0)
    ev = [e for e in ev if e[0] >= cut]
    busy, gaps, end, prev = 0, [], ev[0][0], None
    for s, e, n in ev:
        if s > end:
            gaps.append((s - end, prev, n))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        prev = n
    span = end - ev[0][0]
    idle = sum(g for g, _, _ in gaps)
    print(f"window {span / 1e6:.2f} ms, kernels busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %), "
          f"idle {idle / 1e6:.2f} ms in {len(gaps)} gaps")
    for g, p, n in sorted(gaps, reverse=True)[: a.top]:
        print(f"  {g / 1e3:9.1f} us   after {p}   before {n}")


if __name__ == "__main__":
    main()
