#!/usr/bin/env python
"""Per-kernel shader clock from one rocprofv3 run with ``--pmc GRBM_GUI_ACTIVE ... --kernel-trace``: the
counter's active cycles over the dispatch's wall time.  GRBM_GUI_ACTIVE is summed over the XCD instances,
so the ratio is divided by ``--xcd`` (8 on MI355X).

    python tools/clock_summary.py <dir with *_counter_collection.csv and *_kernel_trace.csv> [--match gemm]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--xcd", type=int, default=8)
    a = ap.parse_args()
    cc = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)[0]
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    dur = {}
    for r in csv.DictReader(open(kt)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"])
    ctr = collections.defaultdict(dict)
    for r in csv.DictReader(open(cc)):
        ctr[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    for d, cs in ctr.items():
        if d not in dur or "GRBM_GUI_ACTIVE" not in cs:
            continue
        ns, name = dur[d]
        if a.match not in name or ns < 20000:
            continue
        key = name.replace("void (anonymous namespace)::", "").split("(")[0][:70]
        g = agg[key]
        g[0] += ns
        g[1] += cs["GRBM_GUI_ACTIVE"]
        for k, v in cs.items():
            g[2][k] += v
    print(f"{'kernel':70s} {'ms':>8s} {'GHz':>6s} {'mfma_busy':>9s}")
    for k, (ns, act, cs) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        ghz = act / a.xcd / ns
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(cs.get("SQ_BUSY_CYCLES", 0), 1)
        print(f"{k:70s} {ns / 1e6:8.2f} {ghz:6.3f} {busy:9.3f}")


if __name__ == "__main__":
    main()
