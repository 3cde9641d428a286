#!/usr/bin/env python
"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch) with derived ratios.

    python tools/pmc_summary.py gpurun_out/pmc/a/a_counter_collection.csv [more.csv ...] [--match attn]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in a.files:
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if a.match and not re.search(a.match, name):
                continue
            mm = re.search(r"(\w+_kernel(?:<[^>(]*>)?)", name)
            short = mm.group(1) if mm else re.sub(r"\(.*", "", name)[:70]
            agg[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:14.4g}")
        mf = m.get("SQ_INSTS_MFMA")
        if mf:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if c in m:
                    print(f"   {c + ' / MFMA':28s} {m[c] / mf:14.3f}")
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_INST_ANY" in m:
            print(f"   {'wait_inst / wave_cycles':28s} {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:14.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            # MFMA busy cycles summed over SIMDs vs (GPU-active cycles per XCD x 1024 SIMDs)
            util = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
            print(f"   {'mfma_busy / simd_cycles':28s} {util:14.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            print(f"   {'lds_conflict / lds_active':28s} {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:14.3f}")


if __name__ == "__main__":
    main()
