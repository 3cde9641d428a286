#!/usr/bin/env python
"""Per-kernel register / scratch / occupancy table from hipcc's kernel-resource-usage remarks.

    python tools/kres.py csrc/kernels/attention.hip [--match ring]
"""
import argparse
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    inc = os.path.join(ROOT, "ml_recipe_distributed_pytorch_amd", "csrc", "include")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + inc, "-D__HIP_PLATFORM_AMD__=1",
           "-c", a.src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split()[0]] = int(m.group(2))
        if "error" in line:
            print(line, file=sys.stderr)
    for r in rows:
        if a.match and not re.search(a.match, r["name"]):
            continue
        name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', 0):>3} agpr {r.get('ScratchSize', '?'):>4} scratch "
              f"occ {r.get('Occupancy', '?')}  {name}")


if __name__ == "__main__":
    main()
