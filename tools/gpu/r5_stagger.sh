#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5_stagger
mkdir -p "$O"
timeout -k 10 400 python tools/gemm_stagger2.py > "$O/stagger.log" 2>&1 || { tail -20 "$O/stagger.log"; exit 1; }
python -c "
import json
for l in open('$O/stagger.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['N'],d['K'],d['epi'],d['sched'],d['stagger'],d['groups'],d['us'])
"
