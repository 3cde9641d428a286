#!/bin/bash
# fp8 backward (e5m2 dgrads + fp8 weight gradients): tr_b8 lane-map probe, kernel tests, then same-box
# bf16 vs fp8 (full fp8 backward) vs fp8 with bf16 dgrads step throughput, then kernel tables of both.
# Any failing GPU step ends the script (no further GPU work after a fault or timeout).
set -o pipefail
mkdir -p gpurun_out/fp8b
hipcc -O2 --offload-arch=gfx950 tools/fp8_lab/tr8_probe.hip -o gpurun_out/fp8b/tr8 || exit 1
timeout -k 5 30 gpurun_out/fp8b/tr8 > gpurun_out/fp8b/tr8_probe.txt 2>&1
rc=$?
echo "tr8 probe rc=$rc"; tail -2 gpurun_out/fp8b/tr8_probe.txt
[ $rc -le 2 ] || exit 1   # 2 = hypothesis mismatch (printed), anything else = the probe itself failed
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py \
  > gpurun_out/fp8b/tests.log 2>&1 || { tail -40 gpurun_out/fp8b/tests.log; exit 1; }
tail -3 gpurun_out/fp8b/tests.log
timeout -k 10 240 python -u bench.py --steps 6 --warmup 3 > gpurun_out/fp8b/bf16.json 2> gpurun_out/fp8b/bf16.err || exit 1
timeout -k 10 240 python -u bench.py --steps 6 --warmup 3 --precision fp8 > gpurun_out/fp8b/fp8.json 2> gpurun_out/fp8b/fp8.err || exit 1
timeout -k 10 240 python -u bench.py --steps 6 --warmup 3 --precision fp8 --fp8_dgrad 0 > gpurun_out/fp8b/fp8_nodg.json \
  2> gpurun_out/fp8b/fp8_nodg.err || exit 1
cat gpurun_out/fp8b/bf16.json gpurun_out/fp8b/fp8.json gpurun_out/fp8b/fp8_nodg.json
export TMPDIR=/tmp
for prec in fp8 bf16; do
  timeout -k 10 300 scripts/profile_kernels.sh gpurun_out/fp8b/prof_$prec -- python bench.py --steps 3 --warmup 2 \
    --precision $prec > gpurun_out/fp8b/prof_$prec.log 2>&1 || exit 1
  python tools/kernel_table.py "$(find gpurun_out/fp8b/prof_$prec -name 'run_kernel_stats.csv' | head -n 1)" --top 40 \
    --steps 5 > gpurun_out/fp8b/kernel_table_$prec.txt
done
head -32 gpurun_out/fp8b/kernel_table_fp8.txt
