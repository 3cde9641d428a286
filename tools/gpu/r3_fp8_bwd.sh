#!/bin/bash
# fp8 backward: kernel tests, then same-box bf16 vs fp8 (fp8 dgrad on) step throughput
set -o pipefail
mkdir -p gpurun_out/fp8b
hipcc -O2 --offload-arch=gfx950 tools/fp8_lab/tr8_probe.hip -o gpurun_out/fp8b/tr8 && \
  timeout -k 5 30 gpurun_out/fp8b/tr8 > gpurun_out/fp8b/tr8_probe.txt 2>&1; echo "tr8 probe rc=$?"; tail -2 gpurun_out/fp8b/tr8_probe.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py \
  > gpurun_out/fp8b/tests.log 2>&1 || { tail -40 gpurun_out/fp8b/tests.log; exit 1; }
tail -3 gpurun_out/fp8b/tests.log
timeout -k 10 240 python -u bench.py --steps 6 --warmup 3 > gpurun_out/fp8b/bf16.json 2> gpurun_out/fp8b/bf16.err && \
timeout -k 10 240 python -u bench.py --steps 6 --warmup 3 --precision fp8 > gpurun_out/fp8b/fp8.json 2> gpurun_out/fp8b/fp8.err && \
cat gpurun_out/fp8b/bf16.json gpurun_out/fp8b/fp8.json &&
timeout -k 10 240 python -u bench.py --steps 6 --warmup 3 --precision fp8 --fp8_dgrad 0 > gpurun_out/fp8b/fp8_nodg.json 2> gpurun_out/fp8b/fp8_nodg.err && \
cat gpurun_out/fp8b/fp8_nodg.json
