#!/usr/bin/env bash
# Tune hipBLASLt algorithm choices (PyTorch TunableOp) for the bench shapes; results -> gpurun_out/tunable/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/tunable2
mkdir -p $O
export HQ_TUNABLEOP=tune HQ_TUNABLEOP_FILE=$O/tuned.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
timeout -k 10 900 python bench.py --batch 256 --steps 2 --warmup 1 > $O/tune_b256.log 2>&1 || { tail -20 $O/tune_b256.log; exit 1; }
tail -1 $O/tune_b256.log
ls -la $O
unset HQ_TUNABLEOP HQ_TUNABLEOP_FILE
timeout -k 10 400 python bench.py --batch 256 --steps 20 --warmup 5 > $O/bench_b256_before.log 2>&1 && tail -1 $O/bench_b256_before.log
