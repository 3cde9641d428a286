set -o pipefail
mkdir -p gpurun_out/tunable
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
timeout -k 10 800 python bench.py --batch 64 --steps 3 --warmup 2 > gpurun_out/tunable/tune.log 2>&1 || { tail -20 gpurun_out/tunable/tune.log; exit 1; }
tail -1 gpurun_out/tunable/tune.log
ls -la gpurun_out/tunable/
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python bench.py --batch 64 --steps 20 --warmup 5 2>&1 | tail -1
unset PYTORCH_TUNABLEOP_ENABLED
timeout -k 10 300 python bench.py --batch 64 --steps 20 --warmup 5 2>&1 | tail -1
