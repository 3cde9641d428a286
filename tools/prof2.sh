set -o pipefail
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=ml_recipe_distributed_pytorch_amd/tuning/tunableop_mi355x.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python bench.py --steps 5 --warmup 3 --batch 64 > gpurun_out/prof2/bench.log 2>&1 || { echo prof_fail; tail -30 gpurun_out/prof2/bench.log; exit 1; }
tail -1 gpurun_out/prof2/bench.log
