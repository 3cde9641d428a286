set -o pipefail
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --steps 5 --warmup 3 --batch 64 > gpurun_out/prof1/bench.log 2>&1 || { echo prof_fail; tail -30 gpurun_out/prof1/bench.log; exit 1; }
ls -R gpurun_out/prof1 | head -20
find gpurun_out/prof1 -name "*kernel_stats.csv" -exec head -40 {} \;
