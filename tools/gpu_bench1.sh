set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke_fail; cat gpurun_out/smoke.log | tail -20; exit 1; }
tail -2 gpurun_out/smoke.log
for b in 32 64 128; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 5 --batch $b --profile > gpurun_out/bench_prof_b$b.log 2>&1 || { echo bench_fail_$b; tail -20 gpurun_out/bench_prof_b$b.log; exit 1; }
  tail -1 gpurun_out/bench_prof_b$b.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch $b > gpurun_out/bench_b$b.log 2>&1 || { echo bench_fail_$b; tail -20 gpurun_out/bench_b$b.log; exit 1; }
  tail -1 gpurun_out/bench_b$b.log
done
