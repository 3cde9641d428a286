set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sched1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_sched_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_gemm.log 2>&1 || { tail -30 $O/pytest_gemm.log; exit 1; }
tail -2 $O/pytest_gemm.log
timeout -k 10 300 python -u tools/gemm_contention_bench.py --rounds 9 > $O/contention.log 2>&1 || { tail -30 $O/contention.log; exit 1; }
cat $O/contention.log
for s in 0 1; do HQ_GEMM_SCHED=$s timeout -k 10 300 python bench.py > $O/bench_sched$s.log 2>&1 || { tail -20 $O/bench_sched$s.log; exit 1; }; tail -1 $O/bench_sched$s.log | cut -c1-200; done
