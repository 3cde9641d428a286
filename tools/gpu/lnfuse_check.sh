set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lnfuse
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ln_fuse_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for f in 0 1; do
  HQ_LN_FUSE=$f timeout -k 10 300 python bench.py --steps 30 > $O/bench_f${f}_r$r.log 2>&1 || { tail -20 $O/bench_f${f}_r$r.log; exit 1; }
  echo "fuse=$f round=$r $(tail -1 $O/bench_f${f}_r$r.log | cut -c80-175)"
done; done
