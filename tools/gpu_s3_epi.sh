set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s3_epi
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_gemm.log 2>&1 || { tail -30 $O/test_gemm.log; exit 1; }
tail -2 $O/test_gemm.log
timeout -k 10 300 python tools/gemm_epi_bench.py > $O/gemm_epi.txt 2>&1 && cat $O/gemm_epi.txt
