set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_default.log 2>&1 || { tail -20 gpurun_out/gemm_default.log; exit 1; }
cat gpurun_out/gemm_default.log | grep -v "^{"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/gemm_bench.py --tunable > gpurun_out/gemm_tunable.log 2>&1 || { tail -20 gpurun_out/gemm_tunable.log; exit 1; }
echo TUNABLE; cat gpurun_out/gemm_tunable.log | grep -v "^{"
