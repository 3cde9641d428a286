set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/lnfuse_ab
mkdir -p $O
for r in 1 2 3 4; do for f in 0 1; do
  HQ_LN_FUSE=$f timeout -k 10 300 python bench.py --steps 30 > $O/bench_f${f}_r$r.log 2>&1 || { tail -20 $O/bench_f${f}_r$r.log; exit 1; }
  echo "fuse=$f round=$r $(tail -1 $O/bench_f${f}_r$r.log | cut -c80-175)"
done; done
