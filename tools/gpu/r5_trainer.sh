#!/usr/bin/env bash
# Drop-in Trainer (modules/train.py, config/test_bert.cfg with debug off, batch 256 in one micro-batch, seq 384,
# 40 steps) vs bench.py on the same box.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r5_trainer
mkdir -p "$O"
sed -e 's/^debug = True/debug = False/' -e 's/^n_epochs = 2/n_epochs = 1/' -e 's/^max_seq_len = 512/max_seq_len = 384/' \
    -e "s#^dump_dir = .*#dump_dir = /tmp/hq_trainer_perf#" -e "s/^n_jobs = 128/n_jobs = 8/" \
    -e 's/^batch_split = 128/batch_split = 1/' config/test_bert.cfg > "$O/perf.cfg"
echo "dummy_dataset_len = 10240" >> "$O/perf.cfg"
echo "log_every = 5" >> "$O/perf.cfg"
timeout -k 10 500 python3 modules/train.py -c "$O/perf.cfg" --local_rank 0 > "$O/train.log" 2>&1 || { tail -30 "$O/train.log"; exit 1; }
grep -E "Train throughput|batch_split|Precision" "$O/train.log" | sed 's/^.* - //' | tail -5
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-200
