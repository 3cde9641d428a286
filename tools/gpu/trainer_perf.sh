#!/usr/bin/env bash
# Steady-state throughput of the Trainer / DataLoader path (modules/train.py with config/test_bert.cfg:
# BERT-base, dummy data, loss=smooth, AdamW, clip 1) at the bench.py shape (batch 256, seq 384), to be
# compared with bench.py's samples/s.  The cfg is the repo's test_bert.cfg with debug off, one epoch of
# 40 optimizer steps, max_seq_len 384 and 8 DataLoader workers (the box has a 16-CPU share).  Usage: tools/gpu/trainer_perf.sh <outdir>
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-trainer_perf}
mkdir -p "$O"
sed -e 's/^debug = True/debug = False/' -e 's/^n_epochs = 2/n_epochs = 1/' -e 's/^max_seq_len = 512/max_seq_len = 384/' \
    -e "s#^dump_dir = .*#dump_dir = /tmp/hq_trainer_perf#" -e "s/^n_jobs = 128/n_jobs = 8/" config/test_bert.cfg > "$O/perf.cfg"
echo "dummy_dataset_len = 10240" >> "$O/perf.cfg"
echo "log_every = 5" >> "$O/perf.cfg"
timeout -k 10 500 python3 modules/train.py -c "$O/perf.cfg" > "$O/train.log" 2>&1 || { tail -30 "$O/train.log"; exit 1; }
grep -E "Train throughput|batch_split|Precision" "$O/train.log" | sed 's/^.* - //'
