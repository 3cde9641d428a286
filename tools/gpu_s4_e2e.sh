#!/usr/bin/env bash
# Drop-in CLI on one MI355X: the reference's launch script + config/test_bert.cfg verbatim (debug run),
# then a real (non-debug) epoch on the dummy-QA data that writes best.ch, then validate.py on it.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s4_e2e
mkdir -p $O
R=/tmp/hq_e2e
rm -rf $R; mkdir -p $R
MASTER_PORT=29533 timeout -k 10 300 bash scripts/run_distributed_on_single_node.sh -c config/test_bert.cfg --dump_dir $R > $O/train_debug.log 2>&1 || { tail -30 $O/train_debug.log; exit 1; }
echo "debug run ok: $(ls $R/test)"
sed -e 's/^debug = True/debug = False/' -e 's/^n_epochs = 2/n_epochs = 1/' -e 's/^experiment_name = test/experiment_name = real/' config/test_bert.cfg > $R/real.cfg
echo "dummy_dataset_len = 8192" >> $R/real.cfg
MASTER_PORT=29534 timeout -k 10 600 bash scripts/run_distributed_on_single_node.sh -c $R/real.cfg --dump_dir $R > $O/train_real.log 2>&1 || { tail -30 $O/train_real.log; exit 1; }
echo "real run ok: $(ls $R/real)"
timeout -k 10 300 python modules/validate.py -c config/validate.cfg --checkpoint $R/real/best.ch --dummy_dataset --dummy_dataset_len 2048 --dump_predictions $O/pred.json > $O/validate.log 2>&1 || { tail -30 $O/validate.log; exit 1; }
tail -5 $O/validate.log
cp $R/real/*.log $R/real/*.cfg $O/ 2>/dev/null
cp $R/test/*.log $O/ 2>/dev/null
ls -la $R/real
du -sh $O
