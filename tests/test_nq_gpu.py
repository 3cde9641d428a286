"""The real-data (Natural Questions) training path on the GPU — reference ``modules/init.py:148-201`` (dataset
factory), ``modules/model/dataset/split_dataset.py:202-520`` (SplitDataset + collate_fun, which pads every batch
to ITS max length) and ``modules/validate.py:15-54`` (ChunkDataset + Predictor).

On the dummy path every batch has L = max_seq_len; here each batch has its own L, most of them not multiples of
128, so the CLI trainer exercises the M-tail GEMM tiles, the attention length tails, merge planning with
unequal segments and the graph-shape cap (``TrainEngine.max_graph_shapes``: shapes beyond the cap run eagerly
beside the captured graphs).  Data: ``data/synth_nq.py`` documents over the toy WordPiece vocab (no NQ download
in this environment), BERT-base architecture with random-init weights."""
import math
import os
import re
import subprocess
import sys

import pytest
import torch

from conftest import FIXTURES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NQ_CFG = os.path.join(ROOT, "config", "nq_bert.cfg")

pytestmark = pytest.mark.gpu


def _run(cmd, cwd, timeout=500):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=cwd, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r


def _nq_data(tmp_path, n=160):
    from ml_recipe_distributed_pytorch_amd.data.synth_nq import write_jsonl
    vocab = os.path.join(FIXTURES, "toy_vocab.txt")
    data = str(tmp_path / "nq.jsonl")
    write_jsonl(data, n, seed=11, vocab_file=vocab, n_par=(1, 6), par_len=(6, 40))
    return data, vocab


@pytest.mark.parametrize("graph", [False, True])
def test_nq_train_then_validate_gpu(cuda, tmp_path, graph):
    """``modules/train.py -c config/nq_bert.cfg`` on a synthetic NQ jsonl: variable batch lengths (collate pads to
    each batch's max, L not a multiple of 128), batch_split 2 (merged exact-objective passes), one epoch with
    eval + checkpoints — eagerly and with HIP graphs (more distinct shapes than the graph cap) — then
    ``modules/validate.py`` on the real chunk path (every window of every test document)."""
    data, vocab = _nq_data(tmp_path)
    proc = str(tmp_path / "proc")
    args = ["-c", NQ_CFG, "--local_rank", "0", "--random_init", "--data_path", data, "--processed_data_path", proc,
            "--vocab_file", vocab, "--dump_dir", str(tmp_path), "--experiment_name", "nq", "--n_epochs", "1",
            "--train_batch_size", "16", "--batch_split", "2", "--test_batch_size", "16", "--max_seq_len", "200",
            "--doc_stride", "48", "--n_jobs", "0", "--seed", "3"]
    if graph:
        args += ["--cuda_graph", "True"]
    _run([sys.executable, os.path.join(ROOT, "modules", "train.py")] + args, cwd=str(tmp_path))
    exp = tmp_path / "nq"
    log = open(next(exp.glob("*.log"))).read()
    assert "Used device: cuda" in log, log[-2000:]
    for f in ("last.ch", "epoch_1.ch", "best.ch"):
        assert (exp / f).exists(), (f, log[-3000:])
    st = torch.load(exp / "last.ch", weights_only=True, map_location="cpu")
    assert st["global_step"] >= 3, st["global_step"]
    assert all(torch.isfinite(v).all() for v in st["model"].values() if v.is_floating_point())
    from ml_recipe_distributed_pytorch_amd.utils.tb import read_events
    ev = list((tmp_path / "board" / "nq").glob("events.out.tfevents.*"))
    vals = {}
    for _, t, v in read_events(str(ev[0])):
        vals.setdefault(t, []).append(v)
    # (one eval batch holds the whole 5 % test split: a batch whose items all lack an answer span would make the
    # reference's CrossEntropyLoss(ignore_index=-1) a 0/0 = NaN — the CPU oracle does the same)
    assert all(math.isfinite(v) for v in vals["train/loss"]) and math.isfinite(vals["test/loss"][-1])
    assert 0 <= vals["test/map"][-1] <= 1
    # validate.py: the real ChunkDataset (split by sentence, truncate) + Predictor on the written checkpoint
    vcfg = os.path.join(ROOT, "config", "validate.cfg")
    pred = tmp_path / "pred.json"
    v = _run([sys.executable, os.path.join(ROOT, "modules", "validate.py"), "-c", vcfg, "--checkpoint",
              str(exp / "last.ch"), "--data_path", data, "--processed_data_path", proc, "--vocab_file", vocab,
              "--gpu", "--max_seq_len", "200", "--doc_stride", "48", "--dump_predictions", str(pred), "--n_jobs", "0",
              "--limit", "None", "--batch_size", "8"], cwd=str(tmp_path))
    out = v.stdout + v.stderr
    m = re.search(r"Validation metrics: (.*)", out)
    assert m, out[-3000:]
    nums = [float(x) for x in re.findall(r": (-?[0-9.]+(?:e-?[0-9]+)?)", m.group(1))]
    assert nums and all(math.isfinite(x) for x in nums), m.group(1)
    assert pred.exists()


def _nq_micro_batches(n_steps, split, seq=200):
    """Real collated NQ micro-batches (SplitDataset + collate_fun): every batch padded to its own max length."""
    import tempfile
    from ml_recipe_distributed_pytorch_amd.data.collate import collate_fun
    from ml_recipe_distributed_pytorch_amd.data.nq import RawPreprocessor, SplitDataset
    from ml_recipe_distributed_pytorch_amd.data.tokenizer import Tokenizer
    tmp = tempfile.mkdtemp()
    from pathlib import Path
    data, vocab = _nq_data(Path(tmp), n=96)
    tok = Tokenizer("bert", vocab_file=vocab, lowercase=True)
    pre = RawPreprocessor(raw_json=data, out_dir=os.path.join(tmp, "proc"))
    _, _, (train_idx, _, _, _) = pre()
    ds = SplitDataset(os.path.join(tmp, "proc"), tok, train_idx, max_seq_len=seq, max_question_len=32, doc_stride=48)
    b = 4
    items = [ds[i] for i in range(n_steps * split * b)]
    batches = [collate_fun(items[i * b:(i + 1) * b], tok) for i in range(n_steps * split)]
    return [batches[s * split:(s + 1) * split] for s in range(n_steps)]


def test_graph_and_eager_agree_beyond_the_shape_cap(cuda):
    """TrainEngine with HIP graphs (cap: 2 captured shapes) vs eager, over real NQ micro-batches of more distinct
    lengths than the cap: uncaptured shapes run eagerly beside the graphs, and the loss trajectory and final weights
    match the all-eager run (same dropout seeds: both draw one host seed per micro-step)."""
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    steps = _nq_micro_batches(n_steps=7, split=2)
    shapes = {mb[0]["input_ids"].shape[1] for st in steps for mb in st}
    assert len(shapes) > 2, shapes                         # more lengths than the graph cap
    assert any(L % 128 for L in shapes), shapes
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)

    def run(graph):
        torch.manual_seed(0)
        m = BertForQuestionAnswering(get_config("bert-base-uncased"), seed=5).to(cuda).train()
        opt = FusedAdamW(optimizer_groups(m.named_parameters(), 1e-4), m.store, lr=1e-4, eps=1e-6,
                         correct_bias=False, zero_grad_fn=m.zero_grad)
        eng = TrainEngine(m, build_loss(lp), opt, max_grad_norm=1.0, batch_split=2, graph=graph, max_graph_shapes=2)
        losses = []
        for st in steps:
            res = eng.step([tuple(to_device(x, cuda) for x in mb) for mb in st])
            losses.append(res.losses.to_floats()["loss"])
        torch.cuda.synchronize()
        return losses, m.store.master.clone(), eng

    le, we, _ = run(False)
    lg, wg, eng = run(True)
    assert eng.graph_replays > 0 and eng.graph_eager_steps > 0, (eng.graph_replays, eng.graph_eager_steps)
    assert all(math.isfinite(x) for x in le)
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), (le, lg)
    assert torch.equal(we, wg) or float((we - wg).abs().max()) <= 1e-6, float((we - wg).abs().max())
