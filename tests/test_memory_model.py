"""HBM memory model (train/memory.py) — CPU checks against the per-sample slopes measured on MI355X
(profiles/s3_mem: torch.cuda.max_memory_allocated of full bench.py steps at three batch sizes)."""
import pytest

from ml_recipe_distributed_pytorch_amd.models.config import get_config
from ml_recipe_distributed_pytorch_amd.train.memory import estimate, max_micro_batch, plan_batch_split

# (model, seq, measured GB per sample, measured intercept GB): slopes of max_memory_allocated over
# b = 256 -> 512 (base) and b = 128 -> 256 (large) on one MI355X
MEASURED = [("bert-base-uncased", 384, 0.1248, 2.5), ("bert-large-uncased", 512, 0.4315, 7.06)]


@pytest.mark.parametrize("model,seq,per_sample_gb,intercept_gb", MEASURED)
def test_per_sample_bytes_match_measured(model, seq, per_sample_gb, intercept_gb):
    est = estimate(get_config(model), seq)
    per = (est.act_bytes_per_sample + est.transient_bytes_per_sample) / 1e9
    assert per == pytest.approx(per_sample_gb, rel=0.05)
    assert est.params_bytes / 1e9 == pytest.approx(intercept_gb, rel=0.25)


def test_max_micro_batch_on_288gb():
    hbm = 288 * 2**30
    base = max_micro_batch(get_config("bert-base-uncased"), 384, hbm)
    large = max_micro_batch(get_config("bert-large-uncased"), 512, hbm)
    assert base > 1500 and 400 < large < 700       # test_bert.cfg's 256 fits in one micro-batch either way
    assert max_micro_batch(get_config("bert-base-uncased"), 384, 12 * 2**30) < 100   # a K80-class 12 GB card


def test_plan_batch_split():
    cfg = get_config("bert-base-uncased")
    assert plan_batch_split(cfg, 384, 256, 288 * 2**30) == 1
    split = plan_batch_split(cfg, 384, 256, 12 * 2**30)
    assert split > 1 and 256 % split == 0
    assert estimate(cfg, 384).total(256 // split) <= 0.9 * 12 * 2**30
    assert plan_batch_split(cfg, 384, 256, 288 * 2**30, requested=4, merge=False) == 4  # raise-only mode
    assert plan_batch_split(cfg, 512, 256, 288 * 2**30, requested=128) == 1  # reference cfg: 128 × 2 → 1 × 256


def test_auto_batch_split_flag_parses():
    from ml_recipe_distributed_pytorch_amd.utils.flags import get_trainer_parser
    ns, _ = get_trainer_parser().parse_known_args(["--data_path", "x", "--processed_data_path", "y",
                                                   "--experiment_name", "e", "--auto_batch_split"])
    assert ns.auto_batch_split is True
