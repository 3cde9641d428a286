"""Config surface: configargparse-compatible parsing, two-parser split, round trip."""
import os

import pytest

from ml_recipe_distributed_pytorch_amd.utils import flags
from ml_recipe_distributed_pytorch_amd.utils.cfgparse import ArgumentParser

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "config", "test_bert.cfg")
REF_CFG = os.path.join(ROOT, "tests", "fixtures", "reference_test_bert.cfg")  # verbatim reference file


def _write(tmp_path, text, name="a.cfg"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_config_file_basic(tmp_path):
    p = ArgumentParser()
    p.add_argument("-c", "--config_file", is_config_file=True)
    p.add_argument("--lr", type=float, default=1.0)
    p.add_argument("--name", type=str, default="x")
    p.add_argument("--flag", action="store_true")
    p.add_argument("--off", action="store_true")
    p.add_argument("--none", type=flags.cast2(int), default=3)
    path = _write(tmp_path, "# comment\nlr = 0.5\nname=abc  # trailing\nflag=True\noff = False\nnone=None\n")
    a = p.parse_args(["-c", path])
    assert a.lr == 0.5 and a.name == "abc" and a.flag is True and a.off is False and a.none is None


def test_cli_overrides_config(tmp_path):
    p = ArgumentParser()
    p.add_argument("-c", "--config_file", is_config_file=True)
    p.add_argument("--lr", type=float, default=1.0)
    path = _write(tmp_path, "lr = 0.5\n")
    assert p.parse_args(["-c", path, "--lr", "2"]).lr == 2.0
    assert p.parse_args(["--lr", "3", "-c", path]).lr == 3.0
    assert p.parse_args(["-c", path]).lr == 0.5


def test_unknown_keys_surface(tmp_path):
    p = ArgumentParser()
    p.add_argument("-c", "--config_file", is_config_file=True)
    p.add_argument("--lr", type=float, default=1.0)
    path = _write(tmp_path, "lr = 0.5\nmystery = 7\n")
    a, unknown = p.parse_known_args(["-c", path])
    assert a.lr == 0.5 and "--mystery=7" in unknown


@pytest.mark.parametrize("cfg", [REF_CFG, CFG], ids=["reference_verbatim", "shipped"])
def test_reference_config_two_parsers(cfg):
    (tp, mp), (params, model_params) = flags.get_params((flags.get_trainer_parser, flags.get_model_parser),
                                                        ["-c", cfg])
    assert model_params.model == "bert-base-uncased" and model_params.lowercase is True
    assert model_params.merges_file is None
    assert params.dummy_dataset and params.debug and params.apex_level == "O1"
    assert params.train_batch_size == 256 and params.loss == "smooth" and params.smooth_alpha == 0.01
    assert params.best_order == ">" and params.last is None and params.seed is None
    assert str(params.dump_dir) == "results"
    assert params.batch_split == 128 and params.n_jobs == 128  # reference micro-batch of 2


def test_shipped_config_equals_reference():
    """config/test_bert.cfg (reformatted, commented) parses to exactly the reference file's values."""
    getters = (flags.get_trainer_parser, flags.get_model_parser)
    _, (p_ref, m_ref) = flags.get_params(getters, ["-c", REF_CFG])
    _, (p_our, m_our) = flags.get_params(getters, ["-c", CFG])
    skip = {"config_file", "trainer_config_file", "model_config_file"}
    assert {k: v for k, v in vars(p_ref).items() if k not in skip} == {k: v for k, v in vars(p_our).items() if k not in skip}
    assert {k: v for k, v in vars(m_ref).items() if k not in skip} == {k: v for k, v in vars(m_our).items() if k not in skip}


def test_get_params_rejects_unknown_everywhere(tmp_path):
    path = _write(tmp_path, open(CFG).read() + "\nnot_a_flag = 1\n")
    with pytest.raises(SystemExit):
        flags.get_params((flags.get_trainer_parser, flags.get_model_parser), ["-c", path])


def test_write_and_reload_config(tmp_path):
    (tp, mp), (params, model_params) = flags.get_params((flags.get_trainer_parser, flags.get_model_parser),
                                                        ["-c", CFG, "--lr", "3e-5"])
    out = tmp_path / "trainer.cfg"
    flags.write_config_file(tp, params, out)
    text = out.read_text()
    assert "lr = 3e-05" in text and "config_file" not in text
    _, again = flags.load_config_file(flags.get_trainer_parser, str(out))
    for k in ("lr", "train_batch_size", "loss", "dummy_dataset", "apex_level", "warmup_coef", "best_order"):
        assert getattr(again, k) == getattr(params, k), k
    mo = tmp_path / "model.cfg"
    flags.write_config_file(mp, model_params, mo)
    _, m2 = flags.load_config_file(flags.get_model_parser, str(mo))
    assert m2.model == model_params.model and m2.hidden_dropout_prob == model_params.hidden_dropout_prob


def test_predictor_parser_validate_cfg():
    path = os.path.join(ROOT, "config", "validate.cfg")
    _, (p, m) = flags.get_params((flags.get_predictor_parser, flags.get_model_parser), ["-c", path])
    assert p.limit == 100 and p.split_by_sentence and p.truncate and p.max_seq_len == 512


def test_set_seed_selects_deterministic_kernels(monkeypatch):
    """Like the reference's set_seed (cudnn.deterministic = True), a seed selects the run-to-run
    reproducible kernels (ops.deterministic); no seed leaves the choice alone."""
    import random

    from ml_recipe_distributed_pytorch_amd import ops
    from ml_recipe_distributed_pytorch_amd.utils.logging import set_seed
    monkeypatch.setenv("HQ_DETERMINISTIC", "0")   # restored (unset) at teardown
    assert set_seed(None) is None and not ops.deterministic()
    assert set_seed("7") == 7 and ops.deterministic()
    a = random.random()
    set_seed(7)
    assert random.random() == a


def test_hw_queue_reservation_skipped_when_ranks_share_a_gpu(monkeypatch):
    """8 HIP hardware queues per process only when each rank has its own GPU: ranks sharing one (the
    gloo rehearsal, more local ranks than visible GPUs) keep HIP's default."""
    import ml_recipe_distributed_pytorch_amd as pkg
    monkeypatch.delenv("HQ_BENCH_BACKEND", raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert not pkg._ranks_share_a_gpu()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    assert pkg._ranks_share_a_gpu()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setenv("HQ_BENCH_BACKEND", "gloo")
    assert pkg._ranks_share_a_gpu()
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    pkg._reserve_hw_queues()
    import os
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
    monkeypatch.setenv("HQ_BENCH_BACKEND", "nccl")
    pkg._reserve_hw_queues()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "8"
