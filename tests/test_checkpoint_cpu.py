"""Checkpoint compatibility (tmrnet_amd/checkpoint.py): both trunk namespaces,
DataParallel prefixes, explicit reporting of keys the reference's strict=False drops silently,
and torch's lr schedulers on tmrnet_amd.SGD (parameter containers only -- no GPU needed)."""
import warnings

import pytest
import torch

import tmrnet_amd
from tmrnet_amd import checkpoint as ck
from tmrnet_amd.model import MemoryBankModel


def test_namespace_round_trip():
    torch.manual_seed(0)
    a = MemoryBankModel(seq_len=10)                       # share.*
    b = MemoryBankModel(seq_len=10, indexed_trunk=True)   # res.* (code/models.py)
    sd_res = ck.convert_trunk_namespace(a.state_dict(), "res")
    assert set(sd_res) == set(b.state_dict())
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        missing, unexpected = ck.load_checkpoint(b, a.state_dict())
    assert not missing and not unexpected
    for k, v in b.state_dict().items():
        assert torch.equal(v, sd_res[k])
    back = ck.convert_trunk_namespace(sd_res, "share")
    assert all(torch.equal(back[k], v) for k, v in a.state_dict().items())


def test_memory_bank_checkpoint_into_lfb_model(tmp_path):
    """train_memorybank.py saves res.* keys; the LFB/TMRNet scripts load them with strict=False
    into share.* models, which in the reference silently keeps the random trunk."""
    torch.manual_seed(0)
    from tmrnet_amd.compat import models as mb_models
    mb = mb_models.resnet_lstm(
        type("A", (), {"num_frames": 10, "opt": 0, "lr": 1e-3, "momentum": 0.9, "dampening": 0,
                       "weightdecay": 5e-4, "nesterov": False})(), 7)
    p = tmp_path / "mb.pth"
    torch.save({"module." + k: v for k, v in mb.state_dict().items()}, p)   # DataParallel form
    lfb = tmrnet_amd.resnet_lstm_LFB(seq_len=10)
    with pytest.warns(ck.CheckpointKeyWarning) as rec:
        missing, unexpected = ck.load_checkpoint(lfb, str(p))
    assert missing == [] and unexpected == ["fc.weight", "fc.bias"]
    assert "fc.weight" in str(rec[0].message)
    assert torch.equal(lfb.share.layer4[2].conv3.weight, mb.res[7][2].conv3.weight)
    assert torch.equal(lfb.lstm.weight_hh_l0, mb.lstm.weight_hh_l0)
    with pytest.raises(RuntimeError):
        ck.load_checkpoint(lfb, str(p), strict=True)


def test_tmrnet_partial_load_reports_missing(tmp_path):
    """resnet_lstm <- resnet_lstm_LFB checkpoint (:625): nl_block/fc keys stay at init, reported."""
    src = tmrnet_amd.resnet_lstm_LFB(seq_len=10)
    dst = tmrnet_amd.resnet_lstm(seq_len=10)
    p = tmp_path / "lfb.pth"
    ck.save_checkpoint(src, str(p))
    with pytest.warns(ck.CheckpointKeyWarning):
        missing, unexpected = ck.load_checkpoint(dst, str(p))
    assert unexpected == []
    assert set(missing) == {k for k in dst.state_dict() if k.split(".")[0] in
                            ("fc_c", "fc_h_c", "nl_block")}


def test_save_other_namespace(tmp_path):
    m = tmrnet_amd.resnet_lstm_LFB(seq_len=10)
    p = tmp_path / "r.pth"
    ck.save_checkpoint(m, str(p), namespace="res")
    sd = torch.load(str(p), weights_only=True)
    assert "res.4.0.conv1.weight" in sd and "share.conv1.weight" not in sd


def test_reduce_lr_on_plateau_drives_sgd_groups():
    m = tmrnet_amd.resnet_lstm(seq_len=10)
    from oracle.tmrnet_ref import sgd_param_groups
    opt = tmrnet_amd.SGD(sgd_param_groups(m, 5e-7), lr=5e-8, momentum=0.9, weight_decay=5e-4)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "max", factor=0.1, patience=0)
    sch.step(0.5)
    sch.step(0.4)            # no improvement -> every group's lr x0.1
    lrs = [g["lr"] for g in opt.param_groups]
    assert lrs[0] == pytest.approx(5e-9) and lrs[-1] == pytest.approx(5e-8)
