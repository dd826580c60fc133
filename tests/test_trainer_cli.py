"""CLI mirror: flags and defaults identical to the reference config.py files (CPU only)."""
import pytest


def test_ddp_flags_match_reference_defaults(dtc):
    h = dtc.trainer.load_config([], "ddp")
    assert (h.seed, h.workers, h.eval_step, h.amp, h.contain_test) == (42, 4, 300, False, False)
    assert (h.world_size, h.rank, h.dist_backend, h.dist_url) == (1, 0, "nccl", "tcp://127.0.0.1:3456")
    assert (h.epoch, h.batch_size, h.model, h.lr, h.weight_decay) == (100, 128, "resnet18", 0.1, 0.0001)
    assert (h.lr_decay_step_size, h.lr_decay_gamma, h.ckpt_path) == (60, 0.1, "src/ddp/checkpoints/")


def test_single_flags_and_launcher_overrides(dtc):
    h = dtc.trainer.load_config(["--seed=42", "--epoch=50", "--batch-size=128", "--lr=0.1", "--weight-decay=0.0001",
                                 "--lr-decay-step-size=25", "--lr-decay-gamma=0.1", "--amp", "--contain-test"],
                                "single")  # run_single.sh:13-22
    assert not hasattr(h, "dist_url")
    assert (h.epoch, h.batch_size, h.lr_decay_step_size, h.amp, h.contain_test) == (50, 128, 25, True, True)
    assert dtc.trainer.load_config([], "single").epoch == 200


def test_accuracy_and_meter(dtc):
    import torch
    out = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1], [0.2, 0.3, 0.5]])
    tgt = torch.tensor([1, 2, 2])
    top1, top2 = dtc.trainer.accuracy(out, tgt, topk=(1, 2))
    assert abs(float(top1) - 200 / 3) < 1e-4 and abs(float(top2) - 200 / 3) < 1e-4
    m = dtc.trainer.AverageMeter()
    m.update(2.0)
    m.update(4.0, 3)
    assert m.avg == 3.5


def test_dp_flags_match_reference_defaults(dtc):
    h = dtc.trainer.load_config([], "dp")  # src/dp/config.py:8-28
    assert not hasattr(h, "dist_url") and h.device_ids is None
    assert (h.epoch, h.batch_size, h.lr_decay_step_size, h.ckpt_path) == (100, 128, 60, "src/dp/checkpoints/")
    assert dtc.trainer.load_config(["--device-ids", "0,0"], "dp").device_ids == [0, 0]
    with pytest.raises(ValueError):
        dtc.trainer.main([], "bogus")


def test_sync_bn_flag_and_conversion(dtc):
    """--sync-bn (ddp mode only, off by default as in the reference) and
    SyncBatchNorm.convert_sync_batchnorm: marks the native ResNet in place (BN modules and
    state_dict keys unchanged); anything else is refused rather than silently left unsynchronised."""
    assert dtc.trainer.load_config([], "ddp").sync_bn is False
    assert dtc.trainer.load_config(["--sync-bn"], "ddp").sync_bn is True
    assert not hasattr(dtc.trainer.load_config([], "single"), "sync_bn")
    m = dtc.ResNet18()
    keys = list(m.state_dict().keys())
    out = dtc.SyncBatchNorm.convert_sync_batchnorm(m)
    assert out is m and m._sync_bn and list(m.state_dict().keys()) == keys
    import torch.nn as tnn
    with pytest.raises(NotImplementedError):
        dtc.SyncBatchNorm.convert_sync_batchnorm(tnn.BatchNorm2d(4))
