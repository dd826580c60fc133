"""On-device CIFAR input pipeline: the HIP gather + RandomCrop + flip +
ToTensor + Normalize launch against the numpy oracle (oracle.ops.cifar_augment), BIT-EXACT (the
kernel performs the same fp32 operations in the same order), and the DeviceLoader's epoch
stream against the sampler/Subset composition of the reference (src/ddp/dataset.py:95-108)."""
import numpy as np
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


def _data(n=64, h=32, w=32, seed=0):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, (n, h, w, 3), dtype=np.uint8), g.integers(0, 100, n, dtype=np.int64)


@pytest.mark.parametrize("h,w,pad,n", [(32, 32, 4, 37), (32, 32, 4, 1), (8, 12, 2, 19), (32, 32, 0, 5)])
def test_augment_matches_oracle_bit_exact(dtc, cuda, h, w, pad, n):
    imgs, tg = _data(50, h, w)
    g = np.random.default_rng(1)
    idx = g.integers(0, 50, n)
    crop = g.integers(0, 2 * pad + 1, (n, 2)).astype(np.uint8)
    crop[0] = (0, 2 * pad)  # both extremes of the padded window
    flip = g.integers(0, 2, n).astype(np.uint8)
    ref, ref_lab = O.cifar_augment(imgs, tg, idx, crop, flip, O.CIFAR_MEAN, O.CIFAR_STD, pad)
    D = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    out, lab = dtc.ops.cifar_augment(D(imgs), D(idx), D(crop), D(flip), O.CIFAR_MEAN, O.CIFAR_STD, pad,
                                     targets=D(tg), status=status)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert np.array_equal(lab.cpu().numpy(), ref_lab)
    assert int(status.item()) == 0


def test_augment_valid_transform_and_test_normalization(dtc, cuda):
    """crop/flip NULL = the valid/test transform (ToTensor + Normalize only); the test loader's
    ImageNet statistics (dataset.py:139-142) are plain arguments."""
    imgs, tg = _data(20)
    D = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    for mean, std in ((O.CIFAR_MEAN, O.CIFAR_STD), (O.IMAGENET_MEAN, O.IMAGENET_STD)):
        out, lab = dtc.ops.cifar_augment(D(imgs), None, None, None, mean, std, 4, targets=D(tg))
        ref, ref_lab = O.cifar_augment(imgs, tg, None, None, None, mean, std, 4)
        assert np.array_equal(out.cpu().numpy(), ref)
        assert np.array_equal(lab.cpu().numpy(), ref_lab)


def test_augment_out_of_range_flags_status(dtc, cuda):
    imgs, tg = _data(10)
    D = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    status = torch.zeros(1, dtype=torch.int32, device=cuda)
    idx = np.array([0, 10, -1, 3], np.int64)  # two bad rows
    out, lab = dtc.ops.cifar_augment(D(imgs), D(idx), None, None, O.CIFAR_MEAN, O.CIFAR_STD, 4, targets=D(tg),
                                     status=status)
    assert int(status.item()) == 1
    o, lb = out.cpu().numpy(), lab.cpu().numpy()
    zero = (np.float32(0) - np.asarray(O.CIFAR_MEAN, np.float32)) / np.asarray(O.CIFAR_STD, np.float32)
    assert np.array_equal(o[1], np.broadcast_to(zero[:, None, None], o[1].shape)) and lb[1] == 0 and lb[2] == 0
    ref, _ = O.cifar_augment(imgs, tg, idx[[0, 3]], None, None, O.CIFAR_MEAN, O.CIFAR_STD, 4)
    assert np.array_equal(o[[0, 3]], ref)
    status.zero_()
    bad_crop = np.array([[9, 0]], np.uint8)  # offset beyond 2*pad
    dtc.ops.cifar_augment(D(imgs), D(idx[:1]), D(bad_crop), None, O.CIFAR_MEAN, O.CIFAR_STD, 4, status=status)
    assert int(status.item()) == 1
    with pytest.raises(Exception, match="bad shape"):
        dtc.ops.cifar_augment(D(np.zeros((2, 32, 30, 3), np.uint8)), None, None, None, O.CIFAR_MEAN, O.CIFAR_STD)


def test_device_loader_epoch_matches_sampler_and_oracle(dtc, cuda):
    """Two ranks' DeviceLoaders over Subset(train_idx) + DistributedSampler: the rows of every
    batch are the reference's (sampler order through the Subset map, drop_last), each batch equals
    the oracle on the loader's own crop/flip draws, and draws are reproducible per epoch."""
    imgs, tg = _data(300)
    train_idx = np.random.default_rng(5).permutation(300)[30:]
    seen = []
    for rank in range(2):
        sampler = dtc.data.DistributedSampler(range(len(train_idx)), num_replicas=2, rank=rank)
        loader = dtc.data.DeviceLoader(imgs, tg, 32, subset_idx=train_idx, sampler=sampler, device=cuda, seed=3)
        loader.set_epoch(1)
        order = train_idx[dtc.data.shard_indices(len(train_idx), 2, rank, epoch=1)]
        assert len(loader) == len(order) // 32
        first = None
        for k, (x, y) in enumerate(loader):
            idx, crop, flip = loader.last_params
            assert np.array_equal(idx.cpu().numpy(), order[k * 32:(k + 1) * 32])
            ref, ref_lab = O.cifar_augment(imgs, tg, idx.cpu().numpy(), crop.cpu().numpy(), flip.cpu().numpy(),
                                           O.CIFAR_MEAN, O.CIFAR_STD, 4)
            assert np.array_equal(x.cpu().numpy(), ref) and np.array_equal(y.cpu().numpy(), ref_lab)
            if first is None:
                first = (crop.cpu().numpy().copy(), flip.cpu().numpy().copy())
            seen.extend(idx.cpu().tolist())
        loader.set_epoch(1)
        next(iter(loader))
        assert np.array_equal(loader.last_params[1].cpu().numpy(), first[0])
        assert np.array_equal(loader.last_params[2].cpu().numpy(), first[1])
    assert len(set(seen)) == len(seen)  # ranks' shards are disjoint


def test_device_loader_trains_native_resnet(dtc, cuda):
    """One epoch slice of the DDP loop body fed by the DeviceLoader (the loader's fp32 NCHW output
    is the model's input boundary)."""
    imgs, tg = dtc.data.synthetic_cifar_u8(n=512, seed=7)
    loader = dtc.data.DeviceLoader(imgs, tg, 64, device=cuda)
    torch.manual_seed(42)
    model = dtc.ResNet18().to(cuda)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, nesterov=True)
    losses = []
    for x, y in loader:
        opt.zero_grad()
        loss = crit(model(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert len(losses) == 8 and all(np.isfinite(losses))


def test_single_trainer_with_device_data(dtc, cuda, tmp_path):
    """`train.py single --device-data`: the reference loop fed by DeviceLoaders (train with
    crop/flip, valid, ImageNet-normalized test) through fit -> validate -> checkpoint -> test."""
    import os

    t = dtc.trainer.main(["--epoch", "2", "--batch-size", "64", "--max-steps", "3", "--amp", "--contain-test",
                          "--synthetic-train", "1000", "--synthetic-test", "200", "--device-data",
                          "--ckpt-path", str(tmp_path)], "single")
    assert isinstance(t.train_loader, dtc.data.DeviceLoader)
    assert t.train_loader.epoch == 1 and len(t.train_loader) == 900 // 64
    assert len(t.val_loader) == 2 and len(t.test_loader) == 4
    assert t.test_loader.mean == dtc.data.IMAGENET_MEAN
    assert os.path.exists(os.path.join(str(tmp_path), "version-0", "experiment.log"))
