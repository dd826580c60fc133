"""Data-side plumbing of the reference, kept bit-compatible.

* ``fix_seed`` — src/ddp/utils.py:8-15.
* ``train_valid_split`` — the 45k/5k split of src/ddp/dataset.py:85-92: ``np.random.shuffle`` of
  ``list(range(50000))`` under the global numpy state seeded by fix_seed(42).
* ``shard_indices`` / ``DistributedSampler`` — the per-epoch sharding of
  ``torch.utils.data.distributed.DistributedSampler`` as used at src/ddp/dataset.py:98 with
  ``set_epoch(epoch)`` (src/ddp/trainer.py:125): ``randperm(n, Generator.manual_seed(seed+epoch))``,
  padded to a multiple of the world size, then ``[rank::world]``.
* ``SyntheticCIFAR100`` — CIFAR-100 is not downloadable here (dataset.py:70-82 uses
  ``download=True``), so training uses a seeded synthetic stand-in of the same shape
  (SURVEY.md §8(d)): ``x = 0.5*T[y] + N(0,1)`` with class templates ``T`` (seed 1234), which keeps
  the loss learnable for loss-curve checks.
"""
from __future__ import annotations

import math
import random
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch
import torch.utils.data as tud

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)  # dataset.py:43-46
CIFAR_STD = (0.2023, 0.1994, 0.2010)
IMAGENET_MEAN = (0.485, 0.456, 0.406)  # dataset.py:139-142 (test loader)
IMAGENET_STD = (0.229, 0.224, 0.225)


def fix_seed(seed: int) -> None:
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)


def train_valid_split(num_train: int = 50000, valid_size: float = 0.1, shuffle: bool = True
                      ) -> Tuple[List[int], List[int]]:
    if not (0 <= valid_size <= 1):
        raise ValueError("[!] valid_size should be in the range [0, 1].")
    indices = list(range(num_train))
    split = int(np.floor(valid_size * num_train))
    if shuffle:
        np.random.shuffle(indices)
    return indices[split:], indices[:split]


def shard_indices(n: int, num_replicas: int, rank: int, epoch: int = 0, seed: int = 0, shuffle: bool = True,
                  drop_last: bool = False) -> List[int]:
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g).tolist()
    else:
        indices = list(range(n))
    if drop_last and n % num_replicas != 0:
        num_samples = math.ceil((n - num_replicas) / num_replicas)
    else:
        num_samples = math.ceil(n / num_replicas)
    total = num_samples * num_replicas
    if not drop_last:
        pad = total - len(indices)
        if pad <= len(indices):
            indices += indices[:pad]
        else:
            indices += (indices * math.ceil(pad / len(indices)))[:pad]
    else:
        indices = indices[:total]
    return indices[rank:total:num_replicas]


class DistributedSampler(tud.Sampler):
    """Same index stream as torch's DistributedSampler (dataset.py:98) with set_epoch()."""

    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None, shuffle=True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            import torch.distributed as dist
            num_replicas = dist.get_world_size() if num_replicas is None else num_replicas
            rank = dist.get_rank() if rank is None else rank
        self.n = len(dataset)
        self.num_replicas, self.rank = num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def __iter__(self) -> Iterator[int]:
        return iter(shard_indices(self.n, self.num_replicas, self.rank, self.epoch, self.seed, self.shuffle,
                                  self.drop_last))

    def __len__(self) -> int:
        if self.drop_last and self.n % self.num_replicas != 0:
            return math.ceil((self.n - self.num_replicas) / self.num_replicas)
        return math.ceil(self.n / self.num_replicas)


def class_templates(num_classes=100, height=32, width=32, seed=1234) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn(num_classes, 3, height, width, generator=g)


class SyntheticCIFAR100(tud.Dataset):
    """Seeded CIFAR-100-shaped data: image i = 0.5*T[y_i] + N(0,1) (per-index generator), normalized
    like dataset.py:43-46 would leave it (zero-mean, unit-scale)."""

    def __init__(self, n: int = 50000, height: int = 32, width: int = 32, num_classes: int = 100, seed: int = 1234):
        self.n, self.h, self.w, self.num_classes, self.seed = n, height, width, num_classes, seed
        self.templates = class_templates(num_classes, height, width, seed)
        g = torch.Generator().manual_seed(seed + 1)
        self.labels = torch.randint(0, num_classes, (n,), generator=g)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        y = int(self.labels[i])
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        x = 0.5 * self.templates[y] + torch.randn(3, self.h, self.w, generator=g)
        return x, y


def synthetic_batch(step: int, batch: int, height: int = 32, width: int = 32, num_classes: int = 100,
                    device="cpu", templates: Optional[torch.Tensor] = None, seed: int = 1234):
    """One batch of the §8(d) stream: labels randint(seed+step), x = 0.5*T[y] + randn (CPU RNG, so
    the stream is identical on every machine), returned on `device`."""
    if templates is None:
        templates = class_templates(num_classes, height, width, seed)
    g = torch.Generator().manual_seed(seed + step)
    y = torch.randint(0, num_classes, (batch,), generator=g)
    x = 0.5 * templates[y] + torch.randn(batch, 3, height, width, generator=g)
    return x.to(device), y.to(device)


def get_trn_val_loader(batch_size: int, valid_size: float = 0.1, num_workers: int = 0, pin_memory: bool = True,
                       distributed: bool = True, dataset: Optional[tud.Dataset] = None, **_):
    """dataset.py:15-116 with the synthetic dataset; returns (train_loader, train_sampler, valid_loader)."""
    ds = dataset if dataset is not None else SyntheticCIFAR100()
    train_idx, valid_idx = train_valid_split(len(ds), valid_size, True)
    train_ds, valid_ds = tud.Subset(ds, train_idx), tud.Subset(ds, valid_idx)
    if distributed:
        sampler = DistributedSampler(train_ds)
        shuffle = False
    else:
        sampler = tud.SubsetRandomSampler(list(range(len(train_ds))))
        shuffle = False
    train_loader = tud.DataLoader(train_ds, batch_size=batch_size, sampler=sampler, num_workers=num_workers,
                                  pin_memory=pin_memory, drop_last=True, shuffle=shuffle)
    valid_loader = tud.DataLoader(valid_ds, batch_size=batch_size, num_workers=num_workers, pin_memory=pin_memory)
    return train_loader, sampler, valid_loader


def get_tst_loader(batch_size: int, num_workers: int = 0, pin_memory: bool = False, distributed: bool = True,
                   n: int = 10000, **_):
    """dataset.py:119-168 with a synthetic 10k test split (different seed)."""
    ds = SyntheticCIFAR100(n=n, seed=4321)
    sampler = DistributedSampler(ds) if distributed else None
    return tud.DataLoader(ds, batch_size=batch_size, shuffle=False, sampler=sampler, num_workers=num_workers,
                          pin_memory=pin_memory)


# ----------------------------------------------------------------------------- on-device input pipeline
def synthetic_cifar_u8(n: int = 50000, height: int = 32, width: int = 32, num_classes: int = 100, seed: int = 1234):
    """CIFAR-100 in its stored form (uint8 [n, h, w, 3] HWC + int64 targets), seeded synthetic:
    pixel = clip(128 + 48*T[y] + 40*N(0,1)) with per-class templates T (numpy, CPU-deterministic)."""
    rng = np.random.default_rng(seed)
    templates = rng.standard_normal((num_classes, height, width, 3), dtype=np.float32)
    targets = rng.integers(0, num_classes, n, dtype=np.int64)
    images = np.empty((n, height, width, 3), np.uint8)
    for s in range(0, n, 4096):  # bounded temporaries
        e = min(n, s + 4096)
        v = 128.0 + 48.0 * templates[targets[s:e]] + 40.0 * rng.standard_normal((e - s, height, width, 3),
                                                                                  dtype=np.float32)
        images[s:e] = np.clip(np.rint(v), 0, 255).astype(np.uint8)
    return images, targets


class DeviceLoader:
    """``DataLoader(Subset(dataset, subset_idx), batch_size, sampler=sampler, drop_last=...)`` with
    the reference's train (or valid/test) transform (src/ddp/dataset.py:43-64, 95-116) executed on
    the GPU: the uint8 dataset stays resident in HBM (153.6 MB for CIFAR's 50k images); per epoch
    the sampler's index list (bit-identical to torch's DistributedSampler) is composed with the
    Subset map on the host and uploaded once; per batch one HIP launch gathers, crops, flips and
    normalizes (``ops.cifar_augment``). Crop offsets / flips are drawn on the device from a
    generator seeded with ``seed + epoch`` (torchvision draws them with the worker processes' CPU
    RNG, which no run reproduces across worker counts either; distributions are the same:
    offsets uniform on [0, 2*pad], flip with p = 0.5). Out-of-range indices are detected on the
    device and raised at the end of the epoch (one host sync per epoch)."""

    def __init__(self, images, targets, batch_size: int, subset_idx=None, sampler=None, train: bool = True,
                 mean=CIFAR_MEAN, std=CIFAR_STD, pad: int = 4, drop_last: bool = True, seed: int = 0,
                 device=None):
        from . import ops

        self._ops = ops
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.images = torch.as_tensor(images).to(dev).contiguous()
        self.targets = torch.as_tensor(targets, dtype=torch.int64).to(dev).contiguous()
        self.subset_idx = (np.arange(self.images.shape[0], dtype=np.int64) if subset_idx is None
                           else np.asarray(subset_idx, np.int64))
        self.batch_size, self.sampler, self.train = int(batch_size), sampler, bool(train)
        self.mean, self.std, self.pad, self.drop_last = tuple(mean), tuple(std), int(pad), bool(drop_last)
        self.seed, self.device, self.epoch = int(seed), dev, 0
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.last_params = None  # (index, crop, flip) of the last batch, for tests

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _rows(self) -> np.ndarray:
        order = np.fromiter(iter(self.sampler), np.int64) if self.sampler is not None else \
            np.arange(len(self.subset_idx), dtype=np.int64)
        return self.subset_idx[order]

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.subset_idx)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        rows = torch.from_numpy(self._rows()).to(self.device)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(self.seed + self.epoch)
        B = self.batch_size
        finished = False
        try:
            for k in range(len(self)):
                idx = rows[k * B:(k + 1) * B]
                n = idx.numel()
                crop = flip = None
                if self.train:
                    crop = torch.randint(0, 2 * self.pad + 1, (n, 2), dtype=torch.uint8, device=self.device,
                                         generator=gen)
                    flip = torch.randint(0, 2, (n,), dtype=torch.uint8, device=self.device, generator=gen)
                self.last_params = (idx, crop, flip)
                yield self._ops.cifar_augment(self.images, idx, crop, flip, self.mean, self.std, self.pad,
                                              targets=self.targets, status=self.status)
            finished = True
        finally:
            # checked however the epoch ends (also when the consumer breaks early, e.g. --max-steps),
            # and reset, so a bad index is reported for the epoch it happened in, never a later one
            if int(self.status.item()):
                self.status.zero_()
                msg = "DeviceLoader: a sampler index or crop offset was out of range this epoch"
                if finished:
                    raise IndexError(msg)
                import warnings

                warnings.warn(msg + " (epoch ended early)", RuntimeWarning)
