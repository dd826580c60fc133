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
