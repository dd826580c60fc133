"""MI355X-native ResNet-18 / CIFAR-100 data-parallel training step.

Drop-in for the hot path of youngerous/distributed-training-comparison (src/{single,dp,ddp}):
the reference's PyTorch operator surface (ResNet18, CrossEntropyLoss, SGD, GradScaler,
autocast, DistributedDataParallel, DistributedSampler sharding) on top of hand-written gfx950
HIP kernels and an RCCL reducer exposed through the C ABI in include/dtc.h.

The directory name is not a Python identifier; importing it by path also registers the alias
``dtc_amd`` so ``import dtc_amd`` works afterwards.
"""
import sys as _sys

from . import _native  # noqa: F401  (loads libdtc_amd.so; raises if it is missing)
from ._native import NativeError  # noqa: F401
from . import data, ops  # noqa: F401
from .amp import GradScaler, autocast  # noqa: F401
from .nn import BasicBlock, CrossEntropyLoss, ResNet, ResNet18, SyncBatchNorm  # noqa: F401
from .optim import SGD  # noqa: F401
from .parallel import DDP, Comm, DataParallel, DistributedDataParallel, barrier  # noqa: F401
from . import parallel  # noqa: F401
from . import trainer  # noqa: F401

_sys.modules.setdefault("dtc_amd", _sys.modules[__name__])

__version__ = "0.1.0"
