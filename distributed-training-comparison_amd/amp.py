"""GradScaler / autocast mirrors with device-side state (no host synchronisation).

Reference: ``torch.cuda.amp.GradScaler()`` (src/ddp/main.py:25) used as
``scaler.scale(loss).backward(); scaler.step(optimizer); scaler.update()`` (trainer.py:157-159)
inside ``torch.cuda.amp.autocast()`` (trainer.py:153).

Inside ``autocast`` the native network computes in bf16 with fp32 accumulation and fp32 master
weights (the reference's fp16 autocast replaced by bf16, BASELINE.json north_star); outside it in
fp32, like the reference without --amp. GradScaler keeps torch's semantics exactly: the loss is
multiplied by ``scale``; before the step every gradient is checked for inf/NaN (after the DDP
all-reduce, so all ranks agree); an overflowing step is skipped; ``scale`` backs off by 0.5 on
overflow and grows by 2 after 2000 clean steps. ``found_inf`` and the scale never leave the GPU.
"""
from __future__ import annotations

import contextlib
import weakref

import torch

from . import ops
from .nn import _PRESCALER, is_autocast_enabled, scaled_loss, set_autocast_enabled


@contextlib.contextmanager
def autocast(enabled: bool = True, dtype=torch.bfloat16):
    """torch.cuda.amp.autocast() (trainer.py:153): inside it the native ResNet runs its bf16 executor
    (bf16 activations, fp32 accumulation / statistics / master weights; the reference autocasts to
    fp16, north_star asks for bf16); outside it, or with enabled=False, the fp32 executor -- the
    reference's non-AMP path (trainer.py:160-165). Thread-local and nestable, as torch's."""
    prev = is_autocast_enabled()
    set_autocast_enabled(enabled)
    try:
        yield
    finally:
        set_autocast_enabled(prev)


class GradScaler:
    def __init__(self, init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        self._enabled = enabled
        self._init_scale = float(init_scale)
        self._growth = float(growth_factor)
        self._backoff = float(backoff_factor)
        self._interval = int(growth_interval)
        self._scale = None
        self._inv_scale = None
        self._tracker = None
        self._found_inf = None
        self._unscaled = False
        self._version = 0  # bumped whenever the scale may change (update): invalidates prescaled losses

    def _lazy_init(self, device):
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=device)
            self._inv_scale = torch.full((1,), 1.0 / self._init_scale, dtype=torch.float32, device=device)
            self._tracker = torch.zeros(1, dtype=torch.int32, device=device)
            self._found_inf = torch.zeros(1, dtype=torch.int32, device=device)
            _PRESCALER[0] = weakref.ref(self)

    def is_enabled(self):
        return self._enabled

    def scale(self, outputs: torch.Tensor) -> torch.Tensor:
        if not self._enabled:
            return outputs
        self._lazy_init(outputs.device)
        return scaled_loss(outputs, self._scale, self._version)

    def unscale_(self, optimizer) -> None:
        if not self._enabled or self._unscaled:
            return
        flat = optimizer._flat if optimizer._flat is not None else None
        if flat is None:
            optimizer.attach(optimizer._find_flat())
            flat = optimizer._flat
        self._lazy_init(flat.grads.device)
        ops.amp_check_finite(flat.grads, self._found_inf)
        self._unscaled = True

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        self.unscale_(optimizer)
        # the kernel applies grad * inv_scale and skips the update when found_inf != 0
        optimizer.step(inv_scale=self._inv_scale, found_inf=self._found_inf)
        return None

    def update(self, new_scale=None) -> None:
        if not self._enabled or self._scale is None:
            return
        self._version += 1
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
            self._inv_scale.fill_(1.0 / float(new_scale))
            self._found_inf.zero_()
        else:
            ops.amp_update_scale(self._scale, self._inv_scale, self._tracker, self._found_inf, self._growth,
                                 self._backoff, self._interval)
        self._unscaled = False

    def get_scale(self) -> float:
        if not self._enabled:
            return 1.0
        return self._init_scale if self._scale is None else float(self._scale.item())

    def state_dict(self):
        return {"scale": self.get_scale(), "growth_factor": self._growth, "backoff_factor": self._backoff,
                "growth_interval": self._interval,
                "_growth_tracker": 0 if self._tracker is None else int(self._tracker.item())}
