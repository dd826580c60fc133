"""optim.SGD mirror running the fused flat-buffer Nesterov kernel.

Reference: ``optim.SGD(self.model.parameters(), lr, weight_decay, momentum=0.9, nesterov=True)``
(src/ddp/trainer.py:92-98) stepped through ``GradScaler.step`` (trainer.py:158). The class
subclasses ``torch.optim.Optimizer`` so ``optim.lr_scheduler.StepLR`` (trainer.py:101-105)
drives ``param_groups[0]['lr']`` unchanged; ``step()`` enqueues ONE kernel over the model's
flat parameter / gradient / momentum buffers that also refreshes the bf16 weight shadow.
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from . import ops
from ._native import NativeError


class SGD(Optimizer):
    def __init__(self, params, lr, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        params = list(params)
        if isinstance(params[0], dict):
            raise NotImplementedError("per-parameter groups are not used by the reference (trainer.py:92-98)")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)
        if not nesterov or dampening != 0.0 or momentum <= 0.0:
            raise NotImplementedError("the fused kernel implements SGD(momentum>0, dampening=0, nesterov=True) "
                                      "as used by the reference (trainer.py:92-98)")
        self._flat = None
        self._mom = None

    def attach(self, model):
        """Bind to the model's flat buffers (done lazily on the first step)."""
        flat = model.flat
        ids = {p.data_ptr() for p in self.param_groups[0]["params"]}
        if len(ids) != len(flat.layout.params):
            raise NativeError("SGD must own every parameter of the model (flat-buffer update)")
        self._flat = flat
        self._mom = torch.zeros_like(flat.params)

    def _find_flat(self):
        ref = getattr(self.param_groups[0]["params"][0], "_dtc_model", None)
        model = ref() if ref is not None else None
        if model is None:
            raise NativeError("SGD parameters do not belong to a native ResNet moved to the GPU "
                              "(create the optimizer after model.to('cuda'))")
        return model

    def zero_grad(self, set_to_none: bool = True):
        # The native backward WRITES every gradient (it never accumulates), which is exactly
        # the state zero_grad() + backward() produces in the reference; nothing to clear.
        return None

    @torch.no_grad()
    def step(self, closure=None, inv_scale=None, found_inf=None):
        if closure is not None:
            raise NotImplementedError("closures are not used by the reference")
        if self._flat is None:
            self.attach(self._find_flat())
        g = self.param_groups[0]
        ops.sgd_nesterov_flat(self._flat.params, self._flat.grads, self._mom, self._flat.params_bf16, g["lr"],
                              g["weight_decay"], g["momentum"], inv_scale, found_inf)
        return None
