"""Stock-torch CPU restatement of the reference's single-device training step — TEST / BASELINE
INFRASTRUCTURE ONLY (see oracle/ops.py for the rules: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product path never does).

This is BASELINE.json config 1 (SURVEY.md §8(d) "CPU timing"): the reference's `src/single` step
(single/trainer.py:131-147: zero_grad -> forward -> CrossEntropyLoss -> backward -> SGD.step) in fp32
on the host cores, written functionally over a ResNet18() state_dict so that no reference source
ships with the build:

* forward = net.py:107-116 / BasicBlock.forward net.py:40-45 with F.conv2d / F.batch_norm(training)
  / F.relu / F.avg_pool2d(4) / F.linear (the same ATen CPU kernels nn.Conv2d etc. dispatch to);
* loss = nn.CrossEntropyLoss() mean (trainer.py:40);
* update = torch.optim.SGD(lr, weight_decay, momentum=0.9, nesterov=True) (trainer.py:92-98).

tests/test_oracle_golden.py pins it against the reference-produced fp32 fixture (resnet18_b2.json).
"""
from __future__ import annotations

import statistics
import time
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F


def _blocks() -> List[Tuple[str, int, bool]]:
    out = []
    for L in range(1, 5):
        for b in range(2):
            stride = 2 if (L > 1 and b == 0) else 1
            out.append((f"layer{L}.{b}", stride, L > 1 and b == 0))
    return out


class TorchCPUStep:
    """Functional ResNet-18 (CIFAR) train step in stock torch on the CPU, fp32."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], lr=0.1, weight_decay=1e-4, momentum=0.9):
        self.p = {k: v.detach().float().clone().requires_grad_(True) for k, v in state_dict.items()
                  if not (k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"))}
        self.buf = {k: v.detach().clone() for k, v in state_dict.items()
                    if k.endswith("running_mean") or k.endswith("running_var")}
        # registration order (net.py:86-105) = the optimizer's parameter order
        self.order = [k for k in state_dict if k in self.p]
        self.opt = torch.optim.SGD([self.p[k] for k in self.order], lr=lr, weight_decay=weight_decay,
                                   momentum=momentum, nesterov=True)

    def _bn(self, x, name, training=True):
        return F.batch_norm(x, self.buf[name + ".running_mean"], self.buf[name + ".running_var"],
                            self.p[name + ".weight"], self.p[name + ".bias"], training, 0.1, 1e-5)

    def forward(self, x, training=True):
        p = self.p
        out = F.relu(self._bn(F.conv2d(x, p["conv1.weight"], stride=1, padding=1), "bn1", training))
        for pre, stride, proj in _blocks():
            h = F.relu(self._bn(F.conv2d(out, p[pre + ".conv1.weight"], stride=stride, padding=1), pre + ".bn1",
                                training))
            h = self._bn(F.conv2d(h, p[pre + ".conv2.weight"], stride=1, padding=1), pre + ".bn2", training)
            if proj:
                sc = self._bn(F.conv2d(out, p[pre + ".shortcut.0.weight"], stride=stride), pre + ".shortcut.1",
                              training)
            else:
                sc = out
            out = F.relu(h + sc)
        out = F.avg_pool2d(out, 4).view(out.size(0), -1)
        return F.linear(out, p["linear.weight"], p["linear.bias"])

    def step(self, x, y) -> float:
        """single/trainer.py:131-147: zero_grad, forward, CE, backward, optimizer.step."""
        self.opt.zero_grad()
        loss = F.cross_entropy(self.forward(x), y)
        loss.backward()
        self.opt.step()
        return float(loss.detach())

    def grads(self) -> Dict[str, torch.Tensor]:
        return {k: v.grad for k, v in self.p.items()}


def time_cpu_step(state_dict, batch=128, warmup=3, steps=50, max_seconds=30.0, threads=None, seed=0):
    """Median step time of TorchCPUStep at `batch` (config 1: 128, fp32, 32x32): `warmup` untimed
    steps, then up to `steps` timed steps or `max_seconds`, whichever ends first (the bench keeps
    the CPU leg bounded). Returns dict(img_per_s, median_s, steps, threads, seconds)."""
    if threads:
        torch.set_num_threads(int(threads))
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch, 3, 32, 32, generator=g)
    y = torch.randint(0, 100, (batch,), generator=g)
    m = TorchCPUStep(state_dict)
    for _ in range(warmup):
        m.step(x, y)
    times = []
    t_all = time.perf_counter()
    while len(times) < steps and time.perf_counter() - t_all < max_seconds:
        t0 = time.perf_counter()
        m.step(x, y)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"img_per_s": batch / med, "median_s": med, "steps": len(times), "threads": torch.get_num_threads(),
            "seconds": time.perf_counter() - t_all}
