"""Generate the golden vectors in tests/golden/ from the REFERENCE's own code.

Run in the build container only (it imports /root/reference, which does not exist on the GPU
box):  python tests/golden/make_golden.py

What it runs (reference = youngerous/distributed-training-comparison @ /root/reference):
  * src/ddp/utils.py fix_seed and src/ddp/dataset.py get_trn_val_loader (torchvision is not
    installed here, so a stub module provides `datasets.CIFAR100` of the right length and identity
    transforms — only indices are used), world-1 gloo process group for its DistributedSampler;
    torch's DistributedSampler (the reference's dependency) for W = 2, 4, 8.
  * src/single/net.py ResNet18 under fix_seed(42): initial-parameter checksums, forward/backward
    at batch 2 in fp32 and under CPU bf16 autocast (the build's AMP dtype), summarised as norms and
    sampled elements per tensor, plus per-module output summaries.
  * torch.optim.SGD(nesterov) and torch.amp.GradScaler sequences for the optimizer/AMP kernels.
  * a 200-step fp32 loss curve of the reference net + SGD recipe on the seeded synthetic stream.
  * src/ddp DDP semantics on 2 gloo ranks: all-reduced gradients vs the per-rank local gradients.
Fixtures hold numbers only — no reference source is copied.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src"
SAMPLES = 32


def _hash_list(xs):
    return hashlib.sha256(np.asarray(xs, dtype=np.int64).tobytes()).hexdigest()


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    ds = types.ModuleType("torchvision.datasets")
    tf = types.ModuleType("torchvision.transforms")

    class CIFAR100(torch.utils.data.Dataset):
        def __init__(self, root, train=True, download=False, transform=None):
            self.n = 50000 if train else 10000

        def __len__(self):
            return self.n

        def __getitem__(self, i):
            return torch.zeros(3, 32, 32), 0

    class _Id:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    ds.CIFAR100 = CIFAR100
    for name in ("Compose", "Normalize", "ToTensor", "RandomCrop", "RandomHorizontalFlip"):
        setattr(tf, name, _Id)
    tv.datasets, tv.transforms = ds, tf
    sys.modules.update({"torchvision": tv, "torchvision.datasets": ds, "torchvision.transforms": tf})


def _import_from(variant, module):
    path = os.path.join(REF, variant)
    sys.path.insert(0, path)
    try:
        for m in ("net", "utils", "dataset", "config"):
            sys.modules.pop(m, None)
        return __import__(module)
    finally:
        sys.path.remove(path)


# ----------------------------------------------------------------------------- sampler
def gen_sampler():
    import torch.distributed as dist

    _stub_torchvision()
    utils = _import_from("ddp", "utils")
    dataset = _import_from("ddp", "dataset")
    net = _import_from("ddp", "net")
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", rank=0, world_size=1)
    utils.fix_seed(42)
    net.ResNet18()  # ddp/main.py builds the model before the loaders (consumes torch RNG only)
    train_loader, train_sampler, valid_loader = dataset.get_trn_val_loader(
        data_dir="data/", batch_size=256, valid_size=0.1, num_workers=0, pin_memory=False)
    train_idx = list(train_loader.dataset.indices)
    valid_idx = list(valid_loader.dataset.indices)
    out = {"train_len": len(train_idx), "valid_len": len(valid_idx), "train_head": train_idx[:16],
           "valid_head": valid_idx[:16], "train_sha256": _hash_list(train_idx), "valid_sha256": _hash_list(valid_idx),
           "shards": {}}
    from torch.utils.data.distributed import DistributedSampler
    for W in (1, 2, 4, 8):
        for epoch in range(3):
            for r in range(W):
                if W == 1:
                    s = train_sampler
                else:
                    s = DistributedSampler(train_loader.dataset, num_replicas=W, rank=r)
                s.set_epoch(epoch)
                idx = list(iter(s))
                out["shards"][f"W{W}_e{epoch}_r{r}"] = {"len": len(idx), "head": idx[:8], "sha256": _hash_list(idx)}
    out["steps_per_epoch_global256"] = {str(W): len(train_idx) // W // (256 // W) for W in (1, 2, 4, 8)}
    dist.destroy_process_group()
    with open(os.path.join(HERE, "sampler.json"), "w") as f:
        json.dump(out, f, indent=1)


# ----------------------------------------------------------------------------- network
def _sample_idx(name, numel):
    seed = int(hashlib.md5(name.encode()).hexdigest()[:8], 16)
    return np.sort(np.random.default_rng(seed).choice(numel, size=min(SAMPLES, numel), replace=False))


def _summ(name, t):
    a = t.detach().float().reshape(-1).numpy().astype(np.float64)
    idx = _sample_idx(name, a.size)
    return {"norm": float(np.linalg.norm(a)), "sum": float(a.sum()), "idx": idx.tolist(),
            "val": a[idx].astype(np.float32).tolist()}


def gen_network():
    utils = _import_from("single", "utils")
    net = _import_from("single", "net")
    out = {}
    utils.fix_seed(42)
    model = net.ResNet18()
    out["init"] = {k: _summ(k, v) for k, v in model.state_dict().items() if v.dtype.is_floating_point}
    g = np.random.default_rng(0)
    x = g.standard_normal((2, 3, 32, 32)).astype(np.float32)
    y = g.integers(0, 100, 2)
    out["input"] = {"x_seed": 0, "batch": 2}
    for mode in ("fp32", "bf16"):
        utils.fix_seed(42)
        m = net.ResNet18()
        acts = {}
        hooks = []
        for name, mod in m.named_modules():
            if isinstance(mod, (torch.nn.Conv2d, torch.nn.BatchNorm2d, net.BasicBlock)):
                hooks.append(mod.register_forward_hook(
                    lambda mod, inp, o, name=name: acts.__setitem__(name, o.detach().clone())))
        ctx = torch.autocast("cpu", dtype=torch.bfloat16) if mode == "bf16" else torch.autocast("cpu", enabled=False)
        with ctx:
            logits = m(torch.from_numpy(x))
            loss = torch.nn.CrossEntropyLoss()(logits, torch.from_numpy(y))
        loss.backward()
        for h in hooks:
            h.remove()
        out[mode] = {
            "loss": float(loss),
            "logits": logits.detach().float().numpy().tolist(),
            "grads": {k: _summ(k, p.grad) for k, p in m.named_parameters()},
            "acts": {k: _summ(k, v.float().permute(0, 2, 3, 1).contiguous()) for k, v in acts.items()},
            "running": {k: _summ(k, v) for k, v in m.state_dict().items() if "running" in k},
        }
    with open(os.path.join(HERE, "resnet18_b2.json"), "w") as f:
        json.dump(out, f)


# ----------------------------------------------------------------------------- optimizer / amp
def gen_optim():
    g = np.random.default_rng(11)
    p0 = g.standard_normal(64).astype(np.float32)
    grads = [g.standard_normal(64).astype(np.float32) for _ in range(3)]
    p = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    opt = torch.optim.SGD([p], lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)  # trainer.py:92-98
    traj = []
    for gr in grads:
        p.grad = torch.from_numpy(gr.copy())
        opt.step()
        traj.append(p.detach().numpy().copy().tolist())
    scaler = torch.amp.GradScaler("cpu", init_scale=2.0 ** 16, growth_interval=3)
    q = torch.nn.Parameter(torch.ones(4))
    o2 = torch.optim.SGD([q], lr=0.1)
    pattern = [False, True, False, False, False, True, False, False, False, False]
    scales = []
    for bad in pattern:
        loss = (q * q).sum()
        scaler.scale(loss).backward()
        if bad:
            q.grad[0] = float("inf")
        scaler.step(o2)
        scaler.update()
        o2.zero_grad()
        scales.append(scaler.get_scale())
    out = {"sgd": {"p0": p0.tolist(), "grads": [x.tolist() for x in grads], "traj": traj, "lr": 0.1, "mu": 0.9,
                   "wd": 1e-4},
           "scaler": {"init": 2.0 ** 16, "interval": 3, "pattern": pattern, "scales": scales,
                      "q_final": q.detach().numpy().tolist()}}
    with open(os.path.join(HERE, "optim.json"), "w") as f:
        json.dump(out, f, indent=1)


# ----------------------------------------------------------------------------- loss curve
def synthetic_stream(step, batch, seed=1234, templates=None):
    """SURVEY §8(d) stream (restated here so the fixture does not depend on product code):
    labels randint(seed+step), x = 0.5*T[y] + randn, T = randn(100,3,32,32) under seed."""
    if templates is None:
        templates = torch.randn(100, 3, 32, 32, generator=torch.Generator().manual_seed(seed))
    gen = torch.Generator().manual_seed(seed + step)
    y = torch.randint(0, 100, (batch,), generator=gen)
    x = 0.5 * templates[y] + torch.randn(batch, 3, 32, 32, generator=gen)
    return x, y


def _perturb_ulp(model, seed):
    """Multiply every float parameter by (1 +- 2^-23): a 1-ulp perturbation of the seed-42 init,
    to measure how far two numerically equivalent runs of the same recipe drift apart."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for prm in model.parameters():
            sign = torch.randint(0, 2, prm.shape, generator=g).float() * 2 - 1
            prm.mul_(1 + sign * 2.0 ** -23)


def gen_loss_chaos(steps=200, batch=128, seeds=tuple(range(1, 100))):
    """Reference bf16-autocast curves from 1-ulp-perturbed inits (loss_curve.json: bf16_ulp[seed-1]);
    seeds already present in the fixture are kept, not recomputed. 99 perturbed + the seed-42 curve
    = 100 per side: the 200-step means spread 2.4% (s.d.), so 3 s.e. of the difference of two
    100-curve ensemble means is 1.0% -- the size at which north_star's 1% becomes resolvable."""
    utils = _import_from("single", "utils")
    net = _import_from("single", "net")
    templates = torch.randn(100, 3, 32, 32, generator=torch.Generator().manual_seed(1234))
    path = os.path.join(HERE, "loss_curve.json")
    out = json.load(open(path))
    curves = list(out.get("bf16_ulp", []))
    for sd in seeds[len(curves):]:
        utils.fix_seed(42)
        m = net.ResNet18()
        _perturb_ulp(m, sd)
        opt = torch.optim.SGD(m.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
        crit = torch.nn.CrossEntropyLoss()
        losses = []
        for s in range(steps):
            x, y = synthetic_stream(s, batch, templates=templates)
            opt.zero_grad()
            with torch.autocast("cpu", dtype=torch.bfloat16):
                loss = crit(m(x), y)
            loss.backward()
            opt.step()
            losses.append(float(loss.detach()))
        curves.append(losses)
        print("ulp seed", sd, losses[:3], sum(losses) / len(losses), flush=True)
        out["bf16_ulp"] = curves
        with open(path, "w") as f:  # checkpoint after every run
            json.dump(out, f)


def gen_loss_curve(steps=200, batch=128, modes=("fp32", "bf16")):
    utils = _import_from("single", "utils")
    net = _import_from("single", "net")
    templates = torch.randn(100, 3, 32, 32, generator=torch.Generator().manual_seed(1234))
    out = {"batch": batch, "steps": steps, "lr": 0.1, "momentum": 0.9, "wd": 1e-4, "nesterov": True}
    x0, y0 = synthetic_stream(0, batch, templates=templates)
    out["stream_check"] = {"y0": y0.tolist()[:16], "x0_sum": float(x0.sum()), "x0_00": x0[0, 0, 0, :8].tolist()}
    torch.set_num_threads(os.cpu_count() or 8)
    for mode in modes:
        utils.fix_seed(42)
        m = net.ResNet18()
        opt = torch.optim.SGD(m.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
        crit = torch.nn.CrossEntropyLoss()
        losses = []
        for s in range(steps):
            x, y = synthetic_stream(s, batch, templates=templates)
            opt.zero_grad()
            ctx = torch.autocast("cpu", dtype=torch.bfloat16) if mode == "bf16" else torch.autocast("cpu", enabled=False)
            with ctx:
                loss = crit(m(x), y)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        out[mode] = losses
        print(mode, losses[:3], losses[-3:], flush=True)
    with open(os.path.join(HERE, "loss_curve.json"), "w") as f:
        json.dump(out, f)


# ----------------------------------------------------------------------------- 2-rank DDP
def _ddp_worker(rank, world, port, q):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    utils = _import_from("ddp", "utils")
    net = _import_from("ddp", "net")
    utils.fix_seed(42)  # ddp/main.py:16 — identical seed on every rank
    model = net.ResNet18()
    local = net.ResNet18()
    local.load_state_dict(model.state_dict())
    ddp = DDP(model, find_unused_parameters=True)  # trainer.py:31 (CPU modules take no device_ids)
    g = np.random.default_rng(100 + rank)
    x = torch.from_numpy(g.standard_normal((2, 3, 32, 32)).astype(np.float32))
    y = torch.from_numpy(g.integers(0, 100, 2))
    crit = torch.nn.CrossEntropyLoss()
    crit(ddp(x), y).backward()
    crit(local(x), y).backward()
    res = {"ddp": {k: _summ(k, p.grad) for k, p in ddp.module.named_parameters()},
           "local": {k: _summ(k, p.grad) for k, p in local.named_parameters()}}
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def gen_ddp():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, 29611, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get() for _ in procs)
    for p in procs:
        p.join()
    with open(os.path.join(HERE, "ddp_2rank.json"), "w") as f:
        json.dump({"world": 2, "per_rank": {str(k): v for k, v in res.items()}}, f)


if __name__ == "__main__":
    which = sys.argv[1:] or ["sampler", "network", "optim", "ddp", "loss"]
    torch.set_num_threads(os.cpu_count() or 8)
    if "sampler" in which:
        gen_sampler()
    if "network" in which:
        gen_network()
    if "optim" in which:
        gen_optim()
    if "ddp" in which:
        gen_ddp()
    if "loss" in which:
        gen_loss_curve()
    if "loss" in which or "loss_chaos" in which:
        gen_loss_chaos()
