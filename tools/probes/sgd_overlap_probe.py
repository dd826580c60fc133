"""Upper-bound probe: how much of the optimizer step can hide under the NEXT step's forward?

The fused SGD (22 B per parameter, HBM-bound) runs alone on the GPU after the backward. Layer4 + fc hold
~76% of the parameters and the forward reads them last, so their update could run beside the forward of
stem..layer3. This probe measures the bound WITHOUT the forward's join (the update may land after the forward
read the weights -- wrong numerics, timing only). The flat layout is bucket order (fc, layer4, ..., stem),
so "tail" = every parameter from the first layer4 offset on = 99.5% of the update (r06bb): an upper bound
for any split, since the whole SGD runs beside the forward and nothing waits for it:
  base  scaler.step(opt) as bench.py
  split head (params before layer4) and tail as two launches on the caller stream
  ovl   head on the caller stream, tail on a low-priority side stream forked after the head, never joined
Option sets alternate in one process (as tools/inproc_ab.py).
usage: python tools/probes/sgd_overlap_probe.py [--batch 256] [--rounds 8] [--steps 40] [--sim-world W]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import dtc_import  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--sim-world", type=int, default=1)
    args = ap.parse_args()
    rank, world, local = bench.init_dist(1)
    dev = torch.device("cuda", local)
    dtc = dtc_import.load()
    from importlib import import_module
    ops = import_module(dtc.__name__ + ".ops")
    torch.manual_seed(42)
    model = dtc.DDP(dtc.ResNet18().to(dev), device_ids=[local], find_unused_parameters=True, bucket_cap_mb=25.0)
    if args.sim_world > 1:
        model.module._comm = dtc.parallel.Comm.loopback(local, factor=1.0, world=args.sim_world)
        model.module._grad_scale = 1.0 / args.sim_world
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
    scaler = dtc.GradScaler()
    B = args.batch
    templates = dtc.data.class_templates(100, 32, 32)
    pool = [dtc.data.synthetic_batch(i, B, 32, 32, 100, dev, templates) for i in range(4)]
    flat = model.module.flat
    split = min(p.offset for p in flat.layout.params if p.name.startswith("layer4."))
    split -= split % 4
    n = flat.params.numel()
    print(f"params {n}, layer4+fc from {split} ({100.0 * (n - split) / n:.1f}%)", flush=True)
    side = torch.cuda.Stream(dev, priority=0)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, 0)
    side_lo = torch.cuda.Stream(dev, priority=lo)

    def sgd_range(a, b):
        g = opt.param_groups[0]
        ops.sgd_nesterov_flat(flat.params[a:b], flat.grads[a:b], opt._mom[a:b], flat.params_bf16[a:b], g["lr"],
                              g["weight_decay"], g["momentum"], scaler._inv_scale, scaler._found_inf)

    def step(i, mode):
        img, label = pool[i % 4]
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(model(img), label)
        dtc.barrier()
        scaler.scale(loss).backward()
        if mode == "base":
            scaler.step(opt)
        else:
            scaler.unscale_(opt)
            sgd_range(0, split)
            if mode == "split":
                sgd_range(split, n)
            else:
                s = side if mode == "ovl" else side_lo
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    sgd_range(split, n)
        scaler.update()
        loss.item()

    opt.step()  # attach the flat buffers
    modes = ["base", "split", "ovl", "ovl_lo"]
    for i in range(10):
        step(i, "base")
    res = {m: [] for m in modes}
    it = 0
    for r in range(args.rounds):
        for m in (modes if r % 2 == 0 else modes[::-1]):
            for _ in range(3):
                step(it, m)
                it += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(it, m)
                it += 1
            torch.cuda.synchronize()
            res[m].append(B * args.steps / (time.perf_counter() - t0))
        print("round", r, " ".join(f"{m}={res[m][-1]:.0f}" for m in modes), flush=True)
    for m in modes:
        d = [a / b - 1.0 for a, b in zip(res[m], res["base"])]
        print(f"B={B} sim={args.sim_world} {m:>7s} median {statistics.median(res[m]):9.0f} img/s  vs base: median "
              f"{100 * statistics.median(d):+.2f}%  (+{sum(x > 0 for x in d)}/-{sum(x < 0 for x in d)})", flush=True)


if __name__ == "__main__":
    main()
