"""In-process A/B of native option sets on bench.py's step (one rank, N=1): the option sets alternate
every block of K steps inside ONE process, so process-to-process variance (allocation layout, clocks
at start-up) cancels out of the paired differences. Prints per-set median img/s and the median paired
difference of every set against the first.

usage: python tools/inproc_ab.py [--rounds 12] [--steps 60] [--batch 256] "tag|name=v,name=v" ...
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import dtc_import  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=3, help="untimed steps after every option switch")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--sim-world", type=int, default=1,
                    help="one rank of a W-rank job (bench.py --sim-world): 1/W pre-scale, bucket all-reduces "
                         "through the one-rank RCCL communicator")
    ap.add_argument("sets", nargs="+")
    args = ap.parse_args()
    rank, world, local = bench.init_dist(1)
    dev = torch.device("cuda", local)
    dtc = dtc_import.load()
    sets = []
    for spec in args.sets:
        tag, _, opts = spec.partition("|")
        kv = [o.split("=") for o in opts.split(",") if o]
        sets.append((tag, [(k.encode(), int(v)) for k, v in kv]))
    names = {k for _, kv in sets for k, _ in kv}
    defaults = {k: int(dtc._native.lib.dtc_get_option(k)) for k in names}

    torch.manual_seed(42)
    model = dtc.DDP(dtc.ResNet18().to(dev), device_ids=[local], find_unused_parameters=True, bucket_cap_mb=25.0)
    if args.sim_world > 1:
        model.module._comm = model.comm
        model.module._grad_scale = 1.0 / args.sim_world
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
    scaler = dtc.GradScaler()
    B = args.batch
    templates = dtc.data.class_templates(100, 32, 32)
    pool = [dtc.data.synthetic_batch(i, B, 32, 32, 100, dev, templates) for i in range(4)]

    def step(i):
        img, label = pool[i % 4]
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(model(img), label)
        dtc.barrier()
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        loss.item()

    for i in range(10):
        step(i)
    res = {tag: [] for tag, _ in sets}
    it = 0
    for r in range(args.rounds):
        order = sets if r % 2 == 0 else sets[::-1]  # alternate the order: no set always follows another
        for tag, kv in order:
            for k in names:
                dtc._native.call("dtc_set_option", k, defaults[k])
            for k, v in kv:
                dtc._native.call("dtc_set_option", k, v)
            for _ in range(args.warmup):
                step(it)
                it += 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(it)
                it += 1
            torch.cuda.synchronize()
            res[tag].append(B * args.steps / (time.perf_counter() - t0))
        print("round", r, " ".join(f"{t}={res[t][-1]:.0f}" for t, _ in sets), flush=True)
    base = sets[0][0]
    for tag, _ in sets:
        d = [a / b - 1.0 for a, b in zip(res[tag], res[base])]
        print(f"{tag:>12s} median {statistics.median(res[tag]):9.0f} img/s  vs {base}: median {100 * statistics.median(d):+.2f}%"
              f"  mean {100 * statistics.mean(d):+.2f}%  (+{sum(x > 0 for x in d)}/-{sum(x < 0 for x in d)})", flush=True)


if __name__ == "__main__":
    main()
