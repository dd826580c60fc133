"""Host-side phase timing of the bench step (no added syncs): where does the host wait?

Replicates bench.py's step and stamps time.perf_counter() after each phase; a phase that blocks
on the device (barrier, item) shows the GPU time it waited for, the others show pure host cost.
Usage: python tools/host_phases.py [--steps 50] [--batch 256] [--loopback W] [--no-barrier] [--cprofile]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
import dtc_import  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--no-barrier", action="store_true")
    ap.add_argument("--torch-barrier", action="store_true", help="dist.barrier() instead of bench.py's dtc.barrier()")
    ap.add_argument("--cprofile", action="store_true", help="cProfile the timed steps (top functions by tottime)")
    ap.add_argument("--loopback", type=int, default=0, help="one rank of a W-rank job: loopback communicator, 1/W")
    ap.add_argument("--spin", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) before init")
    args = ap.parse_args()
    if args.spin:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(1))
    rank, world, local = bench.init_dist(1)
    dev = torch.device("cuda", local)
    dtc = dtc_import.load()
    torch.manual_seed(42)
    model = dtc.DDP(dtc.ResNet18().to(dev), device_ids=[local], find_unused_parameters=True)
    if args.loopback > 1:  # as bench.py --sim-world W --sim-comm loopback
        model.module._comm = dtc.parallel.Comm.loopback(local, factor=1.0, world=args.loopback)
        model.module._grad_scale = 1.0 / args.loopback
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, weight_decay=1e-4, momentum=0.9, nesterov=True)
    scaler = dtc.GradScaler()
    tpl = dtc.data.class_templates(100, 32, 32)
    img, label = dtc.data.synthetic_batch(0, args.batch, 32, 32, 100, dev, tpl)
    names = ["zero_grad", "forward", "loss", "barrier", "scale", "backward", "step", "update", "item"]
    rec = []
    prof = None
    for i in range(args.steps + 10):
        if i == 10 and args.cprofile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t = [time.perf_counter()]
        opt.zero_grad()
        t.append(time.perf_counter())
        with dtc.autocast():
            logit = model(img)
            t.append(time.perf_counter())
            loss = crit(logit, label)
        t.append(time.perf_counter())
        if not args.no_barrier:
            if args.torch_barrier:
                dist.barrier()
            else:
                dtc.barrier()
        t.append(time.perf_counter())
        scaled = scaler.scale(loss)
        t.append(time.perf_counter())
        scaled.backward()
        t.append(time.perf_counter())
        scaler.step(opt)
        t.append(time.perf_counter())
        scaler.update()
        t.append(time.perf_counter())
        loss.item()
        t.append(time.perf_counter())
        if i >= 10:
            rec.append(np.diff(t) * 1e6)
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof).sort_stats("tottime").print_stats(30)
    r = np.array(rec)
    for k, n in enumerate(names):
        print(f"{n:10s} mean {r[:, k].mean():8.1f} us  median {np.median(r[:, k]):8.1f} us")
    print(f"{'total':10s} mean {r.sum(1).mean():8.1f} us")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
