"""Throughput of the on-device CIFAR pipeline kernel (ops.cifar_augment) against HBM peak, and
of the DeviceLoader feeding the native training step. Prints one JSON line.

Algorithmic bytes per image: h*w*3 (uint8 read) + 3*h*w*4 (fp32 write) + 8 (index) + 2 (crop)
+ 1 (flip) + 8 (label read) + 8 (label write) = 15,395 B at 32x32."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dtc_import  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    dtc = dtc_import.load()
    dev = torch.device("cuda:0")
    imgs, tg = dtc.data.synthetic_cifar_u8()
    images = torch.from_numpy(imgs).to(dev)
    targets = torch.from_numpy(tg).to(dev)
    res = {}
    for B in (256, 4096, 45000):
        idx = torch.randint(0, images.shape[0], (B,), device=dev)
        crop = torch.randint(0, 9, (B, 2), dtype=torch.uint8, device=dev)
        flip = torch.randint(0, 2, (B,), dtype=torch.uint8, device=dev)
        out = torch.empty(B, 3, 32, 32, device=dev)
        lab = torch.empty(B, dtype=torch.int64, device=dev)
        args = (images, idx, crop, flip, dtc.data.CIFAR_MEAN, dtc.data.CIFAR_STD, 4)
        for _ in range(5):
            dtc.ops.cifar_augment(*args, targets=targets, out=out, labels=lab)
        iters = 200 if B < 10000 else 40
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            dtc.ops.cifar_augment(*args, targets=targets, out=out, labels=lab)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / iters * 1e3
        gbs = B * 15395 / (us * 1e-6) / 1e9
        res[str(B)] = {"us_per_launch": round(us, 2), "GB_s": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4),
                       "images_per_s": round(B / (us * 1e-6))}
    # DeviceLoader feeding the native train step (batch 256), vs resident synthetic input
    torch.manual_seed(42)
    model = dtc.ResNet18().to(dev)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    loader = dtc.data.DeviceLoader(imgs, tg, 256, device=dev)

    def run(batches):
        n = 0
        for x, y in batches:
            opt.zero_grad()
            loss = crit(model(x), y)
            loss.backward()
            opt.step()
            n += x.shape[0]
        return n

    run(b for _, b in zip(range(5), loader))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = run(b for _, b in zip(range(60), loader))
    torch.cuda.synchronize()
    fed = n / (time.perf_counter() - t0)
    x0, y0 = next(iter(loader))
    t0 = time.perf_counter()
    n = run((x0, y0) for _ in range(60))
    torch.cuda.synchronize()
    resident = n / (time.perf_counter() - t0)
    print(json.dumps({"kernel": "cifar_augment", "bytes_per_image": 15395, "peak_GB_s": HBM_PEAK_GBS, "by_batch": res,
                      "train_step_images_per_s": {"device_loader": round(fed, 1), "resident": round(resident, 1)}}),
          flush=True)


if __name__ == "__main__":
    main()
