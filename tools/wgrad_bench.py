"""Time the batched 3x3 stride-1 weight gradients (dtc_conv2d_wgrad_batch: wgrad_halo + wgrad_reduce)
exactly as the executor issues them at batch B: layer1 four convs per launch, layers 2-4 three.

Each geometry's call is captured ITERS times into a CUDA graph (raw C-ABI calls, buffers
preallocated) and replayed, so the figure is device time. Option variants are interleaved in one
process. Prints us per launch and TFLOP/s (algorithmic 2*N*H*W*K*9*C per conv) per variant.

usage: python tools/wgrad_bench.py --variants "wgrad_xcd=0;wgrad_xcd=1" [--batch 256]"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtc_import  # noqa: E402

# (name, H, C, K, problems per launch)
GEOMS = [("l1", 32, 64, 64, 4), ("l2", 16, 128, 128, 3), ("l3", 8, 256, 256, 3), ("l4", 4, 512, 512, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="wgrad_batch=4")
    ap.add_argument("--layers", default="")
    ap.add_argument("--check", action="store_true", help="max |dw - dw(variant 0)| per geometry")
    args = ap.parse_args()
    dtc = dtc_import.load()
    ops, nat = dtc.ops, dtc._native
    dev = torch.device("cuda:0")
    B = args.batch
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in args.variants.split(";")]
    res = {i: {} for i in range(len(variants))}
    names = sorted({k for v in variants for k in v})
    defaults = {k: nat.lib.dtc_get_option(k.encode()) for k in names}  # restored before every variant
    g = torch.Generator(device=dev).manual_seed(0)
    for (name, H, Cc, K, n) in GEOMS:
        if args.layers and name not in args.layers.split(","):
            continue
        xs = [torch.randn(B, H, H, Cc, device=dev, generator=g).bfloat16() for _ in range(n)]
        dys = [torch.randn(B, H, H, K, device=dev, generator=g).bfloat16() for _ in range(n)]
        dws = [torch.empty(K, 3, 3, Cc, device=dev) for _ in range(n)]
        d = ops.conv_desc(B, H, H, Cc, K, 3, 3, 1, 1)
        arr = C.c_void_p * n
        xa, da, wa = arr(*[nat.ptr(t) for t in xs]), arr(*[nat.ptr(t) for t in dys]), arr(*[nat.ptr(t) for t in dws])
        flops = 2.0 * B * H * H * K * 9 * Cc * n
        ref = None
        for rnd in range(3):
            for vi, var in enumerate(variants):
                for k, v in {**defaults, **var}.items():
                    nat.call("dtc_set_option", k.encode(), int(v))
                nb = nat.lib.dtc_conv2d_wgrad_batch_workspace_size(d, n)
                ws = torch.empty(nb // 4 + 64, device=dev)

                def fn():
                    nat.call("dtc_conv2d_wgrad_batch", d, n, xa, da, wa, 1.0, nat.ptr(ws), nb, nat.stream_ptr())

                fn()
                torch.cuda.synchronize()
                if args.check and rnd == 0:
                    out = torch.cat([w.flatten() for w in dws])
                    if ref is None:
                        ref = out.clone()
                    else:
                        print(f"  check {name} {var}: max|diff| {float((out - ref).abs().max()):.3e}")
                gr = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(gr, stream=s):
                        for _ in range(args.iters):
                            fn()
                gr.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gr.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                prev = res[vi].get(name)
                res[vi][name] = (min(us, prev[0]) if prev else us, flops)
                del gr
    for vi, var in enumerate(variants):
        tot_us = sum(v[0] for v in res[vi].values())
        tot_fl = sum(v[1] for v in res[vi].values())
        print(f"=== variant {var}")
        for name, (us, fl) in res[vi].items():
            print(f"  {name}: {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  ({fl / us / 1e6 / 2500:.3f} of peak)")
        print(json.dumps({"variant": var, "wgrad_us": round(tot_us, 1), "tflops": round(tot_fl / tot_us / 1e6, 1),
                          "per_layer_us": {k: round(v[0], 1) for k, v in res[vi].items()}}))


if __name__ == "__main__":
    main()
