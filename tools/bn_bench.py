"""Device time of the BN-backward reduction (dtc_bn_bwd_reduce: dy, x -> per-channel fp64 sums; with --mask
also the ReLU-masked dz store) at ResNet-18's BN shapes, for bn_red_unroll variants interleaved in one process.

Each call's raw pointers are captured ITERS times into a CUDA graph (no allocation or launch overhead in the
replay). Prints us and achieved GB/s (algorithmic bytes: 2 B of dy + 2 B of x per element, + 2 B of y and 2 B
of dz with --mask). usage: python tools/bn_bench.py [--variants 'bn_red_unroll=1;bn_red_unroll=4'] [--big]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtc_import  # noqa: E402

# (name, rows M at batch 256 / 32x32, C)
SHAPES = [("l1", 262144, 64), ("l2", 65536, 128), ("l3", 16384, 256), ("l4", 4096, 512)]
# the 224x224 model at batch 512 (layer1 / layer2)
BIG = [("l1@224", 25690112, 64), ("l2@224", 6422528, 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="bn_red_unroll=1;bn_red_unroll=4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mask", action="store_true")
    ap.add_argument("--big", action="store_true", help="also the 224x224 model's layer1/2 sizes (GBs per tensor)")
    args = ap.parse_args()
    dtc = dtc_import.load()
    nat = dtc._native
    dev = torch.device("cuda:0")
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in args.variants.split(";")]
    defaults = {k: nat.lib.dtc_get_option(k.encode()) for k in sorted({k for v in variants for k in v})}
    for name, M, C in SHAPES + (BIG if args.big else []):
        dy = torch.randn(M, C, device=dev).bfloat16()
        x = torch.randn(M, C, device=dev).bfloat16()
        ym = torch.randn(M, C, device=dev).bfloat16() if args.mask else None
        dz = torch.empty_like(dy) if args.mask else None
        mean = torch.zeros(C, device=dev)
        inv = torch.ones(C, device=dev)
        acc = dtc.ops.new_stats(C, dev)
        P = nat.ptr
        nbytes = M * C * (8 if args.mask else 4)

        def fn():
            nat.call("dtc_bn_bwd_reduce", P(dy), P(ym), P(x), P(mean), P(inv), P(acc), None, None, None, None, P(dz),
                     M, C, nat.stream_ptr())
        res = {}
        for rnd in range(3):
            for vi, var in enumerate(variants):
                for k, v in {**defaults, **var}.items():
                    nat.call("dtc_set_option", k.encode(), int(v))
                fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for _ in range(args.iters):
                            fn()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
                res[vi] = min(us, res.get(vi, us))
                del g
        for vi, var in enumerate(variants):
            us = res[vi]
            print(f"  {name:7s} M={M:9d} C={C:3d} {var}: {us:9.1f} us  {nbytes / us / 1e3:7.1f} GB/s", flush=True)
        del dy, x, ym, dz
        torch.cuda.empty_cache()
    for k, v in defaults.items():
        nat.call("dtc_set_option", k.encode(), int(v))


if __name__ == "__main__":
    main()
