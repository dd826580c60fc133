"""Time every distinct ResNet-18 conv (batch B) for fwd / dgrad / wgrad on the native kernels,
interleaving kernel-option variants in one process (guide §5.4 rule 24). Prints TFLOP/s
(algorithmic 2*N*P*Q*K*R*S*C) per pass and the per-step weighted total."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtc_import  # noqa: E402

# (name, H, C, K, R, stride, count per step)
LAYERS = [
    ("stem", 32, 64, 64, 1, 1, 1),
    ("l1", 32, 64, 64, 3, 1, 4),
    ("l2.0.c1", 32, 64, 128, 3, 2, 1),
    ("l2.sc", 32, 64, 128, 1, 2, 1),
    ("l2", 16, 128, 128, 3, 1, 3),
    ("l3.0.c1", 16, 128, 256, 3, 2, 1),
    ("l3.sc", 16, 128, 256, 1, 2, 1),
    ("l3", 8, 256, 256, 3, 1, 3),
    ("l4.0.c1", 8, 256, 512, 3, 2, 1),
    ("l4.sc", 8, 256, 512, 1, 2, 1),
    ("l4", 4, 512, 512, 3, 1, 3),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="igemm_stages=2;igemm_stages=3")
    args = ap.parse_args()
    dtc = dtc_import.load()
    ops = dtc.ops
    dev = torch.device("cuda:0")
    B = args.batch
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in args.variants.split(";")]
    results = {i: {} for i in range(len(variants))}
    for (name, H, C, K, R, st, cnt) in LAYERS:
        pad = 1 if R == 3 else 0
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        dy = torch.randn(B, P, P, K, device=dev).bfloat16()
        stats = ops.new_stats(K, dev)
        flops = 2.0 * B * P * P * K * R * R * C
        fns = {
            "fwd": lambda: ops.conv2d_fwd(x, w, st, pad, stats=stats),
            "dgrad": lambda: ops.conv2d_dgrad(dy, w, (H, H), st, pad),
            "wgrad": lambda: ops.conv2d_wgrad(x, dy, R, R, st, pad),
        }
        if name == "stem":
            fns.pop("dgrad")
        for rnd in range(3):  # interleaved rounds
            for vi, var in enumerate(variants):
                for k, v in var.items():
                    dtc._native.call("dtc_set_option", k.encode(), int(v))
                for pname, fn in fns.items():
                    fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / args.iters
                    key = (name, pname)
                    prev = results[vi].get(key)
                    results[vi][key] = (min(us, prev[0]) if prev else us, flops, cnt)
    for vi, var in enumerate(variants):
        print(f"=== variant {var}")
        tot_us, tot_fl = 0.0, 0.0
        for (name, pname), (us, fl, cnt) in results[vi].items():
            tot_us += us * cnt
            tot_fl += fl * cnt
            print(f"  {name:8s} {pname:6s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  x{cnt}")
        print(f"  TOTAL per step {tot_us:.1f} us  {tot_fl / tot_us / 1e6:.1f} TF/s")
        print(json.dumps({"variant": var, "step_conv_us": round(tot_us, 1), "tflops": round(tot_fl / tot_us / 1e6, 1)}))


if __name__ == "__main__":
    main()
