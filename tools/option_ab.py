"""Bit-exactness of kernel-option variants: every distinct ResNet-18 conv (fwd / dgrad / wgrad) run
under each variant on the same random operands; variants that only change scheduling (ring depths,
tile walks) must give identical outputs. Prints the max |difference| per (layer, pass) vs variant 0
and exits non-zero if any differs.

usage: python tools/option_ab.py --variants "wgrad_xcd=0;wgrad_xcd=1" [--batch 64]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtc_import  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--variants", required=True)
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    args = ap.parse_args()
    dtc = dtc_import.load()
    ops, nat = dtc.ops, dtc._native
    dev = torch.device("cuda:0")
    B = args.batch
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in args.variants.split(";")]
    # every variant starts from the library defaults of the options any variant names (no leaks)
    defaults = {k: nat.lib.dtc_get_option(k.encode()) for k in sorted({k for v in variants for k in v})}
    bad = 0
    g = torch.Generator(device=dev).manual_seed(0)
    for (name, H, C, K, R, st, _) in LAYERS:
        pad = 1 if R == 3 else 0
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(B, H, H, C, device=dev, generator=g).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev, generator=g) * 0.05).bfloat16()
        dy = torch.randn(B, P, P, K, device=dev, generator=g).bfloat16()
        d = ops.conv_desc(B, H, H, C, K, R, R, st, pad)
        outs = []
        for var in variants:
            for k, v in {**defaults, **var}.items():
                nat.call("dtc_set_option", k.encode(), int(v))
            wsb = max(nat.lib.dtc_conv2d_workspace_size(d, m) for m in range(3))
            ws = torch.empty(wsb // 4 + 64, device=dev)
            y = torch.zeros(B, P, P, K, device=dev).bfloat16()
            dx = torch.zeros(B, H, H, C, device=dev).bfloat16()
            dw = torch.zeros(K, R, R, C, device=dev)
            stats = ops.new_stats(K, dev)
            P_ = nat.ptr
            res = {}
            if "fwd" in args.passes:
                nat.call("dtc_conv2d_fwd", d, P_(x), P_(w), P_(y), P_(stats), P_(ws), wsb, nat.stream_ptr())
                res["fwd"] = y
            if "dgrad" in args.passes and name != "stem":
                nat.call("dtc_conv2d_dgrad", d, P_(dy), P_(w), P_(dx), None, P_(ws), wsb, nat.stream_ptr())
                res["dgrad"] = dx
            if "wgrad" in args.passes:
                nat.call("dtc_conv2d_wgrad", d, P_(x), P_(dy), P_(dw), 1.0, P_(ws), wsb, nat.stream_ptr())
                res["wgrad"] = dw
            torch.cuda.synchronize()
            outs.append(res)
        for pname, ref in outs[0].items():
            for vi in range(1, len(outs)):
                diff = (outs[vi][pname].float() - ref.float()).abs().max().item()
                flag = "" if diff == 0 else "  <-- DIFFERS"
                bad += diff != 0
                print(f"{name:8s} {pname:6s} variant {vi}: max|diff| {diff:.3e}{flag}")
    for k in variants[0]:
        pass
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
