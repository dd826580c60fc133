"""Time every distinct ResNet-18 conv (batch B) for fwd / dgrad / wgrad on the native kernels.

Each (layer, pass) is captured ITERS times into a torch CUDA graph (buffers preallocated, raw
C-ABI calls), so the replay measures device time only, not Python/allocation overhead. Kernel-
option variants are interleaved in one process (guide §5.4 rule 24). Prints TFLOP/s
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
    ap.add_argument("--variants", default="halo_conv=1;halo_conv=0")
    ap.add_argument("--layers", default="")
    ap.add_argument("--scale", type=int, default=1, help="image side multiplier (7: the 224x224 model's layers)")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--fresh", action="store_true",
                    help="re-write each call's input right before it (as the BN kernel does in the training step) "
                         "and subtract the copy-only time: the conv reads a just-written input, not an L2-warm one")
    args = ap.parse_args()
    dtc = dtc_import.load()
    ops, nat = dtc.ops, dtc._native
    dev = torch.device("cuda:0")
    B = args.batch
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in args.variants.split(";")]
    # every variant starts from the library defaults of the options any variant names (no leaks)
    defaults = {k: nat.lib.dtc_get_option(k.encode()) for k in sorted({k for v in variants for k in v})}
    results = {i: {} for i in range(len(variants))}
    layers = [l for l in LAYERS if not args.layers or l[0] in args.layers.split(",")]
    passes = args.passes.split(",")
    for (name, H, C, K, R, st, cnt) in layers:
        H = H * args.scale
        pad = 1 if R == 3 else 0
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        dy = torch.randn(B, P, P, K, device=dev).bfloat16()
        y = torch.empty(B, P, P, K, device=dev).bfloat16()
        dx = torch.empty(B, H, H, C, device=dev).bfloat16()
        dw = torch.empty(K, R, R, C, device=dev)
        res = torch.randn(B, H, H, C, device=dev).bfloat16()
        stats = ops.new_stats(K, dev)
        d = ops.conv_desc(B, H, H, C, K, R, R, st, pad)
        wsb = max(nat.lib.dtc_conv2d_workspace_size(d, m) for m in range(3))
        ws = torch.empty(wsb // 4 + 64, device=dev)
        flops = 2.0 * B * P * P * K * R * R * C
        flops_of = {"fwdsc": flops * 10.0 / 9.0, "wgradsc": flops * 10.0 / 9.0}
        P_ = nat.ptr
        fns = {
            "fwd": lambda: nat.call("dtc_conv2d_fwd", d, P_(x), P_(w), P_(y), P_(stats), P_(ws), wsb, nat.stream_ptr()),
            "dgrad": lambda: nat.call("dtc_conv2d_dgrad", d, P_(dy), P_(w), P_(dx), None, P_(ws), wsb,
                                      nat.stream_ptr()),
            # dgrad + residual (identity blocks' conv1: the shortcut's gradient added in the epilogue)
            "dgradr": lambda: nat.call("dtc_conv2d_dgrad", d, P_(dy), P_(w), P_(dx), P_(res), P_(ws), wsb,
                                       nat.stream_ptr()),
            "wgrad": lambda: nat.call("dtc_conv2d_wgrad", d, P_(x), P_(dy), P_(dw), 1.0, P_(ws), wsb,
                                      nat.stream_ptr()),
        }
        if R == 3 and st == 2:  # + the block's 1x1 stride-2 shortcut in the same launch (dtc_conv2d_fwd_sc)
            wsc = (torch.randn(K, C, device=dev) * 0.05).bfloat16()
            ysc = torch.empty_like(y)
            stats2 = ops.new_stats(K, dev)
            fns["fwdsc"] = lambda: nat.call("dtc_conv2d_fwd_sc", d, P_(x), P_(w), P_(y), P_(stats), P_(wsc), P_(ysc),
                                            P_(stats2), nat.stream_ptr())
            dwsc = torch.empty(K, C, device=dev)
            dsc = torch.randn(B, P, P, K, device=dev).bfloat16()

            def wgradsc():
                nb = nat.lib.dtc_conv2d_wgrad_sc_workspace_size(d)
                if nb == 0 or nb > wsb:
                    raise RuntimeError("no fused wgrad plan / workspace")
                nat.call("dtc_conv2d_wgrad_sc", d, P_(x), P_(dy), P_(dsc), P_(dw), P_(dwsc), 1.0, P_(ws), wsb,
                         nat.stream_ptr())
            fns["wgradsc"] = wgradsc
        if name == "stem":
            fns.pop("dgrad")
            fns.pop("dgradr")
        fns = {k: v for k, v in fns.items() if k in passes}
        if args.fresh:
            xs, dys = x.clone(), dy.clone()
            copies = {"fwd": lambda: x.copy_(xs), "dgrad": lambda: dy.copy_(dys), "dgradr": lambda: dy.copy_(dys),
                      "wgrad": lambda: dy.copy_(dys)}
            fns = {k: (lambda f=f, c=copies[k]: (c(), f())) for k, f in fns.items()}
            fns.update({"copy_" + k: copies[k] for k in list(fns)})
        for rnd in range(3):  # interleaved rounds
            for vi, var in enumerate(variants):
                for k, v in {**defaults, **var}.items():
                    nat.call("dtc_set_option", k.encode(), int(v))
                need = max([nat.lib.dtc_conv2d_workspace_size(d, m) for m in range(3)] +
                           [nat.lib.dtc_conv2d_wgrad_sc_workspace_size(d)])  # the variant's plan
                if need > wsb:
                    wsb = need
                    ws = torch.empty(wsb // 4 + 64, device=dev)
                for pname, fn in fns.items():
                    try:
                        fn()
                    except Exception as e:  # no plan for this pass under this variant (e.g. fwdsc)
                        print(f"  skip {name} {pname} {var}: {e}")
                        continue
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
                    key = (name, pname)
                    prev = results[vi].get(key)
                    results[vi][key] = (min(us, prev[0]) if prev else us, flops_of.get(pname, flops), cnt)
                    del g
    for vi, var in enumerate(variants):
        print(f"=== variant {var}")
        tot_us, tot_fl = 0.0, 0.0
        for (name, pname), (us, fl, cnt) in list(results[vi].items()):
            if pname.startswith("copy_"):
                continue
            if (name, "copy_" + pname) in results[vi]:
                us -= results[vi][(name, "copy_" + pname)][0]
            tot_us += us * cnt
            tot_fl += fl * cnt
            print(f"  {name:8s} {pname:6s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  x{cnt}")
        print(f"  TOTAL per step {tot_us:.1f} us  {tot_fl / tot_us / 1e6:.1f} TF/s")
        print(json.dumps({"variant": var, "step_conv_us": round(tot_us, 1), "tflops": round(tot_fl / tot_us / 1e6, 1)}))


if __name__ == "__main__":
    main()
