"""Library calibration of the ResNet-18 convs: what MIOpen (torch conv2d, channels_last bf16) and
hipBLASLt (torch.matmul bf16 on pre-built im2col operands -- the GEMM alone, im2col not counted)
take for the same fwd / dgrad / wgrad as tools/conv_bench.py times on the native kernels.

Per (layer, pass) ITERS calls are captured into one CUDA graph and replayed (device time, as
conv_bench.py times the native kernels); a call that cannot be captured is timed eagerly (median
of ITERS event-bracketed launches, which includes host launch overhead -- marked "eager"). FLOPs are the algorithmic
2*N*P*Q*K*R*S*C. Prints one line per (layer, pass, library) and a JSON summary.
usage: python tools/lib_calib.py [--batch 256] [--libs miopen,blas] [--layers l2,l3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conv_bench import LAYERS  # noqa: E402


def timed(fn, iters):
    """Device time per call: ITERS calls captured into one CUDA graph and replayed (no host launch
    overhead, as tools/conv_bench.py); libraries whose calls cannot be captured are timed eagerly."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    try:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(iters):
                    fn()
        g.replay()
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / iters
            best = us if best is None else min(best, us)
        return best, "graph"
    except Exception:
        torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    v = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
    return v[len(v) // 2], "eager"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--libs", default="miopen,blas")
    ap.add_argument("--layers", default="")
    ap.add_argument("--find", action="store_true", help="torch.backends.cudnn.benchmark: MIOpen times its solutions")
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = args.find
    dev = torch.device("cuda:0")
    B = args.batch
    libs = args.libs.split(",")
    out = {}
    tot = {lib: [0.0, 0.0] for lib in libs}
    for (name, H, C, K, R, st, cnt) in LAYERS:
        if args.layers and name not in args.layers.split(","):
            continue
        pad = 1 if R == 3 else 0
        P = (H + 2 * pad - R) // st + 1
        flops = 2.0 * B * P * P * K * R * R * C
        x = torch.randn(B, C, H, H, device=dev).bfloat16().to(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).bfloat16().to(memory_format=torch.channels_last)
        dy = torch.randn(B, K, P, P, device=dev).bfloat16().to(memory_format=torch.channels_last)
        fns = {}
        if "miopen" in libs:
            fns[("fwd", "miopen")] = lambda: F.conv2d(x, w, None, st, pad)
            if name != "stem":
                fns[("dgrad", "miopen")] = lambda: torch.ops.aten.convolution_backward(
                    dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [True, False, False])
            fns[("wgrad", "miopen")] = lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])
        if "blas" in libs:
            M, Kd = B * P * P, R * R * C
            a = torch.randn(M, Kd, device=dev).bfloat16()        # im2col(x)
            bw = torch.randn(Kd, K, device=dev).bfloat16()        # weights
            fns[("fwd", "blas")] = lambda: torch.matmul(a, bw)
            if name != "stem":
                Md, Kdd = B * H * H, R * R * K
                ad = torch.randn(Md, Kdd, device=dev).bfloat16()  # im2col(dy) (stride-1 form)
                bd = torch.randn(Kdd, C, device=dev).bfloat16()
                fns[("dgrad", "blas")] = lambda: torch.matmul(ad, bd)
            dyt = torch.randn(K, M, device=dev).bfloat16()        # dy^T
            fns[("wgrad", "blas")] = lambda: torch.matmul(dyt, a)
        for (pname, lib), fn in fns.items():
            try:
                us, how = timed(fn, args.iters)
            except Exception as e:  # a library without a solution for this shape
                print(f"  skip {name} {pname} {lib}: {e}", flush=True)
                continue
            out.setdefault(name, {})[f"{pname}_{lib}_us"] = round(us, 1)
            tot[lib][0] += us * cnt
            tot[lib][1] += flops * cnt
            print(f"  {name:8s} {pname:6s} {lib:7s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  x{cnt}  ({how})", flush=True)
    for lib, (us, fl) in tot.items():
        if us:
            print(f"  TOTAL {lib} per step {us:.1f} us  {fl / us / 1e6:.1f} TF/s")
    print(json.dumps({"batch": B, "per_layer": out,
                      "step_us": {lib: round(v[0], 1) for lib, v in tot.items()}}))


if __name__ == "__main__":
    main()
