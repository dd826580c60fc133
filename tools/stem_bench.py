"""Time the stem paths at the config-2 shape (B=256, 32x32): the direct stem conv (stem.hip) forward
with and without BN statistics and its weight gradient, against im2col + 1x1 implicit GEMM.
CUDA-graph replay of ITERS calls per measurement (device time only)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dtc_import  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def _with_opt(nat, name, val, fn):
    old = nat.lib.dtc_get_option(name.encode())
    nat.lib.dtc_set_option(name.encode(), val)
    try:
        return fn()
    finally:
        nat.lib.dtc_set_option(name.encode(), old)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dtc = dtc_import.load()
    ops, nat = dtc.ops, dtc._native
    dev = torch.device("cuda:0")
    B, S = a.batch, a.size
    x = torch.randn(B, 3, S, S, device=dev)
    w27 = (torch.randn(64, 27, device=dev) * 0.2).bfloat16()
    y = torch.empty(B, S, S, 64, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(B, S, S, 64, device=dev).bfloat16()
    stats = ops.new_stats(64, dev)
    dw = torch.empty(64, 27, device=dev)
    nb = nat.lib.dtc_stem_wgrad_workspace_size(B, S, S)
    ws = torch.empty(nb // 4 + 64, device=dev)
    P = nat.ptr
    res = {
        "stem_fwd+stats": timeit(lambda: nat.call("dtc_stem_fwd", P(x), P(w27), P(y), P(stats), B, S, S,
                                                  nat.stream_ptr()), a.iters),
        "stem_fwd": timeit(lambda: nat.call("dtc_stem_fwd", P(x), P(w27), P(y), None, B, S, S, nat.stream_ptr()),
                           a.iters),
        "stem_fwd+stats (wlds)": _with_opt(nat, "stem_wlds", 1, lambda: timeit(
            lambda: nat.call("dtc_stem_fwd", P(x), P(w27), P(y), P(stats), B, S, S, nat.stream_ptr()), a.iters)),
        "stem_wgrad(+reduce)": timeit(lambda: nat.call("dtc_stem_wgrad", P(x), P(dy), P(dw), 1.0, B, S, S, P(ws), nb,
                                                       nat.stream_ptr()), a.iters),
        "copy_y_33MB": timeit(lambda: y.copy_(dy), a.iters),
    }
    cols = torch.empty(B, S, S, 64, device=dev, dtype=torch.bfloat16)
    res["im2col"] = timeit(lambda: nat.call("dtc_stem_im2col", P(x), P(cols), B, S, S, nat.stream_ptr()), a.iters)
    for k, v in res.items():
        print(f"{k:24s} {v:8.2f} us")


if __name__ == "__main__":
    main()
