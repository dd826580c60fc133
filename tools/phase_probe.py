"""Phase probe of one conv launch (diagnostics): per-workgroup timestamps at the kernel's marked points.

Needs the diagnostic library (`make -C distributed-training-comparison_amd/csrc phases`); the marks
(tile_common.h phase_mark) are compiled only there. conv_halo marks: 0 entry, 1 first step's operands
landed (prologue), 2 second reduction chunk's first step (chunk 0 + halo reload), 3 main loop done,
4 exit (epilogue). Prints the kernel span, the dispatch spread, per-phase percentiles and how many
workgroups are resident / in each phase over time (s_memrealtime: 100 MHz, chip-wide)."""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
os.environ.setdefault("DTC_LIB", os.path.join(ROOT, "distributed-training-comparison_amd", "_lib",
                                              "libdtc_amd_phases.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dtc_import  # noqa: E402

LAYERS = {"l2": (16, 128, 128), "l3": (8, 256, 256), "l4": (4, 512, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="l2,l3")
    ap.add_argument("--passes", default="fwd,dgrad")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--opts", default="", help="k=v,... options set before the runs")
    args = ap.parse_args()
    dtc = dtc_import.load()
    nat, ops = dtc._native, dtc.ops
    if not hasattr(nat.lib, "dtc_probe_phase_buffer"):
        raise SystemExit("not the phase-probe library (make phases): " + os.environ["DTC_LIB"])
    for kv in filter(None, args.opts.split(",")):
        k, v = kv.split("=")
        nat.call("dtc_set_option", k.encode(), int(v))
    dev = torch.device("cuda:0")
    buf = torch.zeros(16384 * 8, dtype=torch.int64, device=dev)
    fn_set = nat.lib.dtc_probe_phase_buffer
    fn_set.argtypes = [ctypes.c_void_p]  # (a bare Python int would pass as a 32-bit C int)
    fn_set.restype = ctypes.c_int
    fn_set(ctypes.c_void_p(buf.data_ptr()))
    B = args.batch
    P_ = nat.ptr
    for lname in args.layers.split(","):
        H, C, K = LAYERS[lname]
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).bfloat16()
        y = torch.empty(B, H, H, K, device=dev).bfloat16()
        dy = torch.randn(B, H, H, K, device=dev).bfloat16()
        dx = torch.empty(B, H, H, C, device=dev).bfloat16()
        stats = ops.new_stats(K, dev)
        d = ops.conv_desc(B, H, H, C, K, 3, 3, 1, 1)
        wsb = max(nat.lib.dtc_conv2d_workspace_size(d, m) for m in range(3))
        ws = torch.empty(wsb // 4 + 64, device=dev)
        fns = {"fwd": lambda: nat.call("dtc_conv2d_fwd", d, P_(x), P_(w), P_(y), P_(stats), P_(ws), wsb,
                                       nat.stream_ptr()),
               "dgrad": lambda: nat.call("dtc_conv2d_dgrad", d, P_(dy), P_(w), P_(dx), None, P_(ws), wsb,
                                         nat.stream_ptr())}
        for pname in args.passes.split(","):
            fn = fns[pname]
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            buf.zero_()
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            fn()
            ev1.record()
            torch.cuda.synchronize()
            t = buf.view(16384, 8).cpu().numpy()[:, :5].astype(np.float64)
            t = t[t[:, 0] > 0]
            if len(t) == 0:
                print(f"{lname} {pname}: no marks (not a conv_halo launch?)")
                continue
            base = t[:, 0].min()
            t = (t - base) / 100.0  # us
            t[t < 0] = np.nan
            span = np.nanmax(t[:, 4])
            print(f"=== {lname} {pname} B={B}: {len(t)} workgroups, span {span:.2f} us (events {ev0.elapsed_time(ev1) * 1e3:.2f} us)")
            q = lambda a: " ".join(f"{v:6.2f}" for v in np.nanpercentile(a, [0, 10, 50, 90, 100]))  # noqa: E731
            print(f"  start      (p0 p10 p50 p90 p100) {q(t[:, 0])}")
            names = ["prologue", "chunk0+reload", "rest", "epilogue"]
            for i, nm in enumerate(names):
                print(f"  {nm:14s}                     {q(t[:, i + 1] - t[:, i])}")
            print(f"  lifetime                         {q(t[:, 4] - t[:, 0])}")
            bins = np.arange(0.0, span + 1.0, 1.0)
            print("  us   resident  prologue  chunk0  rest  epilogue")
            for b in bins:
                alive = np.sum((t[:, 0] <= b) & (t[:, 4] > b))
                ph = [np.sum((t[:, i] <= b) & (t[:, i + 1] > b)) for i in range(4)]
                print(f"  {b:4.0f} {alive:8d} {ph[0]:9d} {ph[1]:7d} {ph[2]:5d} {ph[3]:9d}")


if __name__ == "__main__":
    main()
