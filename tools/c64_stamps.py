"""Cycle stamps of layer1's persistent conv (conv_c64.hip, diagnostics): where a wave's cycles go, per tile.

Needs the diagnostic library (`make -C distributed-training-comparison_amd/csrc phases`); the stamps are
compiled only there. Every wave writes s_memtime (shader clock) at: 0 entry, 1 prologue issued (filter DMA,
fragment offsets, first halo DMA), 2+2k tile k's halo landed (after the wait + barrier), 3+2k tile k's MFMAs
and the previous tile's epilogue issued, 14 last epilogue issued, 15 statistics done; 16 / 17 s_memrealtime
(100 MHz) at entry / exit give the clock. Prints medians over waves, in cycles, and the MFMA floor of a tile
(288 x 16 cycles)."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="256,128")
    ap.add_argument("--passes", default="fwd,dgrad")
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
    buf = torch.zeros(1024 * 4 * 32, dtype=torch.int64, device=dev)
    fn_set = nat.lib.dtc_probe_phase_buffer
    fn_set.argtypes = [ctypes.c_void_p]
    fn_set.restype = ctypes.c_int
    fn_set(ctypes.c_void_p(buf.data_ptr()))
    P_ = nat.ptr
    for B in map(int, args.batch.split(",")):
        H, C = 32, 64
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w = (torch.randn(C, 3, 3, C, device=dev) * 0.05).bfloat16()
        y = torch.empty(B, H, H, C, device=dev).bfloat16()
        dy = torch.randn(B, H, H, C, device=dev).bfloat16()
        dx = torch.empty(B, H, H, C, device=dev).bfloat16()
        stats = ops.new_stats(C, dev)
        d = ops.conv_desc(B, H, H, C, C, 3, 3, 1, 1)
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
            reps = []
            for _ in range(5):
                buf.zero_()
                torch.cuda.synchronize()
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                fn()
                ev1.record()
                torch.cuda.synchronize()
                reps.append((ev0.elapsed_time(ev1) * 1e3, buf.view(1024 * 4, 32).cpu().numpy().astype(np.float64)))
            reps.sort(key=lambda r: r[0])
            us, t = reps[len(reps) // 2]
            t = t[t[:, 0] > 0]
            if len(t) == 0:
                print(f"B={B} {pname}: no stamps (not a conv_c64 launch?)")
                continue
            ntiles = B * H * H // 256
            waves = len(t)
            grid = waves // 4
            kt = min(6, -(-ntiles // grid))
            mhz = np.median((t[:, 15] - t[:, 0]) / ((t[:, 17] - t[:, 16]) / 100.0))
            span_us = (t[:, 17].max() - t[:, 16].min()) / 100.0
            med = lambda a: float(np.median(a))  # noqa: E731
            print(f"=== layer1 {pname} B={B}: {grid} workgroups, {ntiles} tiles (<= {kt} per workgroup), events "
                  f"{us:.2f} us, stamped span {span_us:.2f} us, clock {mhz:.0f} MHz; cycles, median over waves")
            print(f"  prologue issue          {med(t[:, 1] - t[:, 0]):8.0f}")
            print(f"  first halo wait+barrier {med(t[:, 2] - t[:, 1]):8.0f}")
            for k in range(kt):
                has = t[:, 3 + 2 * k] > 0
                comp = t[has, 3 + 2 * k] - t[has, 2 + 2 * k]
                line = f"  tile {k}: MFMA+epi issue {med(comp):8.0f} (floor 4608)"
                if k + 1 < kt:
                    nxt = t[:, 2 + 2 * (k + 1)] > 0
                    wt = t[nxt, 2 + 2 * (k + 1)] - t[nxt, 3 + 2 * k]
                    line += f"   wait+barrier {med(wt):7.0f}"
                print(line)
            last = np.max(np.where(t[:, 2:14] > 0, t[:, 2:14], 0), axis=1)
            print(f"  last epilogue           {med(t[:, 14] - last):8.0f}")
            print(f"  statistics              {med(t[:, 15] - t[:, 14]):8.0f}")
            print(f"  total                   {med(t[:, 15] - t[:, 0]):8.0f}  (entry spread "
                  f"{(t[:, 16].max() - t[:, 16].min()) / 100.0:.2f} us)")


if __name__ == "__main__":
    main()
