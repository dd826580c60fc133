"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py into a markdown file for profiles/.

usage: python tools/prof_summary.py <rocprof output dir> <out.md> [--bench bench.json] [--gflop-per-step G]

Reports: top kernels (calls, total, average), the conv family (every conv launch bench.py's
`roofline` times: igemm, halo, c64, wgrad_halo, stem fwd / wgrad, and their split-K / wgrad
reductions) per training step with its achieved TFLOP/s and fraction of the bf16 dense peak
(algorithmic conv FLOPs per step, SURVEY §8(d): 852.2 GFLOP at B=256, 32x32 -- --gflop-per-step, else the
bench line's algorithmic_gflop_per_step, else 3.329 GFLOP x its per-GPU batch x (size / 32)^2; no fraction
without one of them), and the per-step timeline of the steady state (busy
time vs wall time between the first and last kernel of a step, i.e. launch gaps). A training step is
delimited by the SGD kernel (one launch per step). Run it on a trace of the SERIALIZED step
(`--opt bwd_streams=0`: no side-stream overlap, every kernel's duration is its own) to reproduce
bench.py's roofline.frac; on an overlapped trace the per-kernel durations are inflated by sharing.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CONV = ("igemm_kernel", "conv_halo_kernel", "conv_c64_kernel", "wgrad_halo_kernel", "splitk_reduce_kernel",
        "wgrad_reduce_kernel", "stem_fwd_kernel", "stem_wgrad_kernel", "stem_wgrad_bn_kernel")
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)


def short(name):
    n = name.replace("void ", "")
    return n.split("(")[0]


CONV_GFLOP_PER_IMAGE = 852.215 / 256  # conv fwd + dgrad + wgrad per 32x32 image


def bench_gflop(bench):
    """(algorithmic conv GFLOP per step, source) of the bench.py line the trace was taken with: the line's
    own live-roofline figure when it measured one, else conv GFLOP per image x its per-GPU batch x
    (image size / 32)^2 (every conv scales with the pixel count). (None, reason) when the line is missing
    or names no batch: no fraction is printed then (a B=256 figure was divided by a
    B=32 trace's conv time)."""
    try:
        b = json.loads([l for l in open(bench) if l.startswith("{")][-1])
    except Exception as e:
        return None, f"bench line unreadable ({e!r})"
    g = (b.get("roofline") or {}).get("algorithmic_gflop_per_step") or 0.0
    if g > 0:
        return g, "bench line roofline.algorithmic_gflop_per_step"
    cfg = b.get("config") or {}
    B, S = cfg.get("per_gpu_batch"), cfg.get("image_size", 32)
    if not B:
        return None, "bench line names no per_gpu_batch"
    return CONV_GFLOP_PER_IMAGE * B * (S / 32) ** 2, f"{CONV_GFLOP_PER_IMAGE:.4f} GFLOP/image x batch {B} x ({S}/32)^2"


def load_rows(src):
    """(start_ns, end_ns, kernel name) per dispatch from a csv kernel trace or a rocpd sqlite db."""
    trace = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
    if trace:
        with open(trace[0]) as f:
            return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                    for r in csv.DictReader(f)]
    dbs = glob.glob(os.path.join(src, "**", "*results.db"), recursive=True)
    assert dbs, f"no kernel_trace.csv or rocpd results.db under {src}"
    import sqlite3

    con = sqlite3.connect(dbs[0])
    return [(int(a), int(b), n) for a, b, n in con.execute("select start, end, name from kernels")]


def main():
    src, out = sys.argv[1], sys.argv[2]
    args = sys.argv[3:]
    bench = args[args.index("--bench") + 1] if "--bench" in args else None
    gflop = float(args[args.index("--gflop-per-step") + 1]) if "--gflop-per-step" in args else None
    gsrc = "--gflop-per-step" if gflop else None
    if gflop is None and bench:
        gflop, gsrc = bench_gflop(bench)
    rows = load_rows(src)
    rows.sort()
    # steps: delimited by the fused SGD kernel
    sgd_idx = [i for i, r in enumerate(rows) if "sgd_nesterov" in r[2]]
    lines = [f"# rocprofv3 kernel trace summary: {os.path.basename(os.path.normpath(src))}", ""]
    stats = defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        stats[short(n)][0] += 1
        stats[short(n)][1] += e - s
    tot = sum(v[1] for v in stats.values())
    lines += ["## All kernels (whole run)", "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for k, (c, d) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:25]:
        lines.append(f"| `{k}` | {c} | {d / 1e6:.3f} | {d / c / 1e3:.2f} | {100 * d / tot:.1f} |")
    if len(sgd_idx) >= 4:
        # steady state: skip the first two steps (graph capture / warmup)
        steps = list(zip(sgd_idx[1:-1], sgd_idx[2:]))[1:]
        # keep training steps only (the modal kernel count): bench.py's HBM probe launches the SGD
        # kernel back to back after the timed regions
        from collections import Counter
        mode = Counter(b - a for a, b in steps).most_common(1)[0][0]
        steps = [(a, b) for a, b in steps if abs(b - a - mode) <= 2]
        busy, wall, conv, nk = [], [], [], []
        per_kernel = defaultdict(lambda: [0, 0])
        for a, b in steps:
            seg = rows[a + 1:b + 1]
            t0, t1 = seg[0][0], seg[-1][1]
            wall.append(t1 - t0)
            # busy = union of kernel intervals
            u, cur_s, cur_e = 0, None, None
            for s, e, n in seg:
                if cur_e is None or s > cur_e:
                    if cur_e is not None:
                        u += cur_e - cur_s
                    cur_s, cur_e = s, e
                else:
                    cur_e = max(cur_e, e)
            u += cur_e - cur_s
            busy.append(u)
            conv.append(sum(e - s for s, e, n in seg if any(c in n for c in CONV)))
            nk.append(len(seg))
            for s, e, n in seg:
                per_kernel[short(n)][0] += 1
                per_kernel[short(n)][1] += e - s
        ns = len(steps)
        avg = lambda v: sum(v) / len(v) / 1e3
        gaps = defaultdict(lambda: [0, 0])
        for a, b in steps:
            seg = rows[a:b + 1]
            for (s0, e0, n0), (s1, e1, n1) in zip(seg, seg[1:]):
                gaps[(short(n0), short(n1))][0] += 1
                gaps[(short(n0), short(n1))][1] += max(0, s1 - e0)
        lines += ["", f"## Steady-state training step (mean of {ns} steps, SGD kernel to SGD kernel)", "",
                  f"* kernels per step: {avg(nk) * 1e3:.0f}",
                  f"* wall (first kernel start to last kernel end): {avg(wall):.1f} us",
                  f"* GPU busy (union of kernel intervals): {avg(busy):.1f} us "
                  f"({100 * sum(busy) / sum(wall):.1f}% of wall)",
                  (f"* conv family (every conv launch incl. stem and split-K / wgrad reductions): {avg(conv):.1f} us "
                   f"per step = {gflop:.1f} GFLOP / {avg(conv):.1f} us = {gflop / avg(conv) * 1e3:.1f} TFLOP/s = "
                   f"{gflop / avg(conv) * 1e3 / BF16_PEAK_TFLOPS:.4f} of the {BF16_PEAK_TFLOPS:.0f} TFLOP/s bf16 dense "
                   f"peak (FLOPs: {gsrc})" if gflop else
                   f"* conv family (every conv launch incl. stem and split-K / wgrad reductions): {avg(conv):.1f} us "
                   f"per step (no fraction of peak: algorithmic FLOPs unknown -- {gsrc or 'pass --bench or --gflop-per-step'})"),
                  "",
                  "| kernel | calls/step | us/step | avg us |", "|---|---|---|---|"]
        for k, (c, d) in sorted(per_kernel.items(), key=lambda kv: -kv[1][1]):
            lines.append(f"| `{k}` | {c / ns:.0f} | {d / ns / 1e3:.1f} | {d / c / 1e3:.2f} |")
        gsum = sum(v[1] for v in gaps.values()) / ns / 1e3
        lines += ["", f"### Idle gaps between consecutive kernels: {gsum:.1f} us per step; largest", "",
                  "| after | before | per step | us/step |", "|---|---|---|---|"]
        for (k0, k1), (c, d) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:15]:
            lines.append(f"| `{k0}` | `{k1}` | {c / ns:.1f} | {d / ns / 1e3:.1f} |")
    if bench:
        try:
            b = json.loads([l for l in open(bench) if l.startswith("{")][-1])
            rf = b.get("roofline", {})
            lines += ["", "## bench.py line of the same run", "", "```", json.dumps(b, indent=1), "```", "",
                      f"bench live conv time per step: {rf.get('conv_ms_per_step')} ms "
                      f"(rocprof conv family above: compare)"]
        except Exception as e:  # keep the summary even if the bench line is missing
            lines += ["", f"(bench line unavailable: {e!r})"]
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:60]))


if __name__ == "__main__":
    main()
