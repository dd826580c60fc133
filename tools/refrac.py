"""Re-derive the conv-family fraction-of-peak line of committed kernel-trace summaries
(profiles/*kernel_trace.md, written by tools/prof_summary.py) from each file's OWN bench.py line:
the algorithmic conv FLOPs of that line's batch and image size (prof_summary.bench_gflop), not a
fixed B=256 figure. Files without a bench line keep their line, marked unchecked.

usage: python tools/refrac.py profiles/*kernel_trace.md"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import BF16_PEAK_TFLOPS, CONV_GFLOP_PER_IMAGE  # noqa: E402

LINE = re.compile(r"^\* conv family \(every conv launch incl\. stem and split-K / wgrad reductions\): ([0-9.]+) us per step.*$",
                  re.M)


def gflop_of(text):
    m = re.search(r"```\n(\{.*?\})\n```", text, re.S)
    if not m:
        return None, "no bench line in the file"
    b = json.loads(m.group(1))
    g = (b.get("roofline") or {}).get("algorithmic_gflop_per_step") or 0.0
    if g > 0:
        return g, "bench line roofline.algorithmic_gflop_per_step"
    cfg = b.get("config") or {}
    B, S = cfg.get("per_gpu_batch"), cfg.get("image_size", 32)
    if not B:
        return None, "bench line names no per_gpu_batch"
    return CONV_GFLOP_PER_IMAGE * B * (S / 32) ** 2, f"{CONV_GFLOP_PER_IMAGE:.4f} GFLOP/image x batch {B} x ({S}/32)^2"


def main():
    for path in sys.argv[1:]:
        text = open(path).read()
        m = LINE.search(text)
        if not m:
            continue
        us = float(m.group(1))
        g, src = gflop_of(text)
        head = "* conv family (every conv launch incl. stem and split-K / wgrad reductions): "
        if g:
            new = (f"{head}{us:.1f} us per step = {g:.1f} GFLOP / {us:.1f} us = {g / us * 1e3:.1f} TFLOP/s = "
                   f"{g / us * 1e3 / BF16_PEAK_TFLOPS:.4f} of the {BF16_PEAK_TFLOPS:.0f} TFLOP/s bf16 dense peak "
                   f"(FLOPs: {src}; re-derived by tools/refrac.py)")
        else:
            new = f"{head}{us:.1f} us per step (no fraction of peak: {src})"
        if new != m.group(0):
            open(path, "w").write(text[:m.start()] + new + text[m.end():])
            print(f"{path}: {m.group(0)[len(head):][:80]} -> {new[len(head):][:100]}")


if __name__ == "__main__":
    main()
