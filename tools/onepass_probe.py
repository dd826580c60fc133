"""Diagnostics for the one-pass BN backward: isolated launch time at the B=256 shapes, and whether the
executor's grid barrier ever timed out (the BNERR flag) in a training step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dtc_import  # noqa: E402

dtc = dtc_import.load()
dev = torch.device("cuda:0")
for opt, (M, C, dual) in [(o, sh) for o in (1, 2) for sh in [(65536, 128, False), (16384, 256, True),
                                                              (4096, 512, False)]]:
    dtc._native.lib.dtc_set_option(b"bn_onepass", opt)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, C, device=dev, generator=g).bfloat16()
    x2 = torch.randn(M, C, device=dev, generator=g).bfloat16() if dual else None
    y = torch.relu(torch.randn(M, C, device=dev, generator=g)).bfloat16()
    dy = torch.randn(M, C, device=dev, generator=g).bfloat16()
    bits = dtc.ops.bn_mask_bits(y)
    mean = torch.zeros(C, device=dev)
    inv = torch.ones(C, device=dev)
    gam = torch.ones(C, device=dev)
    args = (dy, bits, x, mean, inv, gam, x2, mean if dual else None, inv if dual else None, gam if dual else None)
    dtc.ops.bn_bwd_onepass(*args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        dtc.ops.bn_bwd_onepass(*args)
    e1.record()
    torch.cuda.synchronize()
    print(f"onepass(option {opt}) M={M} C={C} dual={dual}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per call (incl. allocs)",
          flush=True)
