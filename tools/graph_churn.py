"""Graph-exec lifecycle stress (diagnostics for the round-2 intermittent crash in
test_live_conv_profile, DESIGN.md "Graph execs"): every cycle changes an option (the next step drops
and destroys the step graphs and re-captures them) and arms / disarms the live conv profile (which
switches between the plain and the profiled graph sets). The native crash handler reports the
faulting thread and its frames if a destroy races anything.

usage: python tools/graph_churn.py [cycles] [batch]
"""
import ctypes as C
import sys
import time

import torch

sys.path.insert(0, ".")
import dtc_import  # noqa: E402

dtc = dtc_import.load()
lib = dtc._native.lib


def main():
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    lib.dtc_install_crash_handler()
    dev = torch.device("cuda:0")
    torch.manual_seed(42)
    model = dtc.ResNet18().to(dev)
    crit = dtc.CrossEntropyLoss()
    x = torch.randn(batch, 3, 32, 32, device=dev)
    y = torch.randint(0, 100, (batch,), device=dev)
    dtc.nn.set_autocast_enabled(True)
    crit(model(x), y).backward()
    exe = model.executor(batch, 32, 32)
    t0 = time.time()
    for i in range(cycles):
        lib.dtc_set_option(b"sc_fuse", i % 2)  # epoch change: the next step drops + re-captures
        crit(model(x), y).backward()
        dtc._native.call("dtc_rn18_profile_begin", exe.handle, 1)
        for _ in range(2):
            crit(model(x), y).backward()
        ms, fl, cnt = (C.c_double * 3)(), (C.c_double * 3)(), (C.c_int * 3)()
        dtc._native.call("dtc_rn18_profile_end", exe.handle, ms, fl, cnt)
        if i % 10 == 0:
            print(f"cycle {i} ok ({time.time() - t0:.1f} s), calls {list(cnt)}", flush=True)
    torch.cuda.synchronize()
    lib.dtc_set_option(b"sc_fuse", 1)
    print(f"graph churn: {cycles} cycles: no crash ({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
