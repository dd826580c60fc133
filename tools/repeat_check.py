"""Repeatability probe: the same training forward + backward N times on fixed weights and data; reports, per
option set, which parameters' gradients differ from the first repetition and by how much (diagnostics for
run-to-run nondeterminism; tests/test_gpu_resnet.py::test_backward_repeatable_across_steps is the test)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dtc_import  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--variants", default="graphs=0;graphs=1;graphs=1,bwd_streams=0;graphs=0,bwd_streams=0")
    args = ap.parse_args()
    dtc = dtc_import.load()
    nat = dtc._native
    dev = torch.device("cuda:0")
    lay = dtc.nn.Layout(100, 25.0)
    g = np.random.default_rng(0)
    x = torch.from_numpy(g.standard_normal((args.batch, 3, 32, 32)).astype(np.float32)).to(dev)
    y = torch.from_numpy(g.integers(0, 100, args.batch)).to(dev)
    names = [v for v in args.variants.split(";")]
    keys = sorted({kv.split("=")[0] for v in names for kv in v.split(",")})
    defaults = {k: nat.lib.dtc_get_option(k.encode()) for k in keys}
    for v in names:
        opts = dict(defaults)
        opts.update({kv.split("=")[0]: int(kv.split("=")[1]) for kv in v.split(",")})
        for k, val in opts.items():
            nat.call("dtc_set_option", k.encode(), val)
        torch.manual_seed(42)
        model = dtc.ResNet18().to(dev)
        crit = dtc.CrossEntropyLoss()
        grads = []
        with dtc.autocast():
            for _ in range(args.reps):
                loss = crit(model(x), y)
                loss.backward()
                grads.append(model.flat.grads.detach().float().cpu().numpy().copy())
        ndiff = []
        for r in range(1, args.reps):
            bad = []
            for pe in lay.params:
                a, b = grads[0][pe.offset:pe.offset + pe.numel], grads[r][pe.offset:pe.offset + pe.numel]
                if not np.array_equal(a, b):
                    bad.append((pe.name, float(np.linalg.norm(a - b) / max(np.linalg.norm(a), 1e-30))))
            ndiff.append(bad)
        print(f"=== {v}: reps differing from rep 0: {sum(1 for b in ndiff if b)}/{args.reps - 1}")
        for r, bad in enumerate(ndiff, 1):
            if bad:
                worst = max(bad, key=lambda t: t[1])
                print(f"  rep {r}: {len(bad)} params differ, last in backward order {bad[-1][0]}... first {bad[0][0]}, "
                      f"worst {worst[0]} {worst[1]:.2e}")
        del model
        torch.cuda.synchronize()
    for k, val in defaults.items():
        nat.call("dtc_set_option", k.encode(), val)


if __name__ == "__main__":
    main()
