"""Run the 200-step loss-curve workload of tests/golden/loss_curve.json on the GPU under option
variants (numerically equivalent summation orders) and print the curve statistics against the
reference's fp32 and bf16 runs. Used to calibrate the loss-curve parity bound."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dtc_import  # noqa: E402


def perturb_ulp(model, seed):
    """Same 1-ulp init perturbation as tests/golden/make_golden.py::_perturb_ulp."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for prm in model.parameters():
            sign = torch.randint(0, 2, prm.shape, generator=g).float() * 2 - 1
            prm.mul_(1 + sign * 2.0 ** -23)


def run(dtc, dev, lc, seed=42, ulp=0):
    batch, steps = lc["batch"], lc["steps"]
    templates = torch.randn(100, 3, 32, 32, generator=torch.Generator().manual_seed(1234))
    torch.manual_seed(seed)
    model = dtc.ResNet18()
    if ulp:
        perturb_ulp(model, ulp)
    model = model.to(dev)
    crit = dtc.CrossEntropyLoss()
    opt = dtc.SGD(model.parameters(), lr=lc["lr"], weight_decay=lc["wd"], momentum=lc["momentum"], nesterov=True)
    losses = []
    for s in range(steps):
        gen = torch.Generator().manual_seed(1234 + s)
        y = torch.randint(0, 100, (batch,), generator=gen)
        x = 0.5 * templates[y] + torch.randn(batch, 3, 32, 32, generator=gen)
        opt.zero_grad()
        with dtc.autocast():
            loss = crit(model(x.to(dev)), y.to(dev))
        loss.backward()
        opt.step()
        losses.append(loss)
    return np.array([float(v) for v in losses])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="", help="';'-separated 'name=v,name=v' option sets")
    ap.add_argument("--seeds", default="42")
    ap.add_argument("--ulp", default="", help="comma-separated 1-ulp perturbation seeds (seed-42 init)")
    ap.add_argument("--out", default="gpurun_out/loss_curves.json")
    args = ap.parse_args()
    dtc = dtc_import.load()
    dev = torch.device("cuda", 0)
    lc = json.load(open(os.path.join(ROOT, "tests", "golden", "loss_curve.json")))
    ref, ref32 = np.array(lc["bf16"]), np.array(lc["fp32"])
    res = {}
    for var in [""] + [v for v in args.variants.split(";") if v]:
        kv = [x.split("=") for x in var.split(",") if x]
        defaults = {k: int(dtc._native.lib.dtc_get_option(k.encode())) for k, _ in kv}
        for k, v in kv:
            dtc._native.call("dtc_set_option", k.encode(), int(v))
        for seed in [int(s) for s in args.seeds.split(",")]:
            cur = run(dtc, dev, lc, seed)
            key = f"{var or 'default'}|seed{seed}"
            res[key] = cur.tolist()
            w = lambda a: a.reshape(-1, 20).mean(1)
            print(key, "mean", round(cur.mean(), 4), "ref bf16", round(ref.mean(), 4), "fp32", round(ref32.mean(), 4),
                  "rel", round((cur.mean() - ref.mean()) / ref.mean(), 4), flush=True)
            print("   win20 ours", np.round(w(cur), 3).tolist(), flush=True)
        for k, _ in kv:  # restore defaults
            dtc._native.call("dtc_set_option", k.encode(), defaults[k])
    for u in [int(v) for v in args.ulp.split(",") if v]:
        cur = run(dtc, dev, lc, 42, u)
        res[f"ulp{u}"] = cur.tolist()
        print(f"ulp{u} mean", round(cur.mean(), 4), "rel", round((cur.mean() - ref.mean()) / ref.mean(), 4), flush=True)
        print("   win20 ours", np.round(cur.reshape(-1, 20).mean(1), 3).tolist(), flush=True)
    print("   win20 ref ", np.round(ref.reshape(-1, 20).mean(1), 3).tolist())
    print("   win20 r32 ", np.round(ref32.reshape(-1, 20).mean(1), 3).tolist())
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"))


if __name__ == "__main__":
    main()
