"""Print one steady-state training step's kernel timeline (start offset, duration, name) from a
rocprofv3 --kernel-trace run of bench.py, steps delimited by the SGD kernel.

usage: python tools/step_timeline.py <rocprof output dir> [--step -3] [--from US] [--to US]"""
import argparse
import glob
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--from", dest="t_from", type=float, default=0.0)
    ap.add_argument("--to", dest="t_to", type=float, default=1e9)
    args = ap.parse_args()
    db = glob.glob(os.path.join(args.src, "**", "*results.db"), recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if "sgd_nesterov" in r[0]]
    a, b = idx[args.step - 1], idx[args.step]
    t0 = rows[a][1]
    for name, s, e in rows[a:b + 1]:
        t = (s - t0) / 1e3
        if args.t_from <= t <= args.t_to:
            print(f"{t:8.1f} {(e - s) / 1e3:7.2f}  {name[:100]}")


if __name__ == "__main__":
    main()
