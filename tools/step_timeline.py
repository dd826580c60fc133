"""Print one steady-state training step's kernel timeline (start offset, duration, name) from a
rocprofv3 --kernel-trace run of bench.py, steps delimited by the SGD kernel.

usage: python tools/step_timeline.py <rocprof output dir> [--step -3] [--from US] [--to US] [--gaps US]
--gaps G: instead, the step's busy fraction (union of kernel intervals over all streams) and every idle
gap longer than G us with the kernels either side of it, over the last five steps."""
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
    ap.add_argument("--gaps", type=float, default=None)
    args = ap.parse_args()
    db = glob.glob(os.path.join(args.src, "**", "*results.db"), recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if "sgd_nesterov" in r[0]]
    if args.gaps is not None:
        for k in range(-6, -1):
            a, b = idx[k - 1], idx[k]
            seg = rows[a + 1:b + 1]  # after one step's SGD .. the next step's SGD (inclusive)
            t0, t1 = rows[a][2], rows[b][2]
            busy, end, gaps = 0.0, t0, []
            prev = rows[a][0]
            for name, s0, e0 in seg:
                if s0 > end:
                    if (s0 - end) / 1e3 > args.gaps:
                        gaps.append(((end - t0) / 1e3, (s0 - end) / 1e3, prev[:48], name[:48]))
                    busy += e0 - s0
                    end = e0
                elif e0 > end:
                    busy += e0 - end
                    end = e0
                if e0 >= end:
                    prev = name
            wall = (t1 - t0) / 1e3
            idle = wall - busy / 1e3
            print(f"step {k}: wall {wall:.1f} us, busy {busy / 1e3:.1f} us ({100 * busy / 1e3 / wall:.1f}%), "
                  f"idle {idle:.1f} us, gaps > {args.gaps} us: {sum(g[1] for g in gaps):.1f} us")
            for g in gaps:
                print(f"    at {g[0]:8.1f}  {g[1]:6.1f} us  after {g[2]}  before {g[3]}")
        return
    a, b = idx[args.step - 1], idx[args.step]
    t0 = rows[a][1]
    for name, s, e in rows[a:b + 1]:
        t = (s - t0) / 1e3
        if args.t_from <= t <= args.t_to:
            print(f"{t:8.1f} {(e - s) / 1e3:7.2f}  {name[:100]}")


if __name__ == "__main__":
    main()
