"""Host-side HIP API time of a rocprofv3 --hip-trace run (rocpd results.db): per API name the call
count, total, mean and max duration, and the 30 longest single calls -- where the host blocks while
issuing a step (e.g. inside ncclAllReduce / hipStreamWaitEvent / hipGraphLaunch).

usage: python tools/api_summary.py <rocprof output dir>"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    db = glob.glob(os.path.join(sys.argv[1], "**", "*results.db"), recursive=True)[0]
    con = sqlite3.connect(db)
    names = [r[0] for r in con.execute("select name from sqlite_master where type in ('table', 'view')")]
    src = next((v for v in ("regions", "rocpd_region") if v in names), None)
    if src is None:
        print("no API region table; tables/views:", names)
        return
    cols = [r[1] for r in con.execute(f"pragma table_info({src})")]
    ncol = "name" if "name" in cols else next(c for c in cols if "name" in c)
    rows = con.execute(f"select {ncol}, start, end from {src}").fetchall()
    agg = defaultdict(lambda: [0, 0, 0])
    for n, s, e in rows:
        d = (e - s) / 1e3
        a = agg[n]
        a[0] += 1
        a[1] += d
        a[2] = max(a[2], d)
    print(f"{len(rows)} API calls from {src}\n")
    print(f"{'api':60s} {'calls':>7s} {'total us':>11s} {'mean us':>9s} {'max us':>9s}")
    for n, (c, t, m) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{str(n)[:60]:60s} {c:7d} {t:11.1f} {t / c:9.2f} {m:9.1f}")
    print("\nlongest calls:")
    for n, s, e in sorted(rows, key=lambda r: r[1] - r[2])[:30]:
        print(f"  {(e - s) / 1e3:9.1f} us  {n}")


if __name__ == "__main__":
    main()
