"""HBM traffic of the conv family (the bench.py roofline kernel) from rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py <FETCH_SIZE run dir> <WRITE_SIZE run dir> <out.json>

Each directory holds a `rocprofv3 --pmc <counter> --output-format csv` run of bench.py (one counter
per run: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2, they do not fit one pass). Per the gfx950
notes in MI355X_MICROARCH.md (§HBM): FETCH_SIZE counts half the bytes of wide (16 B/lane)
coalesced reads, which is every load the conv kernels issue (global_load_lds_dwordx4 /
buffer_load ... lds), so it is doubled; WRITE_SIZE is exact for 16-B stores. Both are in KiB.
One conv call = one igemm_kernel, conv_halo_kernel, conv_c64_kernel or wgrad_halo_kernel dispatch (+ its split-K / wgrad reduction).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

MAIN = ("igemm_kernel", "conv_halo_kernel", "conv_c64_kernel", "wgrad_halo_kernel")
AUX = ("splitk_reduce_kernel", "wgrad_reduce_kernel")


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert f, f"no counter_collection.csv under {d}"
    per = defaultdict(float)
    calls = 0
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] != counter:
            continue
        n = r["Kernel_Name"]
        if any(k in n for k in MAIN + AUX):
            key = n.replace("void ", "").split("(")[0]
            per[key] += float(r["Counter_Value"])
            if any(k in n for k in MAIN):
                calls += 1
    return per, calls


def main():
    fd, wd, out = sys.argv[1:4]
    fetch, calls_f = load(fd, "FETCH_SIZE")
    write, calls_w = load(wd, "WRITE_SIZE")
    fb = 2.0 * 1024.0 * sum(fetch.values())  # gfx950 correction x2, KiB -> B
    wb = 1024.0 * sum(write.values())
    res = {
        "conv_calls_fetch_run": calls_f,
        "conv_calls_write_run": calls_w,
        "fetch_bytes_per_call": fb / max(1, calls_f),
        "write_bytes_per_call": wb / max(1, calls_w),
        "hbm_bytes_per_call": fb / max(1, calls_f) + wb / max(1, calls_w),
        "per_kernel_fetch_KiB_x2": {k: 2 * v for k, v in sorted(fetch.items(), key=lambda kv: -kv[1])},
        "per_kernel_write_KiB": dict(sorted(write.items(), key=lambda kv: -kv[1])),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs of bench.py; FETCH_SIZE x2 "
                  "(gfx950, 16-B/lane reads), KiB x1024; summed over igemm/halo + reduction dispatches, divided "
                  "by the igemm/halo dispatch count",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith("per_kernel")}, indent=1))


if __name__ == "__main__":
    main()
