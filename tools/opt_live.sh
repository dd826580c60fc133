#!/bin/bash
# Interleaved option sets with bench.py's live (serialized, event-timed) regions: img/s, BN family and conv
# family ms per step. usage: tools/opt_live.sh ROUNDS "tag|bench args" ...
set -u
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for spec in "$@"; do
    tag="${spec%%|*}"; opts="${spec#*|}"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-hbm-probe --steps 40 --warmup 10 $opts \
      > gpurun_out/ol_run.json 2> gpurun_out/ol_run.err || { echo "run $tag failed"; tail -5 gpurun_out/ol_run.err; exit 1; }
    python - "$tag" <<'PY' | tee -a gpurun_out/ol_ab.txt
import json, sys
d = json.loads([l for l in open("gpurun_out/ol_run.json") if l.startswith("{")][-1])
bn = d.get("bn_in_step") or {}
r = d["roofline"]
print(sys.argv[1], d["value"], "bn_ms", bn.get("ms_per_step"), "bn_calls", bn.get("calls_per_step"),
      "conv_ms", r.get("conv_ms_per_step"), "by_pass", r.get("conv_ms_by_pass"), "region_ms", r.get("region_ms_per_step"))
PY
  done
done
