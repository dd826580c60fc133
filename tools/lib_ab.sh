#!/bin/bash
# Interleaved A/B of library BUILDS (not options) on one box: R rounds, each build once per round, bench.py
# with the live roofline region, printing the step rate, the serialized BN family (bn_in_step) and conv time.
# usage: tools/lib_ab.sh ROUNDS TAG=path/to/libdtc_amd.so ... (extra bench.py args in $BENCH_ARGS)
set -u
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for spec in "$@"; do
    tag="${spec%%=*}"; lib="${spec#*=}"
    DTC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-hbm-probe --steps 40 --warmup 10 ${BENCH_ARGS:-} \
      > gpurun_out/lab_run.json 2> gpurun_out/lab_run.err || { echo "run $tag failed"; tail -5 gpurun_out/lab_run.err; exit 1; }
    python - "$tag" <<'PY' | tee -a gpurun_out/lab_ab.txt
import json, sys
d = json.loads([l for l in open("gpurun_out/lab_run.json") if l.startswith("{")][-1])
bn = d.get("bn_in_step") or {}
print(sys.argv[1], d["value"], "bn_ms", bn.get("ms_per_step"), "bn_stamp", bn.get("stamp_ms_per_step"),
      "conv_ms", d["roofline"].get("conv_ms_per_step"))
PY
  done
done
