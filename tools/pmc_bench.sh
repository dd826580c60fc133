#!/bin/bash
# HBM traffic per conv launch of the bench step (roofline.traffic): two rocprofv3 PMC passes over a short
# bench.py run (FETCH_SIZE and WRITE_SIZE do not fit one pass: 3 + 2 TCC slots), each under its own time
# limit, summarised ON the box by tools/pmc_traffic.py; the raw counter directories are deleted.
# usage: tools/pmc_bench.sh TAG   -> gpurun_out/TAG_conv_traffic.json
set -u
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${TAG}_$c" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --no-live-roofline --no-hbm-probe \
      > "$OUT/pmc_${TAG}_$c.log" 2>&1 ) || { echo "pmc $c failed"; exit 1; }
done
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc_${TAG}_FETCH_SIZE" "$OUT/pmc_${TAG}_WRITE_SIZE" "$OUT/${TAG}_conv_traffic.json"
rc=$?
rm -rf "$OUT/pmc_${TAG}_FETCH_SIZE" "$OUT/pmc_${TAG}_WRITE_SIZE"
exit $rc
