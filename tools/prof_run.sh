#!/bin/bash
# rocprofv3 kernel trace of one bench.py run, summarised ON the box (the raw trace can exceed gpurun's
# 64 MiB copy-back): gpurun_out/TAG_kernel_trace.md (tools/prof_summary.py), TAG_timeline.txt (one
# steady step, tools/step_timeline.py); the raw rocprof directory is deleted afterwards.
# usage: tools/prof_run.sh TAG [--hip] [--live] bench.py-args...
#   --live: keep bench.py's live (event-timed) roofline region, so the trace and the bench line's event figure
#           come from the same run (with --opt bwd_streams=0 --opt graphs=0 every step of it is serialized)
set -u
TAG=$1; shift
EXTRA=""
LIVE="--no-live-roofline"
if [ "${1:-}" = "--hip" ]; then EXTRA="--hip-trace"; shift; fi
if [ "${1:-}" = "--live" ]; then LIVE=""; shift; fi
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats $EXTRA -d "$OUT/prof_$TAG" -o prof -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline $LIVE --no-hbm-probe "$@" \
    > "$OUT/${TAG}_prof_bench.json" ) || exit $?
python3 "$ROOT/tools/prof_summary.py" "$OUT/prof_$TAG" "$OUT/${TAG}_kernel_trace.md" --bench "$OUT/${TAG}_prof_bench.json" > /dev/null
python3 "$ROOT/tools/step_timeline.py" "$OUT/prof_$TAG" > "$OUT/${TAG}_timeline.txt" 2>&1 || true
python3 "$ROOT/tools/step_timeline.py" "$OUT/prof_$TAG" --gaps 2 > "$OUT/${TAG}_gaps.txt" 2>&1 || true
if [ -n "$EXTRA" ]; then python3 "$ROOT/tools/api_summary.py" "$OUT/prof_$TAG" > "$OUT/${TAG}_hip_api.txt" 2>&1 || true; fi
rm -rf "$OUT/prof_$TAG"
