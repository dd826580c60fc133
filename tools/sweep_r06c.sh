#!/bin/bash
# NOTE: `wgrad_min_steps` was a temporary A/B option of that experiment (removed after it; results in DESIGN.md §3 Round 6
# and profiles/): re-running this script needs it added back to kernels.h.
# Round-6 follow-up: the weight-gradient split floor (pixel steps per workgroup, option wgrad_min_steps) at
# config 3's per-rank batches (in-process paired A/B, tools/inproc_ab.py). usage: tools/sweep_r06c.sh TAG [2]
set -u
T=$1
ab() { local name=$1; shift; timeout -k 10 280 python -u tools/inproc_ab.py "$@" > gpurun_out/${T}_${name}.txt 2>&1 || exit $?; }
if [ "${2:-1}" = 1 ]; then
ab b32 --rounds 16 --steps 150 --batch 32 --sim-world 8 "base|" "ms12|wgrad_min_steps=12" "ms16|wgrad_min_steps=16" "ms24|wgrad_min_steps=24" "wh128|wgrad_halo=128"
ab b64 --rounds 14 --steps 100 --batch 64 --sim-world 4 "base|" "ms16|wgrad_min_steps=16" "ms24|wgrad_min_steps=24"
ab b256 --rounds 8 --steps 60 "base|" "ms16|wgrad_min_steps=16"
else
ab b32 --rounds 16 --steps 150 --batch 32 --sim-world 8 "base|" "ms24|wgrad_min_steps=24" "ms32|wgrad_min_steps=32" "ms48|wgrad_min_steps=48" "ms64|wgrad_min_steps=64"
ab b64 --rounds 14 --steps 100 --batch 64 --sim-world 4 "base|" "ms24|wgrad_min_steps=24" "ms32|wgrad_min_steps=32" "ms48|wgrad_min_steps=48"
ab b128 --rounds 12 --steps 80 --batch 128 --sim-world 2 "base|" "ms32|wgrad_min_steps=32" "ms48|wgrad_min_steps=48"
fi
