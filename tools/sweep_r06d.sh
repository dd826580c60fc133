#!/bin/bash
# NOTE: `wgrad_s2_min_steps` was a temporary A/B option of that experiment (removed after it; results in DESIGN.md §3 Round 6
# and profiles/): re-running this script needs it added back to kernels.h.
# Round-6 follow-up: the stride-2 weight-gradient split floor (pixel steps per workgroup) at B = 32 / 64 / 256
# (in-process paired A/B, tools/inproc_ab.py, temporary option wgrad_s2_min_steps). usage: tools/sweep_r06d.sh TAG
set -u
T=$1
ab() { local name=$1; shift; timeout -k 10 280 python -u tools/inproc_ab.py "$@" > gpurun_out/${T}_${name}.txt 2>&1 || exit $?; }
ab b32 --rounds 16 --steps 150 --batch 32 --sim-world 8 "base|" "s8|wgrad_s2_min_steps=8" "s16|wgrad_s2_min_steps=16" "s24|wgrad_s2_min_steps=24"
ab b64 --rounds 12 --steps 100 --batch 64 --sim-world 4 "base|" "s8|wgrad_s2_min_steps=8" "s16|wgrad_s2_min_steps=16" "s24|wgrad_s2_min_steps=24"
ab b256 --rounds 12 --steps 60 "base|" "s8|wgrad_s2_min_steps=8" "s16|wgrad_s2_min_steps=16" "s24|wgrad_s2_min_steps=24"
