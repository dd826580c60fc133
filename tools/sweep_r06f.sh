#!/bin/bash
# NOTE: `wgrad_l1_min_steps` was a temporary A/B option of that experiment (removed after it; results in DESIGN.md §3 Round 6
# and profiles/): re-running this script needs it added back to kernels.h.
# Round-6 follow-up: the split floor of layer1's one-tile weight-gradient batch (the backward's tail: the compute
# stream waits for it before the stem) at config 3's batches (in-process A/B, temporary option wgrad_l1_min_steps).
set -u
T=$1
ab() { local name=$1; shift; timeout -k 10 280 python -u tools/inproc_ab.py "$@" > gpurun_out/${T}_${name}.txt 2>&1 || exit $?; }
ab b32 --rounds 16 --steps 150 --batch 32 --sim-world 8 "base|" "l1_4|wgrad_l1_min_steps=4" "l1_8|wgrad_l1_min_steps=8" "l1_12|wgrad_l1_min_steps=12" "l1_16|wgrad_l1_min_steps=16"
ab b64 --rounds 14 --steps 100 --batch 64 --sim-world 4 "base|" "l1_4|wgrad_l1_min_steps=4" "l1_12|wgrad_l1_min_steps=12"
