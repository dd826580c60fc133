#!/bin/bash
# Round-6 follow-up: weight-gradient split target and BN-reduce grain at config 3's per-rank batches
# (in-process paired A/B, tools/inproc_ab.py). usage (repo root, GPU box): tools/sweep_r06b.sh TAG
set -u
T=$1
ab() { local name=$1; shift; timeout -k 10 280 python -u tools/inproc_ab.py "$@" > gpurun_out/${T}_${name}.txt 2>&1 || exit $?; }
ab b32 --rounds 16 --steps 150 --batch 32 --sim-world 8 "base|" "wh96|wgrad_halo=96" "wh128|wgrad_halo=128" "wh160|wgrad_halo=160" "bre4k|bn_red_elems=4096" "brb128|bn_red_blocks=128"
ab b64 --rounds 14 --steps 100 --batch 64 --sim-world 4 "base|" "wh128|wgrad_halo=128" "wh160|wgrad_halo=160" "bre4k|bn_red_elems=4096" "brb128|bn_red_blocks=128"
ab b128 --rounds 12 --steps 80 --batch 128 --sim-world 2 "base|" "wh128|wgrad_halo=128" "wh160|wgrad_halo=160" "bre8k|bn_red_elems=8192"
ab b256 --rounds 14 --steps 60 "base|" "fab2048|bn_fa_blocks=2048" "wh160|wgrad_halo=160"
