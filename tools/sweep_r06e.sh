#!/bin/bash
# Round-6 follow-up: kernel-choice options at config 3's per-rank batches (in-process paired A/B,
# tools/inproc_ab.py). usage (repo root, GPU box): tools/sweep_r06e.sh TAG
set -u
T=$1
ab() { local name=$1; shift; timeout -k 10 280 python -u tools/inproc_ab.py "$@" > gpurun_out/${T}_${name}.txt 2>&1 || exit $?; }
ab b32 --rounds 14 --steps 150 --batch 32 --sim-world 8 "base|" "cg512k|bn_cg_elems=524288" "c64_2|conv_c64=2" "wgb2|wgrad_batch=2" "s2h2|dgrad_s2h=2" "isp2|igemm_split=2" "isp4|igemm_split=4"
ab b64 --rounds 12 --steps 100 --batch 64 --sim-world 4 "base|" "cg512k|bn_cg_elems=524288" "c64_2|conv_c64=2" "s2h2|dgrad_s2h=2" "isp2|igemm_split=2"
