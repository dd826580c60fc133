#!/bin/bash
# Round-6 re-check of the tuning defaults at the final kernels (in-process paired A/B, tools/inproc_ab.py).
# usage (repo root, GPU box): tools/sweep_r06.sh TAG
set -u
T=$1
ab() { local name=$1; shift; timeout -k 10 240 python -u tools/inproc_ab.py "$@" > gpurun_out/${T}_${name}.txt 2>&1 || exit $?; }
ab b256_wg --rounds 10 --steps 60 "base|" "wh192|wgrad_halo=192" "wh256|wgrad_halo=256" "s2w96|wgrad_s2_wgs=96" "s2w192|wgrad_s2_wgs=192"
ab b256_bn --rounds 10 --steps 60 "base|" "bre8k|bn_red_elems=8192" "bre32k|bn_red_elems=32768" "fab512|bn_fa_blocks=512" "fab2048|bn_fa_blocks=2048"
ab b256_misc --rounds 10 --steps 60 "base|" "wgb3|wgrad_batch=3" "hs0|halo_small=0" "wl1_112|wgrad_halo_l1=112"
ab b32_a --rounds 10 --steps 150 --batch 32 --sim-world 8 "base|" "hf2|head_fused=2" "hs0|halo_small=0" "wh128|wgrad_halo=128" "wh256|wgrad_halo=256"
ab b32_b --rounds 10 --steps 150 --batch 32 --sim-world 8 "base|" "brb128|bn_red_blocks=128" "fab256|bn_fa_blocks=256" "bre4k|bn_red_elems=4096" "wl1_64|wgrad_halo_l1=64"
