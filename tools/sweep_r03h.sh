#!/bin/bash
# round 3: remaining GPU tests (from the BN-sums test on) + A/B of the fused shortcut dgrad and BN sums in dgrad epilogues
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bn_sums or fused_shortcut or shortcut_fused or stem or loss or dp_ or data_parallel or sync or reducer or native or head or capture or option or bench or trainer or graph or fp32 or augment or config" > gpurun_out/r03h_tests.log 2>&1
timeout -k 10 200 python tools/conv_bench.py --batch 256 --layers l2.0.c1,l3.0.c1,l4.0.c1 --passes dgrad --variants "dgrad_scf=0;dgrad_scf=1" > gpurun_out/r03h_bench.txt 2>&1
timeout -k 10 900 tools/bench_ab.sh 4 "base|" "dscf|--opt dgrad_scf=1" "bnbm|--opt bnb_mask=1" "both|--opt dgrad_scf=1 --opt bnb_mask=1" > gpurun_out/r03h_ab.txt 2>&1
