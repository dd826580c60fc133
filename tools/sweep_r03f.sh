#!/bin/bash
# round 3: stride-2 halo forward (+ fused shortcut) -- parity, isolated timing, step A/B
set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stride2_halo or halo_s2" > gpurun_out/r03f_tests.log 2>&1
timeout -k 10 280 python tools/conv_bench.py --batch 256 --layers l2.0.c1,l3.0.c1,l4.0.c1,l2.sc,l3.sc,l4.sc --passes fwd,fwdsc \
  --variants "halo_s2=0;halo_s2=1;halo_s2=3;halo_s2=4" > gpurun_out/r03f_s2_bench.txt 2>&1
timeout -k 10 280 python tools/conv_bench.py --batch 32 --layers l2.0.c1,l3.0.c1,l4.0.c1,l2.sc,l3.sc,l4.sc --passes fwd,fwdsc \
  --variants "halo_s2=0;halo_s2=1;halo_s2=3;halo_s2=4" > gpurun_out/r03f_s2_bench_b32.txt 2>&1
timeout -k 10 600 tools/bench_ab.sh 3 "base|" "s2|--opt halo_s2=1" "s2c9|--opt halo_s2=3" > gpurun_out/r03f_ab.txt 2>&1
