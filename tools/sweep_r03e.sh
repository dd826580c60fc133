#!/bin/bash
# round-3 tile sweep of the existing conv kernels (isolated launches, B=256)
set -e
timeout -k 10 280 python tools/conv_bench.py --batch 256 --layers l2,l3,l4 --passes fwd,dgrad \
  --variants "halo_conv=1;halo_conv=2;halo_conv=3;halo_conv=4;halo_conv=5;halo_conv=6;halo_conv=7;halo_conv=8;halo_conv=9;halo_conv=1,halo_wstages=2;halo_conv=1,halo_split=1" \
  > gpurun_out/r03e_halo_sweep.txt 2>&1
timeout -k 10 280 python tools/conv_bench.py --batch 256 --layers l2.0.c1,l3.0.c1,l4.0.c1,l2.sc,l3.sc,l4.sc \
  --variants "igemm_tile=0;igemm_tile=1;igemm_tile=2;igemm_tile=3;igemm_stages=3;igemm_tile=2,igemm_stages=3;igemm_split=1" \
  > gpurun_out/r03e_igemm_sweep.txt 2>&1
