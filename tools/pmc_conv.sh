#!/bin/bash
# PMC passes over the conv micro-benchmark (one rocprofv3 run per counter group, each bounded).
set -u
OUT=gpurun_out/pmc
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o run -- \
     python tools/conv_bench.py --iters 3 --variants "igemm_stages=2" > $OUT/$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
