#!/bin/bash
# PMC passes over one conv (layer, pass, option variant) of tools/conv_bench.py: one rocprofv3 run
# per counter group (gfx950 slot limits: 8 SQ, 4 TCC), each bounded by its own time limit.
# usage: tools/pmc_conv.sh <tag> <layers> <passes> <variant>
set -u
TAG=$1; LAYERS=$2; PASSES=$3; VAR=$4
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
     python3 tools/conv_bench.py --iters 5 --layers "$LAYERS" --passes "$PASSES" --variants "$VAR" > $OUT/$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
