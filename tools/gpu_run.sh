#!/bin/bash
# One parameterised GPU session (replaces the per-session command lists of rounds 1-2).
# usage: tools/gpu_run.sh TAG step [step ...]     (run from the repo root, e.g. under gpurun)
# steps:
#   tests            the GPU test suite (one process, per-test timeout)
#   tests:EXPR       GPU tests selected by -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            bench.py $BENCH_ARGS                 -> gpurun_out/TAG_bench.json
#   prof             rocprofv3 kernel trace of a short bench.py $BENCH_ARGS run -> gpurun_out/prof_TAG
#   serprof          serialized kernel trace (bwd_streams=0, graphs=0) WITH the live event roofline of the same run
#                    -> gpurun_out/TAG_ser_kernel_trace.md (events-vs-trace check in one run)
#   pmc              rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate runs) -> gpurun_out/pmc_TAG_{fetch,write}
#   ab:SPEC          tools/bench_ab.sh $AB_ROUNDS SPEC... (SPEC = "tagA|opts;tagB|opts")
#   py:FILE          python FILE $PY_ARGS                 -> gpurun_out/TAG_FILE.log
#   config3          BASELINE config 3 per-rank shapes on one GPU: bench.py --global-batch 256 --sim-world W
#                    for W = 2, 4, 8 (B = 128, 64, 32), each with a rocprofv3 kernel trace
#                    -> gpurun_out/TAG_c3_wW_bench.json, gpurun_out/prof_TAG_c3_wW
# Every step runs under its own time limit via tools/gpu_session.sh (stops on crash / hang).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
BA=${BENCH_ARGS:-}
QUIET="--no-cpu-baseline --no-live-roofline --no-hbm-probe"
specs=()
for st in "$@"; do
  case "$st" in
    tests) specs+=("${TAG}_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread") ;;
    tests:*) specs+=("${TAG}_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k '${st#tests:}'") ;;
    smoke) specs+=("${TAG}_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) specs+=("${TAG}_benchrun|500|python bench.py $BA > gpurun_out/${TAG}_bench.json") ;;
    prof) specs+=("${TAG}_prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_$TAG -o prof -- python3 $ROOT/bench.py --steps 20 --warmup 5 $QUIET $BA") ;;
    serprof) specs+=("${TAG}_serprof|300|tools/prof_run.sh ${TAG}_ser --live --opt bwd_streams=0 --opt graphs=0 $BA") ;;
    pmc) specs+=("${TAG}_pmcf|150|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/pmc_${TAG}_fetch -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 $QUIET $BA")
         specs+=("${TAG}_pmcw|150|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $ROOT/gpurun_out/pmc_${TAG}_write -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 $QUIET $BA") ;;
    ab:*) IFS=';' read -ra parts <<< "${st#ab:}"; q=""; for p in "${parts[@]}"; do q="$q '$p'"; done
          specs+=("${TAG}_ab|900|tools/bench_ab.sh ${AB_ROUNDS:-4}$q") ;;
    config3) for w in 2 4 8; do
               specs+=("${TAG}_c3_w${w}|300|python bench.py --global-batch 256 --sim-world $w --no-cpu-baseline $BA > gpurun_out/${TAG}_c3_w${w}_bench.json")
               specs+=("${TAG}_c3_w${w}_prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_${TAG}_c3_w${w} -o prof -- python3 $ROOT/bench.py --global-batch 256 --sim-world $w --steps 20 --warmup 5 $QUIET $BA")
             done ;;
    py:*) f="${st#py:}"; specs+=("${TAG}_$(basename "$f" .py)|300|python -u $f ${PY_ARGS:-}") ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
tools/gpu_session.sh "${specs[@]}"
exit $?
