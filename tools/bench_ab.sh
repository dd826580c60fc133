#!/bin/bash
# Interleaved A/B of bench.py option sets on one box: R rounds, each config once per round, the timed
# value of every run appended to gpurun_out/ab_<tag>.txt. usage: tools/bench_ab.sh ROUNDS "tag|opts" ...
# opts may start with "ENV:VAR=value VAR2=value;" to run that config under extra environment variables
set -u
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for spec in "$@"; do
    tag="${spec%%|*}"; opts="${spec#*|}"
    envs=""; case "$opts" in ENV:*) envs="${opts%%;*}"; envs="${envs#ENV:}"; opts="${opts#*;}";; esac
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --steps 40 --warmup 10 $opts > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || { echo "run $tag failed"; exit 1; }
    v=$(tail -1 gpurun_out/ab_run.json | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$tag $v" | tee -a gpurun_out/ab_$tag.txt
  done
done
