# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "wb|300|python tools/wgrad_bench.py --check --variants 'wgrad_prio=0;wgrad_prio=1' > gpurun_out/r03w_wb.txt" \
  "ab|900|tools/bench_ab.sh 5 'base|' 'pr|--opt wgrad_prio=1'"
