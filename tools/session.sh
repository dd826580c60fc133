# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "ab|900|tools/bench_ab.sh 4 'base|' 'scs|--opt sc_stream=1' 'pr|--opt wgrad_prio=1' 'd2|--opt wgrad_defer=2' 'bm|--opt bnb_mask=1'"
