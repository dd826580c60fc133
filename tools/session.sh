# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04l_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04l_ab|600|tools/bench_ab.sh 3 'base|' 'hf1|--opt head_fused=1' 's2|--opt wgrad_s2=1' 'w8|$S8' 'w8cg1m|$S8 --opt bn_cg_elems=1048576' 'w8cg2m|$S8 --opt bn_cg_elems=2097152'" \
  "r04l_w8prof|300|tools/prof_run.sh r04l_w8 $S8"
