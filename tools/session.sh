# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04p_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04p_ab|600|tools/bench_ab.sh 4 'base|' 'bnm1|--opt bnb_mask=1' 'bnm2|--opt bnb_mask=2'" \
  "r04p_prof|300|tools/prof_run.sh r04p_bnm1 --opt bnb_mask=1" \
  "r04p_prof2|300|tools/prof_run.sh r04p_b256"
