# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04s_ab|600|tools/bench_ab.sh 3 'base|' 'g0|--opt graphs=0' 'b128|--batch 128' 'b128g0|--batch 128 --opt graphs=0' 'b64|--batch 64' 'b64g0|--batch 64 --opt graphs=0'" \
  "r04s_tests|400|python -u -m pytest tests/test_gpu_ops.py -q -k 'head or xent' --timeout 300 --timeout-method thread"
