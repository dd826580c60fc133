# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04v_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04v_wgb|150|python tools/wgrad_bench.py --variants 'wgrad_ksplit=0;wgrad_ksplit=2;wgrad_ksplit=3' --check" \
  "r04v_s2cb|200|python tools/conv_bench.py --passes wgrad --layers l2.0.c1,l3.0.c1,l4.0.c1 --variants 'wgrad_ksplit=0;wgrad_ksplit=2'" \
  "r04v_ab|500|tools/bench_ab.sh 3 'base|' 'ks0|--opt wgrad_ksplit=0' 'ks3|--opt wgrad_ksplit=3'"
