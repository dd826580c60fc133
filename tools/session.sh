# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04u_tests|300|python -u -m pytest tests/test_gpu_ops.py -q -k wgrad --timeout 300 --timeout-method thread" \
  "r04u_wgb|150|python tools/wgrad_bench.py --variants 'wgrad_ksplit=0;wgrad_ksplit=1;wgrad_ksplit=2' --check" \
  "r04u_ab|500|tools/bench_ab.sh 3 'base|' 'ks2|--opt wgrad_ksplit=2'" \
  "r04u_pmc|400|tools/pmc_bench.sh r04u"
