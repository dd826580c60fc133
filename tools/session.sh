# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04ad_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04ad_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04ad_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04ad_bench.json" \
  "r04ad_prof|300|tools/prof_run.sh r04ad_b256" \
  "r04ad_ser|300|tools/prof_run.sh r04ad_ser --opt bwd_streams=0 --opt graphs=0" \
  "r04ad_pmc|400|tools/pmc_bench.sh r04ad"
