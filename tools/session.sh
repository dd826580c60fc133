# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04aj_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04aj_bench|200|python bench.py > gpurun_out/r04aj_bench.json" \
  "r04aj_tests|800|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread"
