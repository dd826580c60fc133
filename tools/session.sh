# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04t_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04t_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r04t_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04t_bench.json" \
  "r04t_prof|300|tools/prof_run.sh r04t_b256" \
  "r04t_ab|400|tools/bench_ab.sh 2 'base|' 'g2|--opt graphs=2' 'w8|$S8' 'w2|--sim-world 2 --global-batch 512 --sim-comm loopback'"
