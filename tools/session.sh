# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04o_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04o_prof|300|tools/prof_run.sh r04o_b256" \
  "r04o_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04o_bench.json" \
  "r04o_ab|600|tools/bench_ab.sh 4 'base|' 's2gen|--opt wgrad_s2=2'"
