# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04q_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04q_prof|300|tools/prof_run.sh r04q_b256" \
  "r04q_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04q_bench.json" \
  "r04q_w8|300|tools/bench_ab.sh 2 'w8|$S8' 'b32|--batch 32'"
