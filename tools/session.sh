# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04r_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04r_prof|300|tools/prof_run.sh r04r_b256" \
  "r04r_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04r_bench.json" \
  "r04r_w8prof|300|tools/prof_run.sh r04r_w8 $S8" \
  "r04r_w8|400|tools/bench_ab.sh 2 'w8|$S8' 'w8s0|$S8 --opt bwd_streams=0' 'w8g0|$S8 --opt graphs=0' 'b32|--batch 32' 'b32s0|--batch 32 --opt bwd_streams=0' 'b32g0|--batch 32 --opt graphs=0'"
