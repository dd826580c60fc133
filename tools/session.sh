# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04n_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04n_ab|600|tools/bench_ab.sh 3 'base|' 's2gen|--opt wgrad_s2=2' 'hf2|--opt head_fused=2' 'w8|$S8' 'w8hs1|$S8 --opt halo_split=1'" \
  "r04n_prof|300|tools/prof_run.sh r04n_b256" \
  "r04n_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04n_bench.json"
