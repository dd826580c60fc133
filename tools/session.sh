# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04aa_tests|600|python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread" \
  "r04aa_ab|600|tools/bench_ab.sh 4 'base|' 'ring3|--opt wgrad_ring=3' 'wh256|--opt wgrad_halo=256' 'ws96|--opt wgrad_s2_wgs=96'" \
  "r04aa_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04aa_bench.json" \
  "r04aa_prof|300|tools/prof_run.sh r04aa_b256"
