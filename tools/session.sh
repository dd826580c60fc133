# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04i_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r04i_ab|900|tools/bench_ab.sh 3 'b64|--batch 64' 'b64e|--batch 64 --opt graphs=2' 'b128|--batch 128' 'b128e|--batch 128 --opt graphs=2' 'w8|$S8'" \
  "r04i_w8prof|300|tools/prof_run.sh r04i_w8 $S8" \
  "r04i_bench|300|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04i_bench.json"
