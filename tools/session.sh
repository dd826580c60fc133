# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04k_tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r04k_wgb|150|python tools/wgrad_bench.py --variants 'wgrad_ksplit=0;wgrad_ksplit=1' --check" \
  "r04k_ab|600|tools/bench_ab.sh 3 'base|' 'ks1|--opt wgrad_ksplit=1' 'b64|--batch 64' 'b64r|--batch 64 --opt graphs=1' 'b32|--batch 32' 'b32r|--batch 32 --opt graphs=1'" \
  "r04k_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04k_bench.json"
