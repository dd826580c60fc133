# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04j_tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "r04j_wgb|150|python tools/wgrad_bench.py --variants 'wgrad_ksplit=0;wgrad_ksplit=1' --check" \
  "r04j_ab|600|tools/bench_ab.sh 3 'base|' 'ks1|--opt wgrad_ksplit=1' 'bnm2|--opt bnb_mask=2' 'bnm2s|--opt bnb_mask=2 --opt halo_stage_epi=1' 'b64|--batch 64' 'b64e|--batch 64 --opt graphs=2'" \
  "r04j_bench|200|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04j_bench.json"
