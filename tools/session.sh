# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S2='--sim-world 2 --global-batch 512 --sim-comm loopback'
W2='--sim-world 2 --global-batch 256 --sim-comm loopback'
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04g_tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'reducer or ddp_two or config3 or head or bucketed'" \
  "r04g_ab|1000|tools/bench_ab.sh 3 'base|' 'sim2|$S2' 'sim2r|$S2 --opt graphs=1' 'w2|$W2' 'w2old|$W2 --opt comm_on_side=0' 'w8|$S8' 'w8old|$S8 --opt comm_on_side=0 --opt head_fused=0'" \
  "r04g_bench|300|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04g_bench.json"
