# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04c_bench|300|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04c_bench.json" \
  "r04c_ser|300|tools/prof_run.sh r04c_ser --opt bwd_streams=0 --opt graphs=0" \
  "r04c_ab|900|tools/bench_ab.sh 3 'base|' 'simr|--sim-world 2 --global-batch 512 --sim-comm loopback' 'sime|--sim-world 2 --global-batch 512 --sim-comm loopback --opt graphs=2' 'ws2|--opt wgrad_s2=1'" \
  "r04c_tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'profile or graph or reducer or ddp'"
