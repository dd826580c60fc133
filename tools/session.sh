# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
B5="--batch 512 --size 224 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-probe"
tools/gpu_session.sh \
  "tests|600|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resnet.py -m gpu -q -x --timeout 200 --timeout-method thread -k 'wgrad or 224 or general or halo'" \
  "b5gen|400|python bench.py $B5 > gpurun_out/r03o_c5_gen.json" \
  "b5off|400|python bench.py $B5 --opt wgrad_gen=0 --opt halo_gen=0 > gpurun_out/r03o_c5_off.json" \
  "p5|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o prof -- python3 \$GRAFT_REPO_ROOT/bench.py --batch 512 --size 224 --steps 3 --warmup 1 --no-cpu-baseline --no-hbm-probe --no-live-roofline"
