tools/gpu_session.sh \
 "gputest|900|python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --no-cpu-baseline > gpurun_out/r02g_bench.json" \
 "benchab|300|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 > gpurun_out/r02g_bench_nostreams.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02g -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
