tools/gpu_session.sh \
 "dp|400|python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_fp32.py -q -rA --timeout 300 --timeout-method thread -k 'data_parallel or dp_ or native_loss or fp32 or sgd_step'" \
 "benchdp|300|python bench.py --mode dp --dp-devices 0,0 --batch 256 --steps 30 --warmup 5 > gpurun_out/r02_bench_dp.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02b -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
