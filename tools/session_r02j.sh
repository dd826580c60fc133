tools/gpu_session.sh \
 "t0|300|python -u -m pytest tests/test_gpu_ops.py -v --timeout 120 --timeout-method thread -k 'onepass'" \
 "t1|600|python -u -m pytest tests/test_gpu_resnet.py -q --timeout 300 --timeout-method thread -k 'onepass or fused_bn_finalize or teacher_forced'" \
 "bench|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 > gpurun_out/r02j_bench.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02j -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0"
