tools/gpu_session.sh \
 "t_new|300|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -k 'stem_recompute or shortcut_fused or head_direct' -x -v --timeout 120 --timeout-method thread" \
 "gputest|900|python -X faulthandler -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|400|python bench.py > gpurun_out/r03l_bench.json" \
 "ab|700|tools/bench_ab.sh 4 'new|' 'old|--opt sc_fuse=0 --opt head_direct=0' 'srec|--opt stem_recompute=1'" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03l -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt stem_recompute=1"
