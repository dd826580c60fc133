tools/gpu_session.sh \
 "t_stem|300|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -k 'stem_bn_fused or shortcut_compact' -x -v --timeout 120 --timeout-method thread" \
 "ab|900|tools/bench_ab.sh 3 'base|' 'sbf|--opt stem_bn_fuse=1' 'wh128|--opt wgrad_halo=128' 'wh192|--opt wgrad_halo=192'" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03e -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt stem_bn_fuse=1"
