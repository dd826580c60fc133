tools/gpu_session.sh \
 "gputest|600|python -X faulthandler -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03g -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe" \
 "ab|1000|tools/bench_ab.sh 3 'base|' 'sbf|--opt stem_bn_fuse=1' 'fa256|--opt bn_fa_blocks=256' 'red64|--opt bn_red_elems=65536 --opt bn_red_blocks=64'"
