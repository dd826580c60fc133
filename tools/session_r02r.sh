tools/gpu_session.sh \
 "gputest|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "ab|600|tools/bench_ab.sh 3 'base|' 'nohead|--opt head_fused=0' 'noclass|--opt dgrad_class_order=0'" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02r -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
