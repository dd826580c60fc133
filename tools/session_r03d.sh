tools/gpu_session.sh \
 "ab|700|tools/bench_ab.sh 3 'base|' 'tail2|--opt wgrad_tail=2' 'tail1|--opt wgrad_tail=1'" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03d -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt wgrad_tail=2"
