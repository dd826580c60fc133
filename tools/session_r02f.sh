tools/gpu_session.sh \
 "gputest|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "wgb|300|python tools/wgrad_bench.py --check --variants 'wgrad_direct=0;wgrad_direct=1;wgrad_xcd=1;wgrad_stages=4;wgrad_stages=4,wgrad_xcd=1;wgrad_pf=8,wgrad_stages=4;wgrad_kernel=1;wgrad_diag=1;wgrad_diag=2;wgrad_diag=3'" \
 "cb|300|python tools/conv_bench.py --variants 'halo_conv=1' --passes fwd,dgrad,dgradr" \
 "bench|300|python bench.py --no-cpu-baseline > gpurun_out/r02f_bench.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02f -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
