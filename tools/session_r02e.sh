tools/gpu_session.sh \
 "wgb|300|python tools/wgrad_bench.py --variants 'wgrad_stages=2;wgrad_stages=4;wgrad_pf=5;wgrad_stages=4,wgrad_pf=8;wgrad_kernel=1;wgrad_diag=1;wgrad_diag=2;wgrad_diag=3;wgrad_halo=512;wgrad_halo=128'" \
 "wgprof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_wgb -o prof -- python3 $GRAFT_REPO_ROOT/tools/wgrad_bench.py --variants wgrad_batch=4"
