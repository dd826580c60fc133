tools/gpu_session.sh \
 "optest|400|python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread" \
 "wgb|300|python tools/wgrad_bench.py --check --variants 'wgrad_direct=0;wgrad_direct=1;wgrad_xcd=1;wgrad_stages=4;wgrad_stages=4,wgrad_xcd=1;wgrad_pf=8,wgrad_stages=4;wgrad_kernel=1;wgrad_diag=1;wgrad_diag=2;wgrad_diag=3'" \
 "cb|300|python tools/conv_bench.py --variants 'halo_conv=1' --passes fwd,dgrad,dgradr" \
 "bench|300|python bench.py --no-cpu-baseline > gpurun_out/r02f_bench.json"
