tools/gpu_session.sh \
 "gputest|900|python -u -m pytest tests/test_gpu_resnet.py tests/test_gpu_ops.py tests/test_gpu_fp32.py -x -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --no-cpu-baseline > gpurun_out/r02i_bench.json" \
 "bench_nostr|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 > gpurun_out/r02i_bench_nostr.json" \
 "bench_no1p|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bn_onepass=0 > gpurun_out/r02i_bench_no1p.json" \
 "bench_nostr_no1p|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 --opt bn_onepass=0 > gpurun_out/r02i_bench_nostr_no1p.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02i -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0"
