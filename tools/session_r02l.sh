tools/gpu_session.sh \
 "gputest|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --no-cpu-baseline > gpurun_out/r02l_bench.json" \
 "bench_nostr|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 > gpurun_out/r02l_bench_nostr.json" \
 "bench2|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe > gpurun_out/r02l_bench2.json" \
 "bench_nostr2|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 > gpurun_out/r02l_bench_nostr2.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02l -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
