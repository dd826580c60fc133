tools/gpu_session.sh \
 "gputest|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --no-cpu-baseline > gpurun_out/r02m_bench.json" \
 "bench_nosc|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt sc_stream=0 > gpurun_out/r02m_bench_nosc.json" \
 "bench_nostr|200|python bench.py --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt bwd_streams=0 > gpurun_out/r02m_bench_nostr.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02m -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
