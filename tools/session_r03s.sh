tools/gpu_session.sh \
 "gputest|900|python -X faulthandler -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|400|python bench.py > gpurun_out/r03s_bench.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03s -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
