tools/gpu_session.sh \
 "all|600|python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread" \
 "bench|300|python bench.py --steps 50 --warmup 10 > gpurun_out/r02_bench.json" \
 "bench224|400|python bench.py --batch 512 --size 224 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-probe > gpurun_out/r02_bench224.json" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02a -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline" \
 "prof224|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02_224 -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --batch 512 --size 224 --steps 3 --warmup 2 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
