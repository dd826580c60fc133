tools/gpu_session.sh \
 "stemb|120|python tools/stem_bench.py" \
 "prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r03k -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe --opt sc_fuse=2 --opt head_direct=1" \
 "ab|1000|tools/bench_ab.sh 4 'base|' 'sc2hd|--opt sc_fuse=2 --opt head_direct=1'"
