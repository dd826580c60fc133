tools/gpu_session.sh \
 "cbslp|300|DTC_LIB=$GRAFT_REPO_ROOT/distributed-training-comparison_amd/_lib_slp/libdtc_amd.so python tools/conv_bench.py --variants 'halo_conv=1' --passes fwd,dgrad" \
 "cbnoslp|300|python tools/conv_bench.py --variants 'halo_conv=1' --passes fwd,dgrad" \
 "ab|700|tools/bench_ab.sh 3 'noslp|' 'slp|ENV:DTC_LIB=$GRAFT_REPO_ROOT/distributed-training-comparison_amd/_lib_slp/libdtc_amd.so;'"
