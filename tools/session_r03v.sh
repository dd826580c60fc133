tools/gpu_session.sh \
 "ab|800|tools/bench_ab.sh 6 'base|' 'nhb2|--opt halo_nhb2=1' 'wpf5|--opt wgrad_pf=5'"
