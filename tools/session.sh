# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04ac_ab|800|tools/bench_ab.sh 3 'base|' 'hs1|--opt halo_split=1' 'hs4|--opt halo_split=4' 'fa2k|--opt bn_fa_blocks=2048' 'l1_128|--opt wgrad_halo_l1=128' 'l1_160|--opt wgrad_halo_l1=160' 'l1_96|--opt wgrad_halo_l1=96'"
