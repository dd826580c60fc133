# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
AB_ROUNDS=6 tools/gpu_run.sh r03ad "tests:bn_reduce_unrolled or bn_mask_bits or bn_backward or step_matches" "ab:base|;ru1|--opt bn_red_unroll=1;ru2|--opt bn_red_unroll=2" prof
