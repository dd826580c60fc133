# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04ae_ab|600|tools/bench_ab.sh 3 'base|' 'sp0|--opt side_prio=0' 'ks3|--opt wgrad_ksplit=3' 'b128|--batch 128' 'b128hs1|--batch 128 --opt halo_split=1'" \
  "r04ae_ab8|300|tools/bench_ab.sh 2 'w8|$S8' 'w4|--sim-world 4 --global-batch 256 --sim-comm loopback' 'w2|--sim-world 2 --global-batch 256 --sim-comm loopback'"
