# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S2='--sim-world 2 --global-batch 512 --sim-comm loopback'
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04f_ab|1000|tools/bench_ab.sh 3 'base|' 'sime|$S2 --opt graphs=2' 'simeq|ENV:GPU_MAX_HW_QUEUES=8;$S2 --opt graphs=2' 'simrq|ENV:GPU_MAX_HW_QUEUES=8;$S2' 'baseq|ENV:GPU_MAX_HW_QUEUES=8;' 'w8cg|$S8' 'w8nocg|$S8 --opt bn_cg=0'"
