# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
S2='--sim-world 2 --global-batch 512 --sim-comm loopback'
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04f_ab|1000|tools/bench_ab.sh 3 'base|' 'sime|$S2 --opt graphs=2' 'simes|$S2 --opt graphs=2 --opt comm_on_side=1' 'simeq|ENV:GPU_MAX_HW_QUEUES=8;$S2 --opt graphs=2' 'simrq|ENV:GPU_MAX_HW_QUEUES=8;$S2' 'w8cg|$S8' 'w8nocg|$S8 --opt bn_cg=0'" \
  "r04f_tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'reducer or ddp_two or bn_one or mask_bits or config3'"
