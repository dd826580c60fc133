# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04al_ab|600|tools/bench_ab.sh 3 'base|' 'q2|ENV:GPU_MAX_HW_QUEUES=2;' 'q3|ENV:GPU_MAX_HW_QUEUES=3;' 'q8|ENV:GPU_MAX_HW_QUEUES=8;'"
