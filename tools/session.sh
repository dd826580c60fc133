# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04ab_ab|700|tools/bench_ab.sh 4 'base|' 'c192|--opt c64_wgs=192' 'c384|--opt c64_wgs=384' 'c512|--opt c64_wgs=512' 'c128|--opt c64_wgs=128'"
