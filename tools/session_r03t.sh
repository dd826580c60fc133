tools/gpu_session.sh \
 "ab|700|tools/bench_ab.sh 6 'base|' 'prio|--opt side_prio=1'"
