tools/gpu_session.sh \
 "ab|1000|tools/bench_ab.sh 4 'base|' 'lazy|--opt fork_lazy=1' 'prio|--opt side_prio=1' 'lazyprio|--opt fork_lazy=1 --opt side_prio=1' 'st3|--opt igemm_stages=3'"
