tools/gpu_session.sh \
 "gputest|900|python -X faulthandler -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "ab|600|tools/bench_ab.sh 3 'base|' 'nohead|--opt head_fused=0' 'noclass|--opt dgrad_class_order=0'"
