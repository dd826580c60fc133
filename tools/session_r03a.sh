tools/gpu_session.sh \
 "t1|300|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -v --timeout 120 --timeout-method thread -k 'compact or teacher_forced_config2 or free_running'" \
 "gputest|900|python -X faulthandler -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "ab|600|tools/bench_ab.sh 3 'base|' 'nocmp|--opt sc_compact=0'"
