tools/gpu_session.sh \
 "t_sc|300|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -k 'shortcut_fused or stem_bn_fused or head_direct' -x -v --timeout 120 --timeout-method thread" \
 "gputest|600|python -X faulthandler -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "ab|1000|tools/bench_ab.sh 4 'base|' 'sc1|--opt sc_fuse=1' 'sc2|--opt sc_fuse=2' 'hd|--opt head_direct=1'"
