tools/gpu_session.sh \
 "gputest|600|python -X faulthandler -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "t_lazy|200|DTC_OPTIONS=fork_lazy=1 python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 120 --timeout-method thread -k 'wgrad_batch or ddp or bucket or graph'" \
 "ab|1000|tools/bench_ab.sh 3 'base|' 'lazy|--opt fork_lazy=1' 're8k|--opt bn_red_elems=8192' 'rb512|--opt bn_red_blocks=512'"
