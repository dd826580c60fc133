tools/gpu_session.sh \
 "t_wl|300|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -k 'stem_weight_lds or live_conv_profile' -x -v --timeout 120 --timeout-method thread" \
 "stemb|120|python tools/stem_bench.py" \
 "ab|700|tools/bench_ab.sh 4 'base|' 'wl|--opt stem_wlds=1'"
