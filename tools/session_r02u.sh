tools/gpu_session.sh \
 "t_pair|300|python -X faulthandler -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resnet.py -v --timeout 120 --timeout-method thread -k 'onepass or live_conv_profile'"
