tools/gpu_session.sh \
 "t_iso|200|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -x -q --timeout 120 --timeout-method thread -k live_conv_profile" \
 "t_res|600|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -x -v --timeout 300 --timeout-method thread"
