tools/gpu_session.sh \
 "gE|900|python -X faulthandler -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread"
