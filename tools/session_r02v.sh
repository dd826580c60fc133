tools/gpu_session.sh \
 "gA|900|DTC_OPTIONS=head_fused=0,stem_prologue=0,dgrad_class_order=0 python -X faulthandler -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread"
