# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
B5="--batch 512 --size 224 --steps 5 --warmup 2 --no-cpu-baseline --no-hbm-probe --no-live-roofline"
tools/gpu_session.sh \
  "tests|400|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_resnet.py -m gpu -q -x --timeout 200 --timeout-method thread -k 'stride2 or s2 or 224 or general or staged'" \
  "ab5|900|tools/bench_ab.sh 2 'c5|$B5' 'c5w0|$B5 --opt wgrad_s2=0' 'c5bm|$B5 --opt bnb_mask=1'"
