# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "t|600|python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'c64 or bn_fused or general_geometry'" \
  "cb|400|python tools/conv_bench.py --batch 64 --scale 7 --layers l1 --passes fwd,dgrad,dgradr --variants 'c64_gen=1;c64_gen=0' > gpurun_out/r03af_cb.txt" \
  "ab|900|tools/bench_ab.sh 2 'c5|--batch 512 --size 224 --steps 10 --warmup 3' 'c5g0|--batch 512 --size 224 --steps 10 --warmup 3 --opt c64_gen=0'"
