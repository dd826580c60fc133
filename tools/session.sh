# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04b_bench|300|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04b_bench.json" \
  "r04b_prof|300|tools/prof_run.sh r04b" \
  "r04b_ser|300|tools/prof_run.sh r04b_ser --opt bwd_streams=0" \
  "r04b_sim2|300|python bench.py --sim-world 2 --global-batch 512 --no-cpu-baseline --no-hbm-probe > gpurun_out/r04b_sim2_bench.json" \
  "r04b_sim2e|300|python bench.py --sim-world 2 --global-batch 512 --no-cpu-baseline --no-hbm-probe --opt graphs=2 > gpurun_out/r04b_sim2e_bench.json" \
  "r04b_sim2_prof|300|tools/prof_run.sh r04b_sim2 --sim-world 2 --global-batch 512" \
  "r04b_sim2e_prof|300|tools/prof_run.sh r04b_sim2e --hip --sim-world 2 --global-batch 512 --opt graphs=2" \
  "r04b_s2cb|300|python tools/conv_bench.py --passes wgrad --layers l2.0.c1,l3.0.c1,l4.0.c1,l2.sc,l3.sc,l4.sc --variants 'wgrad_s2=2;wgrad_s2=1;wgrad_s2=1,wgrad_s2_wgs=128;wgrad_s2=1,wgrad_s2_wgs=64' > gpurun_out/r04b_s2cb.txt"
