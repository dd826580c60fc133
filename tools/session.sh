# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04e_bench|300|python bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/r04e_bench.json" \
  "r04e_ser|300|tools/prof_run.sh r04e_ser --opt bwd_streams=0 --opt graphs=0" \
  "r04e_base|300|tools/prof_run.sh r04e_base" \
  "r04e_sime|300|tools/prof_run.sh r04e_sime --sim-world 2 --global-batch 512 --sim-comm loopback --opt graphs=2" \
  "r04e_pmc|400|tools/pmc_conv.sh r04e l2,l1 fwd,dgrad halo_conv=1 && python tools/pmc_report.py gpurun_out/pmc_r04e > gpurun_out/r04e_pmc.txt && rm -rf gpurun_out/pmc_r04e"
