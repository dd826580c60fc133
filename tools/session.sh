# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
R=${GRAFT_REPO_ROOT:-$(pwd)}
Q="--no-cpu-baseline --no-live-roofline --no-hbm-probe"
P="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats"
tools/gpu_session.sh \
  "r04a_bench|300|python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench.json" \
  "r04a_prof|300|$P -d $R/gpurun_out/prof_r04a -o prof -- python3 $R/bench.py --steps 20 --warmup 5 $Q" \
  "r04a_ser_prof|300|$P -d $R/gpurun_out/prof_r04a_ser -o prof -- python3 $R/bench.py --steps 20 --warmup 5 $Q --opt bwd_streams=0" \
  "r04a_sim2|300|python bench.py --sim-world 2 --global-batch 512 --no-cpu-baseline > gpurun_out/r04a_sim2_bench.json" \
  "r04a_sim2_prof|300|$P -d $R/gpurun_out/prof_r04a_sim2 -o prof -- python3 $R/bench.py --steps 20 --warmup 5 $Q --sim-world 2 --global-batch 512" \
  "r04a_tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
