# round-3 record session: suite, smoke, PMC conv traffic, config-2 bench + trace, config-3 per-rank shapes,
# config-5 bench + trace (all steps under tools/gpu_session.sh: stops on a crash / hang)
T=r03u
R=$GRAFT_REPO_ROOT
Q="--no-cpu-baseline --no-live-roofline --no-hbm-probe"
B5="--batch 512 --size 224 --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-probe"
tools/gpu_session.sh \
  "${T}_tests|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "${T}_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "${T}_pmcf|150|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_${T}_fetch -o run -- python3 $R/bench.py --steps 10 --warmup 3 $Q" \
  "${T}_pmcw|150|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_${T}_write -o run -- python3 $R/bench.py --steps 10 --warmup 3 $Q" \
  "${T}_traffic|60|python tools/pmc_traffic.py gpurun_out/pmc_${T}_fetch gpurun_out/pmc_${T}_write gpurun_out/${T}_conv_traffic.json && cp gpurun_out/${T}_conv_traffic.json profiles/" \
  "${T}_benchrun|500|python bench.py > gpurun_out/${T}_bench.json" \
  "${T}_prof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T} -o prof -- python3 $R/bench.py --steps 20 --warmup 5 $Q" \
  "${T}_c3_w2|300|python bench.py --global-batch 256 --sim-world 2 --no-cpu-baseline > gpurun_out/${T}_c3_w2_bench.json" \
  "${T}_c3_w4|300|python bench.py --global-batch 256 --sim-world 4 --no-cpu-baseline > gpurun_out/${T}_c3_w4_bench.json" \
  "${T}_c3_w8|300|python bench.py --global-batch 256 --sim-world 8 --no-cpu-baseline > gpurun_out/${T}_c3_w8_bench.json" \
  "${T}_c5|500|python bench.py $B5 > gpurun_out/${T}_c5_bench.json" \
  "${T}_c5prof|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c5 -o prof -- python3 $R/bench.py --batch 512 --size 224 --steps 3 --warmup 1 $Q"
