# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
PMC="timeout -s KILL 120 rocprofv3 --output-format csv"
PROF="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats"
BQ="--steps 20 --warmup 5 --no-cpu-baseline --no-live-roofline --no-hbm-probe"
tools/gpu_session.sh \
  "tests|900|python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "wb|300|python tools/wgrad_bench.py --check --variants 'wgrad_pmap=0;wgrad_pmap=1;wgrad_pmap=1,wgrad_stages=5;wgrad_pmap=0,wgrad_stages=5' > gpurun_out/r03m_wb.txt" \
  "pmc1|150|cd /tmp && export TMPDIR=/tmp && $PMC --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d \$GRAFT_REPO_ROOT/gpurun_out/pmc_wg3 -o run -- python3 \$GRAFT_REPO_ROOT/tools/wgrad_bench.py --iters 5" \
  "pmc2|150|cd /tmp && export TMPDIR=/tmp && $PMC --pmc SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d \$GRAFT_REPO_ROOT/gpurun_out/pmc_wg4 -o run -- python3 \$GRAFT_REPO_ROOT/tools/wgrad_bench.py --iters 5" \
  "cb|300|python tools/conv_bench.py --layers l1,l2,l3,l4 --passes fwd,dgrad --variants 'halo_conv=1;halo_conv=9,halo_split=1;halo_conv=6,halo_split=1;halo_stage_epi=0' > gpurun_out/r03m_cb.txt" \
  "profb|300|$PROF -d \$GRAFT_REPO_ROOT/gpurun_out/prof_bnbm -o prof -- python3 \$GRAFT_REPO_ROOT/bench.py $BQ --opt bnb_mask=1" \
  "prof0|300|$PROF -d \$GRAFT_REPO_ROOT/gpurun_out/prof_m0 -o prof -- python3 \$GRAFT_REPO_ROOT/bench.py $BQ" \
  "ab|900|tools/bench_ab.sh 5 'base|' 'pm0|--opt wgrad_pmap=0' 'bnbm|--opt bnb_mask=1' 'st5|--opt wgrad_stages=5' 'nst|--opt halo_stage_epi=0'"
