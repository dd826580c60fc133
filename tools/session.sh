# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
W2='--sim-world 2 --global-batch 256 --sim-comm loopback'
W4='--sim-world 4 --global-batch 256 --sim-comm loopback'
S8='--sim-world 8 --global-batch 256 --sim-comm loopback'
tools/gpu_session.sh \
  "r04h_ab|1000|tools/bench_ab.sh 3 'w2|$W2' 'w2e|$W2 --opt graphs=2' 'w4|$W4' 'w4e|$W4 --opt graphs=2' 'w8|$S8' 'w8e|$S8 --opt graphs=2'" \
  "r04h_cb32|300|python tools/conv_bench.py --batch 32 --passes fwd,dgrad --layers l2,l3,l4,l3.0.c1,l4.0.c1 --variants 'halo_split=0;halo_split=1' > gpurun_out/r04h_cb32.txt" \
  "r04h_w8prof|300|tools/prof_run.sh r04h_w8 $S8"
