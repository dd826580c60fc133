# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "cb|400|python tools/conv_bench.py --layers l3,l4 --passes fwd,dgrad --variants 'halo_conv=1;halo_conv=6,halo_split=2;halo_conv=6,halo_split=4;halo_conv=6,halo_split=1;halo_conv=7,halo_split=2;halo_conv=4,halo_split=4;halo_conv=9,halo_split=1;halo_conv=9,halo_split=2;halo_conv=8,halo_split=2' > gpurun_out/r03z_cb.txt"
