tools/gpu_session.sh \
 "hsweep|600|python tools/conv_bench.py --layers l2,l3,l4 --passes fwd,dgrad --variants 'halo_conv=1;halo_conv=2;halo_conv=3;halo_conv=4;halo_conv=5;halo_conv=6;halo_conv=7;halo_conv=8;halo_conv=9;halo_conv=1,halo_split=1;halo_conv=1,halo_split=2;halo_conv=1,halo_split=4;halo_conv=1,halo_wstages=2;halo_conv=2,halo_split=2;halo_conv=5,halo_split=2'"
