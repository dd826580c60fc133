tools/gpu_session.sh \
 "cbs2|400|python tools/conv_bench.py --layers l2.0.c1,l2.sc,l3.0.c1,l3.sc,l4.0.c1,l4.sc --passes fwd,dgrad,wgrad --variants 'igemm_tile=0;igemm_stages=3;igemm_tile=1;igemm_tile=2;igemm_tile=2,igemm_split=2;igemm_tile=2,igemm_split=4;igemm_tile=1,igemm_split=2;igemm_tile=3;igemm_tile=2,igemm_stages=3,igemm_split=2;igemm_tile=1,igemm_stages=3,igemm_split=4'"
