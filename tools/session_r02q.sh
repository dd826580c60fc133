tools/gpu_session.sh \
 "ab|300|python tools/option_ab.py --batch 64 --passes dgrad --variants 'dgrad_class_order=0;dgrad_class_order=1'" \
 "cb|300|python tools/conv_bench.py --layers l2.0.c1,l3.0.c1,l4.0.c1 --passes dgrad,dgradr --variants 'dgrad_class_order=0;dgrad_class_order=1'"
