PY_ARGS="--layers l2,l3,l4 --passes fwd,dgrad" tools/gpu_run.sh r05j py:tools/phase_probe.py && tools/gpu_run.sh r05j "tests:data_parallel_step" tests
