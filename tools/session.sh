tools/gpu_run.sh r05h tests bench && timeout -k 10 300 tools/prof_run.sh r05h_ser --opt bwd_streams=0 --opt graphs=0 && timeout -k 10 300 tools/prof_run.sh r05h_b256
