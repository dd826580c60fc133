tools/gpu_run.sh r05zi tests smoke bench && timeout -k 10 300 tools/prof_run.sh r05zi_ser --opt bwd_streams=0 --opt graphs=0
