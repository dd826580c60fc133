AB_ROUNDS=5 tools/gpu_run.sh r05q "ab:base|;df0|--opt dgrad_first=0" && tools/gpu_run.sh r05q tests
