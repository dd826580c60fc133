# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
AB_ROUNDS=4 tools/gpu_run.sh r03am tests "ab:auto|;g1|--opt graphs=1;b64a|--batch 64;b64g1|--batch 64 --opt graphs=1"
