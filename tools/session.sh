# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_run.sh r03ac tests smoke bench
