# scratch GPU session (overwritten per session; see tools/gpu_run.sh for the standard steps)
tools/gpu_session.sh \
  "r04ag_hp32|200|python tools/host_phases.py --batch 32 --loopback 8 --steps 100" \
  "r04ag_hp32p|200|python tools/host_phases.py --batch 32 --loopback 8 --steps 100 --cprofile" \
  "r04ag_hp256|200|python tools/host_phases.py --batch 256 --steps 100"
