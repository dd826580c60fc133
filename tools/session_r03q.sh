tools/gpu_session.sh \
 "hp|200|python tools/host_phases.py --steps 50" \
 "hpc|200|python tools/host_phases.py --steps 30 --cprofile"
