tools/gpu_session.sh \
 "gputest|900|python -X faulthandler -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|400|python bench.py > gpurun_out/r03u_bench.json"
