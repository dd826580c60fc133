tools/gpu_session.sh \
 "t_amp|300|python -X faulthandler -u -m pytest tests/test_gpu_resnet.py -k 'scaled_loss or native_loss or amp or scaler or loss_curve' -x -q --timeout 200 --timeout-method thread" \
 "hp|200|python tools/host_phases.py --steps 50" \
 "bench|400|python bench.py > gpurun_out/r03r_bench.json" \
 "bench2|400|python bench.py --no-cpu-baseline > gpurun_out/r03r_bench2.json"
