export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/r03_base.so split-learning-k8s_amd/splitcnn/libslk.so --ops dgc1 --rounds 20 && \
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_gpu_parity.py tests/test_fc_gpu.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3 && \
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-k5 --no-conv-compare --no-hub-loopback > gpurun_out/b.log 2>&1; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernels": {[^}]*}' gpurun_out/b.log
