export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base.so split-learning-k8s_amd/splitcnn/libslk.so --ops dgc1 --rounds 20 && \
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
