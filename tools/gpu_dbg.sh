export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base4.so split-learning-k8s_amd/splitcnn/libslk.so build_abl/fwdhot.so --ops dgc1,fwdi --rounds 25 > gpurun_out/ab.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.txt 2>&1; rc=$?; cat gpurun_out/ab.txt; tail -15 gpurun_out/t.txt | grep -E "passed|failed|assert|Error"; exit $rc
