export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t.txt 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/t.txt | tail -30; exit $rc
