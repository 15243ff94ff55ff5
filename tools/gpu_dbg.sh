export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base2.so split-learning-k8s_amd/splitcnn/libslk.so --ops fc,fc3 --rounds 30 > gpurun_out/ab_fc.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.txt 2>&1; rc=$?; cat gpurun_out/ab_fc.txt; tail -4 gpurun_out/t.txt; exit $rc
