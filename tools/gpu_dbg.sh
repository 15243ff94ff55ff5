export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base2.so split-learning-k8s_amd/splitcnn/libslk.so --ops c1x3 --rounds 30 > gpurun_out/ab_c1.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-k5 --no-conv-compare --no-hub-loopback > gpurun_out/b.log 2>&1; rc=$?
cat gpurun_out/ab_c1.txt; tail -2 gpurun_out/t.txt
python3 - <<'PY'
import json
for l in open("gpurun_out/b.log"):
    if l.startswith("{"):
        d = json.loads(l); print("value", d["value"], "ms", d["ms_per_step"], "kernels", d.get("kernels"))
PY
exit $rc
