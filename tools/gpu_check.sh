# GPU-box check after a kernel change: chosen tests (TESTS) then a short bench; stops after a crash/timeout
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_x3_gpu.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-k5 ${BENCH_EXTRA:---no-conv-compare --no-hub-loopback} > gpurun_out/b.log 2>&1; echo "bench rc=$?"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernels": {[^}]*}' gpurun_out/b.log
