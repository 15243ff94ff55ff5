export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/x3_ab.py build_abl/r02.so build_abl/r03_base.so build_abl/fe1.so build_abl/fe2.so --ops fwdi,dgc1,wgrad,fc,c1x3 --rounds 40 > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log | tail -12
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-k5 > gpurun_out/b2.log 2>&1; echo "bench rc=$?"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernels": {[^}]*}\|"conv_presets": {[^}]*}' gpurun_out/b2.log
