#!/bin/bash
# GPU check after a change: the named tests (TESTS), then a short K2 bench line and a kernel-trace timeline.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests -m gpu} -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-k5 ${BENCH_EXTRA:---no-conv-compare --no-hub-loopback} > gpurun_out/b.log 2>&1; echo "bench rc=$?"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"kernels": {[^}]*}' gpurun_out/b.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-k5 --no-conv-compare --no-hub-loopback --no-kernel-pass > gpurun_out/tl.log 2>&1; echo "rocprof rc=$?"
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1); python tools/timeline.py $f --steps 2
