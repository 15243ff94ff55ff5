#!/bin/bash
# GPU-box sequence: parity tests -> bench -> rocprofv3 kernel trace. Stops after any crash/timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2, stopping"; exit "$1";; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 30 --warmup 5} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; stop_if_fatal $rc bench
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-pass > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; stop_if_fatal $rc rocprof
  find gpurun_out/prof -name '*stats*' | head
fi
