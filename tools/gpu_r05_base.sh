#!/bin/bash
# Round-5 baseline pass: all -m gpu tests, smoke, the default bench. Stops after any crash/timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2, stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; stop_if_fatal $rc bench
tail -c 3000 gpurun_out/bench.log
