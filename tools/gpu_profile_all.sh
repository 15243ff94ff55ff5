#!/bin/bash
# One GPU-box pass for a round's evidence: all -m gpu tests, smoke, the default bench (K2 headline +
# K5 side object, with CPU baseline), rocprofv3 kernel stats of the K2 and K5 benches, and the PMC
# passes (tools/pmc.sh) for both configs. Stops after any crash/timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2, stopping"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; stop_if_fatal $rc bench
timeout -k 10 300 python -u bench.py --config k5 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k5.log 2>&1
rc=$?; echo "bench k5 rc=$rc"; stop_if_fatal $rc bench_k5
for cfg in k2 k5; do
  # graph-replayed steps, as benched: round 6 measured the profiled process within 0.1-0.7 % of an unprofiled
  # run on the same box (profiles/r06_final*_bench_unprofiled_same_box.txt); rounds 4-5 profiled eager steps
  # because the graph step then ran ~1/3 slower under --kernel-trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- python bench.py --config $cfg --no-k5 --steps 50 --warmup 5 --no-cpu-baseline --no-conv-compare --no-hub-loopback --no-dropin > gpurun_out/prof_$cfg.log 2>&1
  rc=$?; echo "rocprof $cfg rc=$rc"; stop_if_fatal $rc rocprof
  # the library build this profile belongs to (bench.py reports rocprof_avg_ms only for a matching build)
  python -c "import sys; sys.path.insert(0, 'split-learning-k8s_amd'); from splitcnn import _lib; print(_lib.build_id())" > gpurun_out/prof_$cfg.build_id
  # the profiled process's own JSON line (bench.py reads it as roofline.rocprof_process)
  grep '^{' gpurun_out/prof_$cfg.log | tail -1 > gpurun_out/prof_$cfg.bench.json || true
  OUT=gpurun_out/pmc_$cfg KARGS="--config $cfg --steps 3" bash tools/pmc.sh || exit $?
  python tools/pmc_summary.py --dir gpurun_out/pmc_$cfg --out gpurun_out/pmc_${cfg}_summary.json > /dev/null
done
