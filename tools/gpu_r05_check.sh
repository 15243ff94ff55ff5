#!/bin/bash
# Round-5 check: all -m gpu tests, smoke, default bench, gloo rehearsals of the N > 1 bench at N = 2 and 4,
# then a forced stall in the K5 phase at N = 2 (expects the watchdog's partial JSON and rc != 0).
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2, stopping"; exit "$1";; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; stop_if_fatal $rc smoke
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; stop_if_fatal $rc bench
grep '^{' gpurun_out/bench.log | cut -c1-600
fi
for N in 2 4; do
  SLK_BENCH_BACKEND=gloo SLK_BENCH_ONE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --steps 5 --warmup 2 --batch 512 --k5-batch 512 > gpurun_out/reh$N.log 2>&1
  rc=$?; echo "rehearsal N=$N rc=$rc"; stop_if_fatal $rc reh$N
  grep '^{' gpurun_out/reh$N.log | cut -c1-400
done
SLK_BENCH_STALL=k5_splitfed SLK_BENCH_WATCHDOG_SCALE=0.15 SLK_BENCH_BACKEND=gloo SLK_BENCH_ONE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 5 --warmup 2 --batch 512 --k5-batch 512 > gpurun_out/reh_stall.log 2>&1
rc=$?; echo "stall rehearsal rc=$rc (expected != 0)"
grep '^{' gpurun_out/reh_stall.log | cut -c1-300; grep -c "watchdog" gpurun_out/reh_stall.log
