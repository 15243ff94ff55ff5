#!/bin/bash
# Round-6 evidence pass, part 1: all -m gpu tests, smoke, the default bench, the K5 bench, rocprofv3 kernel stats
# of the K2 and K5 benches (graph-replayed steps: on this image the profiled graph step runs within 1 % of the
# unprofiled one, profiles/r06_v2_rocprof_vs_plain.txt), and the PMC passes (tools/pmc.sh). Stops after any
# crash / timeout. PART=2: the multi-rank rehearsals of bench.py (gloo, one GPU) and a forced stall.
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2, stopping"; exit "$1";; esac; }
if [ "${PART:-1}" = "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; stop_if_fatal $rc bench
grep '^{' gpurun_out/bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config k5 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k5.log 2>&1
rc=$?; echo "bench k5 rc=$rc"; stop_if_fatal $rc bench_k5
for cfg in k2 k5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$cfg -o run --output-format csv -- python bench.py --config $cfg --no-k5 --steps 50 --warmup 5 --no-cpu-baseline --no-conv-compare --no-hub-loopback --no-dropin > gpurun_out/prof_$cfg.log 2>&1
  rc=$?; echo "rocprof $cfg rc=$rc"; stop_if_fatal $rc rocprof
  python -c "import sys; sys.path.insert(0, 'split-learning-k8s_amd'); from splitcnn import _lib; print(_lib.build_id())" > gpurun_out/prof_$cfg.build_id
  grep '^{' gpurun_out/prof_$cfg.log | tail -1 > gpurun_out/prof_$cfg.bench.json || true
  OUT=gpurun_out/pmc_$cfg KARGS="--config $cfg --steps 3" bash tools/pmc.sh || exit $?
  python tools/pmc_summary.py --dir gpurun_out/pmc_$cfg --out gpurun_out/pmc_${cfg}_summary.json > /dev/null
done
elif [ "${PART}" = "3" ]; then
# the K2 rocprofv3 kernel-stats pass alone (same command as in part 1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k2 -o run --output-format csv -- python bench.py --config k2 --no-k5 --steps 50 --warmup 5 --no-cpu-baseline --no-conv-compare --no-hub-loopback --no-dropin > gpurun_out/prof_k2.log 2>&1
rc=$?; echo "rocprof k2 rc=$rc"; stop_if_fatal $rc rocprof
python -c "import sys; sys.path.insert(0, 'split-learning-k8s_amd'); from splitcnn import _lib; print(_lib.build_id())" > gpurun_out/prof_k2.build_id
grep '^{' gpurun_out/prof_k2.log | tail -1 > gpurun_out/prof_k2.bench.json || true
timeout -k 10 400 python -u bench.py --no-k5 --no-cpu-baseline --no-dropin --no-hub-loopback > gpurun_out/bench_after_prof.log 2>&1
echo "bench rc=$?"
else
for N in 2 4; do
  SLK_BENCH_BACKEND=gloo SLK_BENCH_ONE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2961$N bench.py --gpus $N --steps 5 --warmup 2 --batch 512 --k5-batch 512 > gpurun_out/reh$N.log 2>&1
  rc=$?; echo "rehearsal N=$N rc=$rc"; stop_if_fatal $rc reh$N
  grep '^{' gpurun_out/reh$N.log | cut -c1-400
done
SLK_BENCH_STALL=k5_splitfed SLK_BENCH_WATCHDOG_SCALE=0.15 SLK_BENCH_BACKEND=gloo SLK_BENCH_ONE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29629 bench.py --gpus 2 --steps 5 --warmup 2 --batch 512 --k5-batch 512 > gpurun_out/reh_stall.log 2>&1
rc=$?; echo "stall rehearsal rc=$rc (expected != 0)"
grep '^{' gpurun_out/reh_stall.log | cut -c1-300; grep -c "watchdog" gpurun_out/reh_stall.log
fi
