# Multi-rank rehearsal of bench.py on a 1-GPU box: every rank on cuda:0 over gloo (never for numbers).
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-2}
SLK_BENCH_TRACE_AFTER=${TRACE_AFTER:-150} SLK_BENCH_BACKEND=gloo SLK_BENCH_ONE_GPU=1 timeout -k 10 ${TLIM:-300} python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $N --steps ${STEPS:-5} --warmup 2 --k5-batch 512 ${ARGS:-} > gpurun_out/reh$N.log 2>&1
rc=$?; echo "rehearsal N=$N rc=$rc"; tail -1 gpurun_out/reh$N.log | cut -c1-1500; exit $rc
