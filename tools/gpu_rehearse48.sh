#!/bin/bash
# gloo rehearsal of bench.py at N = 4 and 8 on one GPU (K4 with 3 and 7 clients; numbers meaningless).
export TMPDIR=/tmp; mkdir -p gpurun_out
for n in 4 8; do
  N=$n ARGS="--batch 512 --exchange-steps 3 --k5-batch 256" TRACE_AFTER=240 bash tools/gpu_rehearse.sh
  rc=$?; case $rc in 0) ;; *) echo "stop rc=$rc"; exit $rc;; esac
done
