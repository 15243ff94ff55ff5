#!/bin/bash
# Profiling only: time x3 kernel ablation variants (tools/build_variant.sh x3aN "-DSLK_X3ABL=N") one
# process each; usage: tools/abl_x3.sh OPS N1 N2 ...  (writes gpurun_out/abl.log)
set -e
mkdir -p gpurun_out
OPS=$1; shift
echo "== base" >> gpurun_out/abl.log
timeout -k 10 120 python -u tools/x3_time.py --ops $OPS --rounds 20 >> gpurun_out/abl.log 2>&1
for v in "$@"; do
  echo "== $v" >> gpurun_out/abl.log
  SLK_LIB_VARIANT=build_abl/x3a$v.so timeout -k 10 120 python -u tools/x3_time.py --ops $OPS --rounds 20 >> gpurun_out/abl.log 2>&1
done
