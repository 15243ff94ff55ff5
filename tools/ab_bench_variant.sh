#!/bin/bash
# Profiling only: step-level A/B of the default library vs a variant build (tools/build_variant.sh),
# interleaved, K2 bench without the side objects. usage: tools/ab_bench_variant.sh build_abl/NAME.so [rounds]
set -e
V=$1; R=${2:-2}
F="--no-conv-compare --no-k5 --no-cpu-baseline --no-kernel-pass --steps 60 --warmup 10"
ms() { python3 -c "import json,sys; print('$1', json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])"; }
for i in $(seq "$R"); do
  timeout -k 10 120 python -u bench.py $F | ms base
  SLK_LIB_VARIANT=$V timeout -k 10 120 python -u bench.py $F | ms "$(basename "$V" .so)"
done
