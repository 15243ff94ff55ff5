#!/bin/bash
# Round-6 profiling pass: the K2 bench unprofiled and under rocprofv3 --kernel-trace, graph and eager, on one box
# (is the profiled process's step within 5 % of the unprofiled one?), plus the drop-in module step's kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2, stopping"; exit "$1";; esac; }
A="--config k2 --no-k5 --steps 20 --warmup 5 --no-cpu-baseline --no-conv-compare --no-hub-loopback --no-dropin"
for g in "" "--no-graph"; do
  tag=$([ -z "$g" ] && echo graph || echo eager)
  timeout -k 10 200 python -u bench.py $A $g > gpurun_out/plain_$tag.log 2>&1
  rc=$?; stop_if_fatal $rc plain_$tag
  echo "plain $tag: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/plain_$tag.log | head -1)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python bench.py $A $g > gpurun_out/prof_$tag.log 2>&1
  rc=$?; stop_if_fatal $rc prof_$tag
  echo "rocprof $tag: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof_$tag.log | head -1)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dropin -o run --output-format csv -- python tools/dropin_prof.py 20 > gpurun_out/prof_dropin.log 2>&1
rc=$?; stop_if_fatal $rc prof_dropin
tail -1 gpurun_out/prof_dropin.log | cut -c1-300
