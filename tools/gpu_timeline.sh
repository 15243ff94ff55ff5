export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-k5 --no-conv-compare --no-hub-loopback --no-kernel-pass > gpurun_out/tl.log 2>&1; echo "rc=$?"
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1); echo $f; python tools/timeline.py $f --steps 3
