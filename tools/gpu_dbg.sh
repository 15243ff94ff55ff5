export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base12.so build_abl/c1split.so --ops c1x3 --rounds 30 > gpurun_out/ab.txt 2>&1; rc=$?; cat gpurun_out/ab.txt; exit $rc
