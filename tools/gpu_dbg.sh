export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base13.so build_abl/fcwu4.so build_abl/fcwu16.so --ops fcw,fc --rounds 20 --flush > gpurun_out/ab.txt 2>&1; rc=$?; cat gpurun_out/ab.txt; exit $rc
