export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base11.so build_abl/wreg.so --ops fc,fc3 --rounds 30 > gpurun_out/ab.txt 2>&1; rc=$?; cat gpurun_out/ab.txt; exit $rc
