export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/base8.so build_abl/wgnody.so build_abl/wgnodma.so build_abl/wgnoboth.so --ops wgrad --rounds 25 > gpurun_out/ab.txt 2>&1; rc=$?; cat gpurun_out/ab.txt; exit $rc
