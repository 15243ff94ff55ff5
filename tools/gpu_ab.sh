# A/B of libslk variant builds (build_abl/*.so) in one process: LIBS="..." OPS="..." bash tools/gpu_ab.sh
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/x3_ab.py $LIBS --ops ${OPS:-fwdi} --rounds ${ROUNDS:-60} > gpurun_out/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep "median\|check" gpurun_out/ab.log || tail -20 gpurun_out/ab.log
