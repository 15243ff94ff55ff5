export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_trainers.py --order --rounds 12 --steps 20 > gpurun_out/ab.txt 2>&1; rc=$?; cat gpurun_out/ab.txt | tail -6; exit $rc
