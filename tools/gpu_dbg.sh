export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/ablate_wide.py build_abl/base10.so build_abl/headnored.so --rounds 7 --reps 5 > gpurun_out/ab.txt 2>&1; rc=$?; python3 -c "
import json; d=json.load(open('gpurun_out/ab.txt'))
for k,v in d.items(): print(k.split('/')[-1], {n: x['ms'] for n, x in v.items() if n.startswith('head')})"; exit $rc
