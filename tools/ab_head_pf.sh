for v in pf1 pf2 pf4 pf1; do
  timeout -k 10 120 python -u tools/bench_with_lib.py build_abl/$v.so --config k5 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$v.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$v.log') if l.startswith('{')][-1]); print('$v', round(d['ms_per_step'],4), d['kernels']['wide_head'], d['loss_first_last'])"
done
