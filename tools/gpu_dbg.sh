export TMPDIR=/tmp; mkdir -p gpurun_out
N=2 TLIM=300 bash tools/gpu_rehearse.sh && N=3 TLIM=300 bash tools/gpu_rehearse.sh; rc=$?
for n in 2 3; do python3 - $n <<'PY'
import json, sys
n = sys.argv[1]
for l in open(f"gpurun_out/reh{n}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d.get("config", {}); e = d.get("exchange", {})
        print(n, c.get("workload", "")[:30], "| choice", e.get("choice"), "m", e.get("micro_batches"), c.get("micro_batches"), e.get("trial_ms_per_step"))
PY
done
exit $rc
