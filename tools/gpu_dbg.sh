export TMPDIR=/tmp; mkdir -p gpurun_out
N=2 TLIM=300 bash tools/gpu_rehearse.sh && N=3 TLIM=300 bash tools/gpu_rehearse.sh; rc=$?
for n in 2 3; do python3 - $n <<'PY'
import json, sys
n = sys.argv[1]
for l in open(f"gpurun_out/reh{n}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d.get("config", {})
        print(n, "workload", c.get("workload", "")[:40], "| exchange", d.get("exchange", {}).get("choice"), d.get("exchange", {}).get("trial_ms_per_step"), "| cut", c.get("cut_exchange", "")[:60], "| loss", d.get("loss_first_last"))
PY
done
exit $rc
