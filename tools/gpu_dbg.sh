export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/bench.log"):
    if l.startswith("{"):
        d = json.loads(l); k = d.get("k4_server_loopback", {})
        print("value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "frac", d["roofline"]["frac"], "rocprof", d["roofline"].get("rocprof_avg_ms"), "events", d["roofline"]["avg_ms"])
        print("k4 codec", k.get("samples_per_s"), "dense", (k.get("dense_exchange") or {}).get("samples_per_s"), "f32", (k.get("dense_f32_cut") or {}).get("samples_per_s"), "k5", (d.get("widened") or {}).get("value"))
PY
