export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/prof_ng
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ng -o run --output-format csv -- python bench.py --config k2 --no-k5 --steps 10 --warmup 3 --no-cpu-baseline --no-conv-compare --no-hub-loopback --no-graph > gpurun_out/prof_ng.log 2>&1; rc=$?
python3 - <<'PY'
import csv, glob, json
for l in open("gpurun_out/prof_ng.log"):
    if l.startswith("{"):
        d = json.loads(l); print("events kernels", d.get("kernels"), "ms/step", round(d["ms_per_step"], 4))
f = glob.glob("gpurun_out/prof_ng/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(t in r["Name"] for t in ("x3_kernel<true>", "fc_head16", "fc_wgrad", "conv1_fwd_x3")):
        print("rocprof", r["Name"][:44], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4))
PY
exit $rc
