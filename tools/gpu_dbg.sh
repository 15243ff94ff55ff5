export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python tools/x3_ab.py build_abl/prev.so split-learning-k8s_amd/splitcnn/libslk.so --ops dgc1 --rounds 25 > gpurun_out/ab.txt 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_new -o pmc --output-format csv -- python3 tools/x3_ab.py split-learning-k8s_amd/splitcnn/libslk.so --ops dgc1 --rounds 3 > gpurun_out/pmc_new.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.txt 2>&1; rc=$?; cat gpurun_out/ab.txt; tail -2 gpurun_out/t.txt
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_new/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "dgrad_x3" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("new", {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
exit $rc
