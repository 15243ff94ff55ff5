# FETCH_SIZE calibration (tools/ubench/fetch_cal.hip): one rocprofv3 --pmc pass per access pattern
export TMPDIR=/tmp; mkdir -p gpurun_out/fcal
for k in w16 w4 dy4 dy1; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fcal/$k -o run --output-format csv -- ./tools/ubench/fetch_cal $k > gpurun_out/fcal/$k.log 2>&1 || { echo "fail $k"; exit 1; }
  f=$(find gpurun_out/fcal/$k -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$k" gpurun_out/fcal/$k.log <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
vals = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == "FETCH_SIZE"]
b = float(open(sys.argv[3]).read().split("bytes_read_per_launch")[1].split()[0])
print(sys.argv[2], "dispatches", len(vals), "FETCH_SIZE KB per launch", [round(v) for v in vals], "bytes read", b,
      "ratio (FETCH KB*1024 / bytes)", [round(v * 1024 / b, 3) for v in vals])
PY
done
