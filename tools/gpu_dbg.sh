export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in base2 dgnowrite dgnoload; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/pmc_$lib -o pmc --output-format csv -- python3 tools/x3_ab.py build_abl/$lib.so --ops dgc1 --rounds 3 > gpurun_out/pmc_$lib.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for lib in ("base2", "dgnowrite", "dgnoload"):
    f = glob.glob(f"gpurun_out/pmc_{lib}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "dgrad_x3" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(lib, {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
