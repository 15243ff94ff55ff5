"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel: mean per dispatch over the last N
dispatches, plus derived HBM traffic (FETCH_SIZE doubled for gfx950's half-counted wide reads, per
MI355X_MICROARCH.md §HBM) and MFMA busy fraction. Writes JSON to stdout or --out."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--dir", default="gpurun_out/pmc")
ap.add_argument("--out")
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--traffic-out", help="write {kernel: {batch: corrected HBM bytes per launch}} for bench.py")
args = ap.parse_args()

vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
for f in glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d = r["Dispatch_Id"]
        names[d] = k
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, cs in per.items():
        for c, v in cs.items():
            vals[names[d]][c].append(v)
out = {}
for k, cs in vals.items():
    m = {c: sum(v[-3:]) / len(v[-3:]) for c, v in cs.items()}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        m["hbm_bytes_raw"] = (m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        m["hbm_bytes_corrected"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # MFMA busy cycles summed over all SIMDs (1024) vs GUI-active cycles (summed over 8 XCDs)
        m["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAVE_CYCLES" in m:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                m[c + "_frac_of_wave_cycles"] = m[c] / m["SQ_WAVE_CYCLES"]
    out[k] = m
if args.traffic_out:
    names = {"conv2_fwd_pool_kernel": "conv2_fwd_pool", "conv2_dgrad_kernel": "conv2_dgrad",
             "conv2_wgrad_kernel": "conv2_wgrad", "conv1_fwd_kernel": "conv1_fwd",
             "conv1_wgrad_kernel": "conv1_wgrad", "conv1_wgrad_kernel<true>": "conv1_wgrad",
             "fc_head_kernel<7>": "fc_xent", "fc_wgrad_kernel": "fc_wgrad"}
    prev = json.load(open(args.traffic_out)) if os.path.exists(args.traffic_out) else {}
    names.update({"conv2_fwd_pool_wino_kernel": "conv2_fwd_pool", "conv2_fwd_pool_wino2_kernel": "conv2_fwd_pool",
                  "conv2_dgrad_wino_kernel": "conv2_dgrad",
                  "conv2_wgrad_wino_kernel": "conv2_wgrad", "fc_head_kernel<8>": "fc_xent",
                  "conv2_fwd_pool_x3_kernel": "conv2_fwd_pool_x3", "conv2_dgrad_x3_kernel": "conv2_dgrad_x3",
                  "conv2_wgrad_x3_kernel": "conv2_wgrad_x3",
                  # round 2: the default step's instantiations (client images in) and the f32-cut ones
                  "conv2_fwd_pool_x3_kernel<true>": "conv2_fwd_pool_x3",
                  "conv2_fwd_pool_x3_kernel<false>": "conv2_fwd_pool_x3_f32in",
                  "conv2_wgrad_x3_kernel<true>": "conv2_wgrad_x3", "conv2_wgrad_x3_kernel<false>": "conv2_wgrad_x3_gather",
                  "conv1_fwd_x3_kernel": "conv1_fwd",
                  "conv2_dgrad_x3_kernel<true>": "conv2_dgrad_x3", "conv2_dgrad_x3_kernel<false>": "conv2_dgrad_x3_cut",
                  # round 5-6: the images wgrad (dense x3q, then the 2:4-sparse x3p) and the split fc head
                  "conv2_wgrad_x3q_kernel": "conv2_wgrad_x3", "conv2_wgrad_x3p_kernel": "conv2_wgrad_x3",
                  "conv1_fwd_x3_kernel<true, false>": "conv1_fwd", "conv2_fwd_pool_x3_kernel<true, false>": "conv2_fwd_pool_x3",
                  "fc_head16_kernel<1>": "fc_logits", "fc_head16_kernel<4>": "fc_dgrad",
                  "fc_head16_kernel<3>": "fc_logits"})  # round 6: logits + CE in one launch
    # widened (K5) template instantiations -> bench.py's kernel names (csrc/slk_wide.hip:824-836, 1055)
    wide = [("wide_conv32_kernel<Conv32Cfg<64, 128, 32", "wide_conv2_fwd"),
            ("wide_conv_kernel<ConvCfg<64, 128, 32", "wide_conv2_fwd"),
            ("wide_conv32_kernel<Conv32Cfg<128, 256, 16", "wide_conv3_fwd"),
            ("wide_conv_kernel<ConvCfg<128, 256, 16", "wide_conv3_fwd"),
            ("wide_conv32_kernel<Conv32Cfg<256, 128, 16", "wide_conv3_dgrad"),
            ("wide_conv_kernel<ConvCfg<256, 128, 16", "wide_conv3_dgrad"),
            ("wide_conv_kernel<ConvCfg<128, 64, 32", "wide_conv2_dgrad"),
            ("wide_wgrad_kernel<WgCfg<64, 128, 32", "wide_conv2_wgrad"),
            ("wide_wgrad_kernel<WgCfg<128, 256, 16", "wide_conv3_wgrad"),
            ("wide_conv1_wgrad_kernel", "wide_conv1_wgrad"), ("wide_conv1_fwd_kernel", "wide_conv1_fwd")]
    for k, m in out.items():
        short = names.get(k) or next((v for pfx, v in wide if k.startswith(pfx)), None)
        if short and "hbm_bytes_corrected" in m:
            prev.setdefault(short, {})[str(args.batch)] = int(m["hbm_bytes_corrected"])
    prev["_note"] = ("HBM bytes per launch from rocprofv3 --pmc (separate FETCH_SIZE and WRITE_SIZE passes, "
                     "tools/pmc.sh); FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts wide reads at half)")
    json.dump(prev, open(args.traffic_out, "w"), indent=1, sort_keys=True)
s = json.dumps(out, indent=1, sort_keys=True)
if args.out:
    open(args.out, "w").write(s)
print(s)
