"""Summarise scripts/pmc_ab.sh output: mean per-dispatch counters of k_rays per variant (+ derived)."""
import csv, glob, json, os, sys
d = sys.argv[1]
res = {}
for path in sorted(glob.glob(os.path.join(d, "v*_g*", "**", "*counter_collection.csv"), recursive=True)):
    var = os.path.relpath(path, d).split(os.sep)[0].rsplit("_g", 1)[0]
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            kn = row.get("Kernel_Name", "")
            if "k_rays" in kn:
                tag = "tail" if "tail" in kn else "main"
                vals.setdefault((tag, row["Counter_Name"]), []).append(float(row["Counter_Value"]))
    for (tag, k), v in vals.items():
        res.setdefault(var + ("" if tag == "main" else "/tail"), {})[k] = sum(v) / len(v)
for var, c in res.items():
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        c["kernel_us_at_2.4GHz"] = cyc / 2400.0
        c["valu_busy"] = c.get("SQ_ACTIVE_INST_VALU", 0) * 4.0 / (1024 * cyc)
        c["waves_per_simd"] = c.get("SQ_WAVE_CYCLES", 0) * 4.0 / (1024 * cyc)
    if "SQ_WAVES" in c and "SQ_INSTS_VALU" in c:
        c["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        c["salu_per_wave"] = c["SQ_INSTS_SALU"] / c["SQ_WAVES"]
print(json.dumps(res, indent=1))
