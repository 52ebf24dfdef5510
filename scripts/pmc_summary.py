"""Mean per-dispatch counters of one kernel from pmc_groups.sh output dirs.
    python scripts/pmc_summary.py gpurun_out/pmc_groups [more dirs] [--kernel k_rays]"""
import csv, glob, json, os, sys
args = [a for a in sys.argv[1:] if not a.startswith("--")]
kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_rays"
args = [a for a in args if a != kern]
out = {}
for d in args:
    vals = {}
    for f in glob.glob(os.path.join(d, "g*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row.get("Kernel_Name", ""):
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    out[os.path.basename(d.rstrip("/"))] = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
