"""Collect the rocprofv3 evidence for one round (run on the GPU box).

  python scripts/profile_round.py r01            # on the GPU box (via gpurun)
  python scripts/profile_round.py r01 --collect  # here: raw csvs merged back under
                                                 # gpurun_out/prof_r01 -> profiles/

1. kernel trace + stats of `bench.py` (same command as the headline, fewer
   steps, no cpu leg) -> profiles/<tag>_kernel_stats.csv (+ summary json)
   (+ k_rays averages split by grid size: sub-shard vs isolated launches)
2. PMC passes (bench --streams 1: every k_rays launch is the isolated E-car one), one counter group per run (FETCH_SIZE, WRITE_SIZE,
   TCC_HIT/TCC_MISS): per-launch HBM-side bytes of k_rays -> profiles/pmc_traffic.json
   FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (rocprofv3 derived counters).
The parent process never touches the GPU; rocprofv3 launches python itself.
"""
import csv, glob, json, os, shutil, subprocess, sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
OUT = os.path.join(REPO, "gpurun_out", f"prof_{tag}")
COLLECT = "--collect" in sys.argv
# only gpurun_out/ comes back from the box: write there, copy into profiles/ locally
PROF = os.path.join(REPO, "profiles") if COLLECT else os.path.join(OUT, "summary")
ENVS = int(os.environ.get("PROFILE_ENVS", "65536"))  # the headline configuration (bench.py default)
# PROFILE_REFILL=<waves per car>: the PMC passes run k_rays_fxs (2 rays per lane) instead of the size's
# default ray kernel (files suffixed _fxs); PROFILE_NO_TRACE=1 skips the bench kernel trace (step 1)
REFILL = os.environ.get("PROFILE_REFILL")
SUFFIX = "" if not REFILL else ("_fx" if REFILL == "0" else f"_fxs{REFILL}")
NO_TRACE = os.environ.get("PROFILE_NO_TRACE") == "1"
BENCH = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "300", "--warmup", "50", "--no-cpu-baseline",
         "--no-secondary", "--no-full-outputs", "--global-envs", str(ENVS)]
env = dict(os.environ, TMPDIR="/tmp")


# PMC target: the headline's ray kernel alone (one BatchSim context, minimal outputs, 100 steps):
# the bench also runs full-output passes whose extra scan writes would mix into the averages
RAYPMC = [sys.executable, os.path.join(REPO, "scripts", "ray_pmc.py")]
env["MB_ENVS"] = str(ENVS)
if REFILL:
    env["MB_REFILL"] = REFILL
    env["MB_LANES"] = "1" if REFILL == "0" else "2"  # 0: k_rays_fx, one ray per lane (the round-4 small-shard default)


def run(name, extra, timeout=400, bench_extra=(), target=None, env_extra=None):
    d = os.path.join(OUT, f"{name}_E{ENVS}{SUFFIX}")
    if COLLECT:
        return d
    shutil.rmtree(d, ignore_errors=True)
    run_env = dict(env, **(env_extra or {}))
    cmd = ["rocprofv3"] + extra + ["--output-format", "csv", "-d", d, "-o", "run", "--"] + (target or BENCH + list(bench_extra))
    print(" ".join(cmd), flush=True)
    with open(d + ".log", "w") as log:
        subprocess.run(["timeout", "-k", "10", str(timeout)] + cmd, cwd="/tmp", env=run_env, stdout=log,
                       stderr=subprocess.STDOUT, check=True)
    return d


def find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not hits:
        raise FileNotFoundError(f"{suffix} under {d}")
    return hits[0]


def counters(d, dst, kernel="k_rays"):
    """Mean per-dispatch counter values for `kernel`; its rows are copied to dst."""
    path = find(d, "counter_collection.csv")
    vals = {}
    with open(path) as f, open(dst, "w", newline="") as g:
        rd = csv.DictReader(f)
        wr = csv.DictWriter(g, fieldnames=rd.fieldnames)
        wr.writeheader()
        for row in rd:
            name = row.get("Kernel_Name", "")
            # k_rays_fxs<..., COUNT = true>: the counting replay of scripts/ray_pmc.py, not the measured launches
            if kernel in name and "true>(f110::RayArgs)" not in name.replace(" ", ""):
                wr.writerow(row)
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


os.makedirs(OUT, exist_ok=True)
os.makedirs(PROF, exist_ok=True)
d = None if NO_TRACE else run("trace", ["--kernel-trace", "--stats"])
stats = None if NO_TRACE else find(d, "kernel_stats.csv")
if not NO_TRACE:
    shutil.copy(stats, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    summary = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            summary[row["Name"][:80]] = {k: row[k] for k in ("Calls", "TotalDurationNs", "AverageNs", "Percentage")
                                         if k in row}
    # the default bench launches k_rays at two grid sizes: the timed region's
    # sub-shards (E/S cars each, concurrent streams) and the isolated full-shard
    # roofline pass (E cars, one stream).  Split the averages by grid size so the
    # roofline's kernel_ms can be matched against the E-car launches.
    trace = find(d, "kernel_trace.csv")
    by_grid = {}
    with open(trace) as f:
        for row in csv.DictReader(f):
            if "k_rays" not in row.get("Kernel_Name", ""):
                continue
            g = next((row[k] for k in ("Grid_Size_X", "Grid_Size", "Grid_X") if k in row), "?")
            dur = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
            e = by_grid.setdefault(str(g), [0, 0.0])
            e[0] += 1
            e[1] += dur
    summary["k_rays_by_grid_size"] = {g: {"Calls": n, "AverageNs": t / n} for g, (n, t) in by_grid.items()}
    json.dump(summary, open(os.path.join(PROF, f"{tag}_kernel_stats.json"), "w"), indent=1)

res = {"kernel": "k_rays", "envs": ENVS, "agents": 1, "refill": REFILL}
for grp in (["FETCH_SIZE"], ["WRITE_SIZE"], ["TCC_HIT_sum", "TCC_MISS_sum"]):
    name = "pmc_" + "_".join(g.lower() for g in grp)
    try:
        dd = run(name, ["--pmc"] + grp, target=RAYPMC)  # the isolated E-car launch
        res.update(counters(dd, os.path.join(PROF, f"{tag}_{name}_E{ENVS}{SUFFIX}.csv")))
    except Exception as exc:  # record, do not hide
        res[name + "_error"] = repr(exc)
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    res["fetch_bytes"] = res["FETCH_SIZE"] * 1024.0
    res["write_bytes"] = res["WRITE_SIZE"] * 1024.0
    res["bytes_per_launch"] = res["fetch_bytes"] + res["write_bytes"]
    res["note"] = ("FETCH_SIZE/WRITE_SIZE (KiB) per k_rays dispatch; gather widths are uncalibrated on gfx950 "
                   "(MI355X_MICROARCH.md HBM section: 16-B streaming reads report 1/2); Infinity-Cache hits are "
                   "counted by these TCC_EA counters")
if "TCC_HIT_sum" in res:
    res["l2_hit_rate"] = res["TCC_HIT_sum"] / max(1.0, res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
json.dump(res, open(os.path.join(PROF, f"pmc_traffic_E{ENVS}_A1{SUFFIX}.json"), "w"), indent=1)
print(json.dumps(res))

# 3. issue / occupancy pass: VALU busy and resident waves per SIMD of the isolated E-car launch.
#    SQ_* cycle counters are quad-cycles summed over waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs
#    (MI355X_MICROARCH.md), so kernel cycles = GRBM_GUI_ACTIVE / 8 and SIMDs = CUs x 4.
busy = {"kernel": "k_rays", "envs": ENVS, "agents": 1, "refill": REFILL}
grp = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
       "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"]
try:
    dd = run("pmc_busy", ["--pmc"] + grp, target=RAYPMC)
    busy.update(counters(dd, os.path.join(PROF, f"{tag}_pmc_busy_E{ENVS}{SUFFIX}.csv")))
    simds = 256 * 4
    cyc = busy["GRBM_GUI_ACTIVE"] / 8.0
    busy["valu_busy"] = busy["SQ_ACTIVE_INST_VALU"] * 4.0 / (simds * cyc)
    busy["waves_per_simd"] = busy["SQ_WAVE_CYCLES"] * 4.0 / (simds * cyc)
    busy["wait_frac"] = busy["SQ_WAIT_ANY"] / max(1.0, busy["SQ_WAVE_CYCLES"])  # share of wave time in s_waitcnt
    busy["note"] = ("valu_busy = SQ_ACTIVE_INST_VALU*4 / (1024 SIMDs * GRBM_GUI_ACTIVE/8); waves_per_simd = "
                    "SQ_WAVE_CYCLES*4 / (1024 * GRBM_GUI_ACTIVE/8); mean per k_rays dispatch, scripts/ray_pmc.py (minimal outputs)")
except Exception as exc:
    busy["error"] = repr(exc)
# 4. issue mix: instructions per wave by type and the scalar unit's load (one SALU per CU on
#    MI300 / MI355X serves the CU's 32 resident waves)
grp = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH",
       "SQ_INST_CYCLES_SALU", "SQ_ACTIVE_INST_SCA", "GRBM_GUI_ACTIVE"]
try:
    dd = run("pmc_issue", ["--pmc"] + grp, target=RAYPMC)
    iss = counters(dd, os.path.join(PROF, f"{tag}_pmc_issue_E{ENVS}{SUFFIX}.csv"))
    busy.update(iss)
    cyc = iss["GRBM_GUI_ACTIVE"] / 8.0
    # SALU instructions issued per CU per kernel cycle (one scalar ALU per CU: 1.0 = every cycle);
    # SQ_INST_CYCLES_SALU equals SQ_INSTS_SALU here, so its unit cannot be quad-cycles of one unit
    busy["salu_insts_per_cu_cycle"] = iss["SQ_INSTS_SALU"] / (256 * cyc)
    busy["valu_insts_per_simd_cycle"] = iss["SQ_INSTS_VALU"] / (1024 * cyc)
    for k in ("VALU", "SALU", "SMEM", "VMEM_RD", "BRANCH"):
        busy[f"insts_{k.lower()}_per_wave"] = iss[f"SQ_INSTS_{k}"] / max(1.0, iss["SQ_WAVES"])
except Exception as exc:
    busy["issue_error"] = repr(exc)
# 5. the vector-memory address path: wave-level vector reads against texture-address
#    busy cycles (TA_BUSY_avr: per TA instance, one per CU), the bound of the gather loop
grp = ["SQ_INSTS_VMEM_RD", "SQ_WAVES", "TA_BUSY_avr", "TA_FLAT_READ_WAVEFRONTS_sum", "GRBM_GUI_ACTIVE"]
try:
    counts_path = os.path.join(OUT, f"ray_counts_pmc_ta_E{ENVS}{SUFFIX}.json")
    dd = run("pmc_ta", ["--pmc"] + grp, target=RAYPMC, env_extra={"RAY_PMC_COUNTS": counts_path})
    ta = counters(dd, os.path.join(PROF, f"{tag}_pmc_ta_E{ENVS}{SUFFIX}.csv"))
    if os.path.exists(counts_path):  # the kernel's own count of its wave-level loads, same launches
        kc = json.load(open(counts_path))
        busy["kernel_counted_loads_per_launch"] = kc["vmem_loads_per_launch"]
        busy["kernel_counted_slot_gathers_per_launch"] = kc["slot_gathers_per_launch"]
        busy["kernel_counted_other_loads_per_launch"] = kc["other_loads_per_launch"]
        busy["vmem_rd_vs_kernel_counted"] = ta["SQ_INSTS_VMEM_RD"] / max(1.0, kc["vmem_loads_per_launch"])
    cyc = ta["GRBM_GUI_ACTIVE"] / 8.0
    busy["vmem_rd_per_launch"] = ta["SQ_INSTS_VMEM_RD"]
    busy["ta_flat_read_wavefronts"] = ta["TA_FLAT_READ_WAVEFRONTS_sum"]
    busy["ta_busy_cycles_per_cu"] = ta["TA_BUSY_avr"]
    busy["ta_busy"] = ta["TA_BUSY_avr"] / max(1.0, cyc)
    busy["ta_cycles_per_vmem_rd"] = ta["TA_BUSY_avr"] * 256 / max(1.0, ta["SQ_INSTS_VMEM_RD"])
except Exception as exc:
    busy["ta_error"] = repr(exc)
json.dump(busy, open(os.path.join(PROF, f"pmc_busy_E{ENVS}_A1{SUFFIX}.json"), "w"), indent=1)
print(json.dumps(busy))
