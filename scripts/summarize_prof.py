"""Summarise a rocprofv3 run (gpurun_out/prof_*) into profiles/<tag>_*.

Copies the kernel-trace stats CSV and writes <tag>_summary.json / .md with, per kernel:
average duration, PMC counters per dispatch (FETCH_SIZE doubled for gfx950's 1/2 under-
report of wide streaming reads, MI355X_MICROARCH.md §HBM), effective clock, VALU
activity and the fp64 instruction mix.
Usage: python scripts/summarize_prof.py <tag> [gpurun_out]
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


out = {"kernels": {}}
stats = os.path.join(src, "prof_trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    for r in csv.DictReader(open(stats)):
        k = out["kernels"].setdefault(short(r["Name"]), {})
        k["calls"] = int(r["Calls"])
        k["avg_ns"] = float(r["AverageNs"])
        k["pct_time"] = float(r["Percentage"])

counters = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("prof_fetch", "prof_write", "prof_sq", "prof_mix"):
    f = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        counters[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "SQ_WAVES":
            counters[short(r["Kernel_Name"])]["_vgpr"] = [float(r["VGPR_Count"])]
            counters[short(r["Kernel_Name"])]["_lds"] = [float(r["LDS_Block_Size"])]
            counters[short(r["Kernel_Name"])]["_grid"] = [float(r["Grid_Size"])]

for kname, cs in counters.items():
    k = out["kernels"].setdefault(kname, {})
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    k["pmc_per_dispatch"] = {c: v for c, v in avg.items() if not c.startswith("_")}
    if "FETCH_SIZE" in avg:
        k["hbm_read_bytes_corrected"] = avg["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in avg:
        k["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "_vgpr" in avg:
        k["vgpr"] = avg["_vgpr"]
        k["lds_bytes"] = avg["_lds"]
        k["grid_threads"] = avg["_grid"]
    if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
        k["valu_active_frac_of_wave_cycles"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in avg and k.get("avg_ns"):
        k["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / k["avg_ns"]
        # VALU issue ceiling: one wave64 VALU instruction per 4 cycles per SIMD = 1 per cycle
        # per CU (256 CUs); meaningful for kernels profiled without overlap (PIPE=0 runs)
        if "SQ_INSTS_VALU" in avg:
            k["valu_issue_util"] = avg["SQ_INSTS_VALU"] / (256 * avg["GRBM_GUI_ACTIVE"] / 8)
    mix = {c: avg[c] for c in avg if c.startswith("SQ_INSTS_VALU_")}
    if mix:
        k["valu_mix_wave_instructions"] = mix

# Wall span of each simulate() call from the kernel trace: the sign kernels of one call run on
# two streams, so per-kernel averages overlap; bench.py's kernel_ms_avg is this span (events
# around the call).  A call = the dispatches between consecutive k_accumulate launches.
trace = os.path.join(src, "prof_trace", "run_kernel_trace.csv")
if os.path.exists(trace):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    spans, cur = [], []
    for r in rows:
        name = short(r["Kernel_Name"])
        if "k_accumulate" in name and "merge" not in name:
            if cur:
                spans.append((max(e for _, e in cur) - min(s for s, _ in cur)) / 1e6)
            cur = []
        elif "k_sign_" in name or "k_subg_" in name:
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if spans:
        out["simulate_call_span_ms"] = {"calls": len(spans), "avg": sum(spans) / len(spans),
                                        "min": min(spans), "max": max(spans)}

json.dump(out, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1, sort_keys=True)
lines = [f"# rocprofv3 summary `{tag}`", "",
         "| kernel | calls | avg µs | % time | VGPR | HBM read B (corr.) | HBM write B | VALU active / wave-cycles | VALU issue util | clock GHz |",
         "|---|---|---|---|---|---|---|---|---|---|"]
for kname, k in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("pct_time", 0)):
    def f(x, fmt="{:.3g}"):
        return fmt.format(x) if isinstance(x, (int, float)) else "—"
    lines.append(f"| {kname} | {k.get('calls', '—')} | {f(k.get('avg_ns', 0) / 1e3)} | {f(k.get('pct_time'))} | "
                 f"{f(k.get('vgpr'))} | {f(k.get('hbm_read_bytes_corrected'))} | {f(k.get('hbm_write_bytes'))} | "
                 f"{f(k.get('valu_active_frac_of_wave_cycles'))} | {f(k.get('valu_issue_util'))} | "
                 f"{f(k.get('effective_clock_ghz'))} |")
if "simulate_call_span_ms" in out:
    sp = out["simulate_call_span_ms"]
    lines += ["", f"simulate() call span from the trace (first sign-kernel start to last end, "
                  f"{sp['calls']} calls): avg {sp['avg']:.3f} ms, min {sp['min']:.3f}, max {sp['max']:.3f} "
                  "-- compare bench.py roofline.kernel_ms_avg (HIP events around the same call)."]
open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
