"""Summarise a rocprofv3 run (scripts/prof.sh -> gpurun_out/prof_<tag>/prof_*) into profiles/<tag>_*.

Copies the kernel-trace stats CSV and writes <tag>_summary.json / .md with, per kernel: average
duration, PMC counters per dispatch (FETCH_SIZE doubled for gfx950's 1/2 under-report of wide
streaming reads, MI355X_MICROARCH.md §HBM), effective clock, VALU activity and the fp64
instruction mix, and the command that produced it (PROF_CMD, set by scripts/prof.sh).

VALU counters, and what they are not:
- valu_busy_4cyc: rocprof's derived VALUBusy, SQ_ACTIVE_INST_VALU x 4 over the dispatch's SIMD-cycles
  (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).  SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU here to ~2 %,
  so this is the instruction count priced at 4 cycles per wave64 instruction.  gfx950 issues a
  wave64 fp32 / int32 instruction in 2 cycles (MI355X_MICROARCH.md §Wave scheduling), so it is NOT
  bounded by 1 and is not a physical fraction (kernels read up to 1.09).  Kept for comparison with
  earlier rounds only.
- cycles_per_valu_inst: the dispatch's SIMD-cycles per VALU wave-instruction it issued (lower =
  denser issue); a stream of 2-cycle instructions cannot go below 2.
- wait_inst_frac / wait_any_frac: SQ_WAIT_INST_ANY / SQ_WAIT_ANY over SQ_WAVE_CYCLES: the share of
  wave-cycles a wave waited for its next instruction's issue / for anything (memory included).
- valu_time_frac: each instruction class of the mix priced at its measured issue cost (SIMD cycles
  per wave64 instruction, scripts/ubench_issue.hip -> profiles/<costs>.json) over the dispatch's
  SIMD-cycles; physical only when the costs file is absolute ("calibration": "absolute").
The physical ceiling of the headline's VALU-bound passes is measured directly instead: bench.py
roofline.issue (dcor_diag_sign_pass ceilings).
L2 -> CU traffic (pass "tcp"): TCP_TCC_READ_REQ_sum x 128 B (gfx950 L1 line) per dispatch.
Usage: python scripts/summarize_prof.py <tag> [prof dir] [issue-costs json]
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
costs_path = sys.argv[3] if len(sys.argv) > 3 else None
if costs_path is None:
    for t in ("r04", "r02"):
        costs_path = os.path.join(dst, f"{t}_issue_costs.json")
        if os.path.exists(costs_path):
            break
_costs = json.load(open(costs_path)) if os.path.exists(costs_path) else {}
COSTS = _costs.get("cycles_per_wave_instruction")
COSTS_ABSOLUTE = _costs.get("calibration") == "absolute"
# instruction class of the mix counters -> the measured instruction that represents it
CLASS_COST = {"SQ_INSTS_VALU_ADD_F64": "v_add_f64", "SQ_INSTS_VALU_MUL_F64": "v_mul_f64",
              "SQ_INSTS_VALU_FMA_F64": "v_fma_f64", "SQ_INSTS_VALU_TRANS_F64": "v_rsq_f64",
              "SQ_INSTS_VALU_INT32": "v_add_u32", "SQ_INSTS_VALU_INT64": "v_mad_u64_u32",
              "SQ_INSTS_VALU_CVT": "v_cvt_f64_i32"}
OTHER_COST = "v_bitop3_b32"   # the rest: bit ops, moves, selects, fp32 (single-issue class)


def valu_cycles(avg):
    """SIMD cycles the dispatch's VALU instructions take at their measured issue costs."""
    mix = {c: avg.get(c, 0.0) for c in CLASS_COST}
    rest = max(0.0, avg["SQ_INSTS_VALU"] - sum(mix.values()))
    return sum(v * COSTS[CLASS_COST[c]] for c, v in mix.items()) + rest * COSTS[OTHER_COST]


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


sys.path.insert(0, root)
from bench import src_sha16  # noqa: E402
import subprocess  # noqa: E402
try:
    head = subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                          text=True, check=True).stdout.strip()
except (OSError, subprocess.CalledProcessError):
    head = None
# the tree this summary describes: the committed head it was profiled at and the hash of the engine
# sources (bench.py compares the hash with its own tree's: roofline.*_source_fresh)
out = {"kernels": {}, "git_head": os.environ.get("PROF_HEAD", head), "src_sha16": src_sha16(root),
       "command": os.environ.get("PROF_CMD"), "issue_costs": os.path.relpath(costs_path, root) if COSTS else None,
       "issue_costs_absolute": COSTS_ABSOLUTE}
stats = os.path.join(src, "prof_trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    for r in csv.DictReader(open(stats)):
        k = out["kernels"].setdefault(short(r["Name"]), {})
        k["calls"] = int(r["Calls"])
        k["avg_ns"] = float(r["AverageNs"])
        k["pct_time"] = float(r["Percentage"])

counters = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("prof_fetch", "prof_write", "prof_sq", "prof_mix", "prof_tcp"):
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
    if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
        for c, nm in (("SQ_WAIT_INST_ANY", "wait_inst_frac"), ("SQ_WAIT_ANY", "wait_any_frac")):
            if c in avg:
                k[nm] = avg[c] / avg["SQ_WAVE_CYCLES"]
    if "TCP_TCC_READ_REQ_sum" in avg:
        k["l2_to_cu_read_bytes"] = avg["TCP_TCC_READ_REQ_sum"] * 128
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg and avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]:
        k["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in avg and k.get("avg_ns"):
        k["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / k["avg_ns"]
        simd_cycles = 1024 * avg["GRBM_GUI_ACTIVE"] / 8   # meaningful for kernels profiled alone (SERIAL=1)
        if "SQ_ACTIVE_INST_VALU" in avg:
            k["valu_busy_4cyc"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles
        if "SQ_INSTS_VALU" in avg and avg["SQ_INSTS_VALU"]:
            k["cycles_per_valu_inst"] = simd_cycles / avg["SQ_INSTS_VALU"]
            if COSTS and all(c in avg for c in CLASS_COST):
                k["valu_time_frac"] = valu_cycles(avg) / simd_cycles
                k["valu_cycles_per_dispatch"] = valu_cycles(avg)
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
    # steady state: back-to-back calls overlap (the next call's first chunks start beside the previous
    # call's tail), so the GPU time per call is the whole run's sign-kernel span over the calls --
    # what bench.py's kernel_ms_avg measures (first call's start to last call's end, / K)
    sk = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
          if "k_sign_" in short(r["Kernel_Name"]) or "k_subg_" in short(r["Kernel_Name"])]
    ncalls = len(spans) + (1 if cur else 0)
    if sk and ncalls:
        out["simulate_steady_ms"] = {"calls": ncalls,
                                     "per_call": (max(e for _, e in sk) - min(t for t, _ in sk)) / 1e6 / ncalls}

json.dump(out, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1, sort_keys=True)
lines = [f"# rocprofv3 summary `{tag}`", "",
         f"Profiled at git head `{out['git_head']}` (engine sources sha256 `{out['src_sha16']}`).",
         f"Command: `{out['command']}`." if out.get("command") else "", "",
         "| kernel | calls | avg µs | % time | VGPR | HBM read B (corr.) | HBM write B | L2->CU read B | "
         "SIMD-cycles / VALU inst | wait-inst / wave-cycles | wait-any / wave-cycles | VALU time / SIMD-cycles | "
         "VALUBusy (4-cycle) | clock GHz |",
         "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
for kname, k in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("pct_time", 0)):
    def f(x, fmt="{:.3g}"):
        return fmt.format(x) if isinstance(x, (int, float)) else "—"
    lines.append(f"| {kname} | {k.get('calls', '—')} | {f(k.get('avg_ns', 0) / 1e3)} | {f(k.get('pct_time'))} | "
                 f"{f(k.get('vgpr'))} | {f(k.get('hbm_read_bytes_corrected'))} | {f(k.get('hbm_write_bytes'))} | "
                 f"{f(k.get('l2_to_cu_read_bytes'))} | {f(k.get('cycles_per_valu_inst'))} | "
                 f"{f(k.get('wait_inst_frac'))} | {f(k.get('wait_any_frac'))} | "
                 f"{f(k.get('valu_time_frac'))} | {f(k.get('valu_busy_4cyc'))} | "
                 f"{f(k.get('effective_clock_ghz'))} |")
lines += ["", "VALUBusy (4-cycle) prices every VALU wave-instruction at 4 SIMD-cycles; gfx950 issues int32 / "
              "fp32 ones in 2, so it is not bounded by 1 (see scripts/summarize_prof.py).  VALU time is "
              + ("priced at absolute measured costs" if out["issue_costs_absolute"] else
                 "priced at RELATIVE issue costs (not a physical fraction)") + "."]
if "simulate_call_span_ms" in out:
    sp = out["simulate_call_span_ms"]
    lines += ["", f"simulate() call span from the trace (first sign-kernel start to last end, "
                  f"{sp['calls']} calls): avg {sp['avg']:.3f} ms, min {sp['min']:.3f}, max {sp['max']:.3f} "
                  "(a call's own kernels, overlapping its neighbours')."]
if "simulate_steady_ms" in out:
    st = out["simulate_steady_ms"]
    lines += ["", f"Steady-state GPU time per call (first sign-kernel start to last end over {st['calls']} "
                  f"back-to-back calls, / calls): {st['per_call']:.3f} ms -- compare bench.py "
                  "roofline.kernel_ms_avg (HIP events, first call's start to last call's end, / K)."]
open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
