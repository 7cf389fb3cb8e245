"""bench.py -- headline benchmark of the MI355X engine (BASELINE.json metric).

Workload (BASELINE.json configs / SURVEY.md §8d "Headline"): the vert-cor.R sign family,
MASS::mvrnorm Gaussian DGP mu=(.5,.5) sigma=(2,2), rho=0.5, eps=(1,1), n=1e5, alpha=.05,
normalise=T, ci_mode auto (mixquant CIs), NI+INT per replicate.  One step = one fused
launch of R replicates per GPU (+ the per-cell accumulation kernel); every step runs fresh
replicate indices (a Monte-Carlo sweep of the cell), so nothing is cached or skipped.
Multi-GPU: one process per GPU, replicates sharded per rank (weak scaling: R per GPU
per step), accumulators all-gathered once at the end (the only collective).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-correlation_amd"))
sys.path.insert(0, ROOT)

METRIC = "MC replicates/sec (Gaussian n=1e5, NI+INT CIs) at 1/8 MI355X + % roofline"
FP64_PEAK_TFLOPS = 78.6          # MI355X FP64 vector (spec); SURVEY §8d: 3.93e13 FMA lane-ops/s
W_SAMPLE = {"gaussian": 260, "bernoulli": 120, "bounded_factor": 292}  # SURVEY §8d pinned weights
W_BATCH = 183
W_REP = 2.0e5


def work_units(cell, m, k):
    """Pinned algorithmic work per replicate: w*n + 183*k + 2e5."""
    return W_SAMPLE[cell.dgp] * cell.n + W_BATCH * k + W_REP


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cell, seconds: float = 12.0):
    """The reference's loop restated on the CPU on a bounded sample of the workload:
    run_sim_one from set.seed(seed) with R's own generators (Mersenne-Twister, inversion rnorm,
    exp_rand, rbinom, extraDistr rlaplace, mvrnorm's eigen factor) and the R-semantics
    estimators (oracle/dcor_rstream.c + dcor_oracle.c).

    Two granularities: (i) one core, run_sim_one's own loop; (ii) the mclapply
    grid equivalent -- mc.cores = detectCores() - 1 workers, each running its own cell (seed
    1e6 + i, vert-cor.R:513,534-552), here threads calling the C restatement (ctypes releases
    the GIL), capped at this box's CPU share.  Runs before the GPU is touched."""
    import concurrent.futures as cf

    from oracle.oracle import rs_sim
    c = cell.to_c()
    t0 = time.perf_counter()
    rs_sim(c, 2)
    per = (time.perf_counter() - t0) / 2
    B = int(max(2, min(2000, seconds / max(per, 1e-9))))
    t0 = time.perf_counter()
    rs_sim(c, B)
    el = time.perf_counter() - t0
    nproc = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    share = int(os.environ.get("OMP_NUM_THREADS", usable) or usable)
    workers = max(1, min(usable, share, nproc) - 1)
    Bw = max(2, int(B * 0.8))

    def one(i):
        ci = cell.to_c()
        ci.seed = 1_000_000 + 1 + i
        rs_sim(ci, Bw)
        return Bw

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        done = sum(ex.map(one, range(workers)))
    elm = time.perf_counter() - t0
    return {"value": B / el, "unit": "replicates/s", "cores": 1, "kind": "port",
            "sample": f"replicates 1..{B} of run_sim_one(seed={cell.seed}) on the headline cell "
                      f"(n={cell.n}) in {el:.1f} s: oracle/dcor_rstream.c (R's own generators) + "
                      "dcor_oracle.c (R-semantics estimators), 1 thread (mclapply granularity: one "
                      "core per cell); faster than R, whose batch loop is interpreted",
            "nproc": nproc, "usable_cores": usable, "cpu_model": _cpu_model(),
            "multi_core_value": done / elm, "multi_core_cores": workers,
            "multi_core_sample": f"{workers} threads x {Bw} replicates, each its own headline-config "
                                 f"cell (seed 1e6 + i), in {elm:.1f} s: the mclapply grid's "
                                 "detectCores() - 1 workers, capped at this box's CPU share",
            "whole_host_projected_value": done / elm / workers * max(1, usable - 1),
            "whole_host_projected_note": f"multi_core_value per thread x {max(1, usable - 1)} "
                                         "(detectCores() - 1 on this host): a linear projection, "
                                         "not a measurement; an upper bound for the host"}


def src_sha16(root: str = ROOT) -> str:
    """sha256 (first 16 hex) of the engine's sources -- csrc/*.hip, *.h, *.cpp and include/dcor.h --
    as they are on disk: stamped into every committed profile summary by scripts/summarize_prof.py,
    so the bench line can tell whether the profile it quotes was taken on this code."""
    import hashlib
    h = hashlib.sha256()
    cs = os.path.join(root, "distributed-correlation_amd", "csrc")
    files = sorted(f for f in os.listdir(cs) if f.endswith((".hip", ".h", ".cpp")))
    for f in [os.path.join(cs, f) for f in files] + [os.path.join(root, "include", "dcor.h")]:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def profile_stamp(path):
    """(git head, fresh) of a committed profile summary: fresh = its source hash equals this tree's."""
    try:
        d = json.load(open(path))
        return d.get("git_head"), d.get("src_sha16") == src_sha16()
    except (OSError, ValueError, TypeError):
        return None, False


def _profile(name):
    for tag in ("r03", "r02", "r01"):
        p = os.path.join(ROOT, "profiles", f"{tag}_{name}_summary.json")
        if os.path.exists(p):
            return p
    return None


def pmc_traffic(path=_profile("headline")):
    """HBM bytes per simulate() call from the committed rocprofv3 PMC passes (FETCH_SIZE x2
    for gfx950's half-count of wide reads, + WRITE_SIZE; scripts/summarize_prof.py), summed
    over the sign kernels of one call.  None if the profile is absent."""
    try:
        ks = json.load(open(path))["kernels"]
        calls = ks["dcor::k_accumulate"]["calls"]
        tot = sum((v["hbm_read_bytes_corrected"] + v["hbm_write_bytes"]) * v["calls"]
                  for name, v in ks.items() if "k_sign_" in name)
        return tot / calls
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None


def issue_frac(path=_profile("serial")):
    """Hardware-measured VALU roofline of the sign kernels from the committed rocprofv3 profile
    (chunks profiled serially, so no kernel shares the SIMDs): rocprof's VALUBusy,
    SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), the fraction of SIMD-cycles the
    vector ALU was executing (scripts/summarize_prof.py valu_busy; <= 1 by construction).
    -> (time-weighted fraction over pass 1 + pass 2 + epilogue, per kernel, source) or Nones."""
    try:
        ks = json.load(open(path))["kernels"]
        per, num, den = {}, 0.0, 0.0
        for name, v in ks.items():
            if "k_sign_" in name and "valu_busy" in v:
                per[name.split("::")[1].split("(")[0]] = round(v["valu_busy"], 3)
                num += v["valu_busy"] * v["avg_ns"] * v["calls"]
                den += v["avg_ns"] * v["calls"]
        return (num / den if den else None), (per or None), os.path.relpath(path, ROOT)
    except (OSError, KeyError, ValueError, IndexError, TypeError):
        return None, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=8192, help="replicates per GPU per step")
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = None
    if world == 1 and not args.no_cpu_baseline:   # before the GPU is touched (the pool forks nothing)
        from dcor.sim import headline_cell as _hc
        cpu = cpu_baseline(_hc(args.n), args.cpu_seconds)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    import dcor
    from dcor import _lib
    from dcor.dist import gather_accums, merge_ranked
    from dcor.sim import accum_from_bytes, accumulate, finalize, headline_cell, simulate

    cell = headline_cell(args.n)
    k, m = dcor.api.batch_geometry(cell.n, cell.eps1, cell.eps2, "sign")
    R = args.reps
    stream = torch.cuda.current_stream()
    buf = torch.empty((R, 6), dtype=torch.float64, device="cuda")
    accs = []

    def step(s):
        r0 = (s * world + rank) * R
        simulate(cell, R, r0, out=buf, stream=stream)
        return accumulate(buf, cell.rho, stream=stream)

    for s in range(args.warmup):          # warmup runs replicate indices after the timed ones
        step(args.steps + s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        r0 = (s * world + rank) * R
        simulate(cell, R, r0, out=buf, stream=stream)
        ev[s][1].record(stream)
        accs.append(accumulate(buf, cell.rho, stream=stream))
    host = [accum_from_bytes(a.cpu().numpy().tobytes()) for a in accs]
    local_acc = [merge_from(host, 0), merge_from(host, 1)]
    if world > 1:
        merged = merge_ranked(gather_accums(local_acc))
    else:
        merged = local_acc
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # GPU time per call at steady state: the first call's start event to the last call's end event
    # over the K calls.  Back-to-back calls overlap (the next call's first chunks start beside the
    # previous call's tail on the library streams), so per-call event pairs on the caller's stream
    # would undercount; this span counts every call's kernels once and excludes only host time
    # before the first launch and after the last.
    kern_ms = ev[0][0].elapsed_time(ev[-1][1]) / args.steps

    total_reps = R * args.steps * world
    value = total_reps / el
    W = work_units(cell, m, k)
    achieved = R * W * 2.0 / (kern_ms * 1e-3) / 1e12  # fp64-equivalent TFLOP/s per GPU
    summ = {"NI": finalize(merged[0], cell.rho), "INT": finalize(merged[1], cell.rho)}

    ifrac, iper, isrc = issue_frac()
    if rank == 0:
        res = {
            "metric": METRIC, "value": value, "unit": "replicates/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (on-device Philox draws of the reference DGP)",
            "config": {"workload": "vert-cor.R sign family, Gaussian mvrnorm mu=(.5,.5) sigma=(2,2), "
                                   "rho=.5, eps=(1,1), NI+INT CIs (mixquant)",
                       "n": cell.n, "m": m, "k": k, "replicates_per_gpu_per_step": R,
                       "parallelism": f"replicate-shard x{world}"},
            "roofline": {"bound": "valu_fp64", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "frac_convention": achieved / FP64_PEAK_TFLOPS,
                         "frac_kind": "pinned-convention: SURVEY §8d work weights (fp64-FMA units) per "
                                      "replicate x replicates / kernel time over the fp64 peak; > 1 means "
                                      "the kernels issue fewer instructions than the weights assume",
                         "issue_frac": ifrac, "issue_frac_per_kernel": iper,
                         "issue_frac_kind": "measured: rocprofv3 VALUBusy (SQ_ACTIVE_INST_VALU x 4 / "
                                            "SIMD-cycles), time-weighted over the sign kernels "
                                            "profiled serially; the VALU-bound kernels' roofline",
                         "issue_source": isrc,
                         "issue_source_head": profile_stamp(os.path.join(ROOT, isrc))[0] if isrc else None,
                         "issue_source_fresh": profile_stamp(os.path.join(ROOT, isrc))[1] if isrc else False,
                         "traffic": pmc_traffic(),
                         "traffic_source": os.path.relpath(_profile("headline"), ROOT) if _profile("headline") else None,
                         "traffic_source_head": profile_stamp(_profile("headline"))[0] if _profile("headline") else None,
                         "traffic_source_fresh": profile_stamp(_profile("headline"))[1] if _profile("headline") else False,
                         "traffic_unit": "HBM B per simulate() call (rocprofv3 PMC, FETCH_SIZE x2 + WRITE_SIZE)",
                         "kernel": "k_sign_pass1 + k_sign_pass2 + k_sign_epilogue_w (one simulate() call)",
                         "kernel_ms_avg": kern_ms,
                         "kernel_ms_kind": "HIP events: first call's start to last call's end over the timed calls, / K",
                         "work_units_per_rep": W},
            "summary": {"coverage_NI": summ["NI"]["coverage"], "coverage_INT": summ["INT"]["coverage"],
                        "ci_len_NI": summ["NI"]["ci_length"], "ci_len_INT": summ["INT"]["ci_length"]},
        }
        if cpu is not None:
            res["cpu_baseline"] = cpu
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def merge_from(host, meth):
    from dcor.sim import merge
    return merge([h[meth] for h in host])


if __name__ == "__main__":
    main()
