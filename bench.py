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
    for tag in ("r06", "r05", "r04", "r03", "r02", "r01"):
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
    except (OSError, KeyError, ValueError, ZeroDivisionError, TypeError):
        return None


def measure_passes(cell, reps: int = 2048, rep_begin: int = 0, iters: int = 5) -> dict:
    """Live per-pass times of the one-pass sign path and their measured issue ceilings, on this
    GPU, now (dcor_diag_sign_pass): each pass over `reps` replicates as one chunk on the current
    stream, alone on the device, median of `iters` launches timed with HIP events on that stream.

      pass1 / pass2 / epilogue   the real kernels (k_sign_pass1 -- which regenerates its own slow
                                 samples -- k_sign_pass2, k_sign_epilogue_w)
      pass1_ceiling              k_sign_pass1's own hot loop -- Philox, ziggurat fast path, mvrnorm
                                 transform, clips, record codes, group sums -- with the slab store
                                 and the slow-normal queue removed, at pass 1's waves per SIMD
      pass1_ceiling_own_occ      the same at the ceiling kernel's own (higher) occupancy
      pass2_ceiling              k_sign_pass2's decision loop with its records held in registers
                                 (no slab stream, no tie fix-up), at pass 2's occupancy
      pass1_ceiling_plus_stores  the pass-1 ceiling with its slab stores put back
      pass1_ceiling_plus_queue   the pass-1 ceiling with its slow-sample list and regenerations put back

    A ceiling is the time the pass's own instruction stream takes when nothing but issue limits
    it: pass / ceiling is how far memory, queueing and fix-ups keep the pass from it."""
    import ctypes as C

    import torch
    from dcor import _lib
    c = cell.to_c()
    st = torch.cuda.current_stream()

    def run(which):
        _lib.check(_lib.lib.dcor_diag_sign_pass(C.byref(c), rep_begin, reps, which, C.c_void_p(st.cuda_stream)))

    def timed(which):
        run(which)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in ev:
            a.record(st)
            run(which)
            b.record(st)
        torch.cuda.synchronize()
        return sorted(a.elapsed_time(b) for a, b in ev)[iters // 2]

    out = {"pass1": timed(1), "pass2": timed(2), "epilogue": timed(3),
           "pass1_ceiling": timed(11), "pass1_ceiling_own_occ": timed(13), "pass2_ceiling": timed(12),
           "pass1_ceiling_plus_stores": timed(14), "pass1_ceiling_plus_queue": timed(15)}
    return {k: round(v, 5) for k, v in out.items()}


def sim_chunking(cell, reps: int):
    """(chunk, chunks) of dcor_sim_launch for `reps` replicates of `cell`: the library's own plan,
    so the live ceilings are timed at the launch shape the timed calls ran."""
    import ctypes as C

    from dcor import _lib
    ch, nc = C.c_int64(), C.c_int64()
    _lib.check(_lib.lib.dcor_sim_chunking(C.byref(cell.to_c()), reps, C.byref(ch), C.byref(nc)))
    return ch.value, nc.value


def serial_valu_time(names=("k_sign_pass1<0>", "k_sign_pass2<0>", "k_sign_epilogue_w<16>")):
    """Hardware-anchored fraction per kernel from the committed serial profile (rocprofv3 PMC,
    scripts/summarize_prof.py): VALU time / SIMD-cycles, each VALU wave-instruction priced at its
    measured absolute issue cost -- the share of the SIMDs' cycles the kernel spends issuing VALU work
    (1.0 = the SIMDs never idle).  Unlike issue_frac it does not depend on the kernel's own
    instruction count."""
    path = _profile("serial")
    if path is None:
        return None
    try:
        ks = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    out = {}
    for nm in names:
        v = ks.get("dcor::" + nm)
        if v is not None and v.get("valu_time_frac") is not None:
            out[nm] = {"valu_time_frac": round(v["valu_time_frac"], 4),
                       "wait_any_frac": round(v.get("wait_any_frac", float("nan")), 4),
                       "simd_cycles_per_valu_inst": round(v.get("cycles_per_valu_inst", float("nan")), 3)}
    head, fresh = profile_stamp(path)
    return {"kernels": out, "source": os.path.relpath(path, ROOT), "source_head": head, "source_fresh": fresh}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, script: str = __file__) -> int:
    """`bench.py --gpus N` (or bench_configs.py) without a launcher: start N rank processes of
    `script` (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT set; rank r on GPU r) and return the
    worst exit code.  Called before anything touches the GPU (no HIP state to inherit); rank 0
    prints the line."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script)] + list(argv), env=env))
    # a rank that fails leaves the others blocked in the rendezvous or a collective: stop them
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for r, p in enumerate(procs):
                try:
                    rcs[r] = p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    rcs[r] = p.wait()
            break
        time.sleep(0.2)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"bench.py: rank exit codes {rcs}", file=sys.stderr)
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); without a launcher's WORLD_SIZE, N > 1 starts N rank processes")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=8192, help="replicates per GPU per step")
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ceilings", action="store_true", help="skip the live pass ceilings (roofline.issue_frac)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--variant", action="append", default=[], metavar="NAME=VALUE",
                    help="engine implementation switch for A/B runs (dcor_set_variant; repeatable)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check on CPU: form the process group over gloo, exchange accumulators, "
                         "print the world size formed; no GPU, no timing")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            sys.exit("bench.py: --gpus must be >= 1")
        if n > 1:
            # the launcher itself loads no GPU library (no torch, no HIP, no amdsmi): each rank checks
            # its own LOCAL_RANK against the GPUs it sees and exits non-zero, which stops the others
            sys.exit(spawn_ranks(n, sys.argv[1:]))
    elif args.gpus is not None and args.gpus != int(env_world):
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher's WORLD_SIZE is {env_world}")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if os.environ.get("DCOR_BENCH_FAIL_RANK") == str(rank):   # launcher test: a rank that dies
            sys.exit(3)
        return dry_run(world, rank)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:   # before the GPU is touched (the pool forks nothing)
        from dcor.sim import headline_cell as _hc
        cpu = cpu_baseline(_hc(args.n), args.cpu_seconds)
    if world > 1:
        vis = torch.cuda.device_count()
        if local >= vis:
            sys.exit(f"bench.py: rank {rank}: LOCAL_RANK {local} but {vis} GPU(s) visible "
                     f"(--gpus {world}); refusing to measure fewer")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        formed = dist.get_world_size()
        if formed != world:
            sys.exit(f"bench.py: process group formed {formed} ranks, expected {world}")
    else:
        torch.cuda.set_device(0)
        formed = 1

    import dcor
    dcor._lib.apply_variant_args(args.variant)
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

    # live pass ceilings (after the timed region; untimed): the physical roofline of the VALU-bound path
    chunk, nch = sim_chunking(cell, R)       # the launch shape dcor_sim_launch used for R replicates
    passes = None
    if rank == 0 and not args.no_ceilings and cell.n > 16384 and m == 8:
        passes = measure_passes(cell, chunk, rep_begin=(args.steps + args.warmup) * world * R)
    issue = None
    if passes:
        ceil_call = nch * (passes["pass1_ceiling"] + passes["pass2_ceiling"] + passes["epilogue"])
        issue = {"call": ceil_call / kern_ms,
                 "pass1": passes["pass1_ceiling"] / passes["pass1"],
                 "pass2": passes["pass2_ceiling"] / passes["pass2"],
                 "pass1_occupancy_gain": passes["pass1_ceiling"] / passes["pass1_ceiling_own_occ"],
                 "chunk_reps": chunk, "chunks_per_call": nch, "ms": passes}
    traffic = pmc_traffic()
    if rank == 0:
        res = {
            "metric": METRIC, "value": value, "unit": "replicates/s", "n_gpus": formed,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (on-device Philox draws of the reference DGP)",
            "config": {"workload": "vert-cor.R sign family, Gaussian mvrnorm mu=(.5,.5) sigma=(2,2), "
                                   "rho=.5, eps=(1,1), NI+INT CIs (mixquant)",
                       "n": cell.n, "m": m, "k": k, "replicates_per_gpu_per_step": R,
                       "parallelism": f"replicate-shard x{formed}",
                       "world_formed": formed, "backend": "nccl (RCCL)" if world > 1 else "single process",
                       **({"variants": args.variant} if args.variant else {})},
            "roofline": {"bound": "valu_fp64", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "frac_kind": "pinned convention: SURVEY §8d work weights (fp64-FMA units) per "
                                      "replicate x replicates / kernel time over the fp64 peak; > 1 means "
                                      "the kernels issue fewer instructions than the weights assume, so it "
                                      "is not a physical fraction -- issue_frac is",
                         "issue_frac": None if issue is None else issue["call"],
                         "issue_frac_kind": "measured live on this GPU: the call's issue-bound time "
                                            "(chunks x (pass-1 ceiling + pass-2 ceiling + epilogue), "
                                            "dcor_diag_sign_pass 11/12/3: each pass's own instruction "
                                            "stream with its memory side removed, at its occupancy) "
                                            "over the call's kernel time (pass 2 includes the "
                                            "regeneration of pass 1's slow samples, which its ceiling "
                                            "does not)",
                         "issue": issue,
                         "valu_time": serial_valu_time(),
                         "valu_time_kind": "per kernel, from the serial rocprofv3 profile: VALU time at the "
                                           "measured absolute issue costs / SIMD-cycles (hardware-anchored: "
                                           "the SIMDs' busy share, not relative to the kernel's own stream)",
                         "traffic": traffic,
                         "traffic_source": os.path.relpath(_profile("headline"), ROOT) if _profile("headline") else None,
                         "traffic_source_head": profile_stamp(_profile("headline"))[0] if _profile("headline") else None,
                         "traffic_source_fresh": profile_stamp(_profile("headline"))[1] if _profile("headline") else False,
                         "traffic_unit": "HBM B per simulate() call (rocprofv3 PMC, FETCH_SIZE x2 + WRITE_SIZE)",
                         "kernel": "k_sign_pass1 + k_sign_pass2 + k_sign_epilogue_w (one simulate() call)",
                         "kernel_ms_avg": kern_ms,
                         "kernel_ms_kind": "HIP events: first call's start to last call's end over the timed calls, / K",
                         "work_units_per_rep": W},
            "engine": {"library_source_sha16": dcor.lib.dcor_source_hash().decode()[:16],
                       "tree_source_sha16": src_sha16(),
                       "fresh": dcor.lib.dcor_source_hash().decode()[:16] == src_sha16()},
            "summary": {"coverage_NI": summ["NI"]["coverage"], "coverage_INT": summ["INT"]["coverage"],
                        "ci_len_NI": summ["NI"]["ci_length"], "ci_len_INT": summ["INT"]["ci_length"]},
        }
        if cpu is not None:
            res["cpu_baseline"] = cpu
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dry_run(world: int, rank: int) -> None:
    """The launcher without a GPU: the ranks form a gloo group on the CPU, all-gather one
    accumulator pair each and merge them in rank order -- the bench's only collective -- and rank 0
    prints the world size formed (no value: nothing is measured)."""
    import torch.distributed as dist

    from dcor import _lib
    from dcor.dist import gather_accums, merge_ranked
    if world > 1:
        dist.init_process_group("gloo")
    formed = dist.get_world_size() if world > 1 else 1
    mine = [_lib.Accum(), _lib.Accum()]
    mine[0].n = rank + 1
    merged = merge_ranked(gather_accums(mine)) if world > 1 else mine
    if rank == 0:
        print(json.dumps({"dry_run": True, "metric": METRIC, "value": None, "n_gpus": formed,
                          "world_formed": formed, "merged_n": merged[0].n}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def merge_from(host, meth):
    from dcor.sim import merge
    return merge([h[meth] for h in host])


if __name__ == "__main__":
    main()
