"""HS breakdown: host enqueue time vs wall time of hrs.sweep_segments at several stream counts."""
import sys, time
sys.path.insert(0, ".")
import numpy as np
import torch
import bench_configs
from dcor import hrs

args = bench_configs.hrs_panel("coded")
segs = [(e, 0, 200) for e in range(23)]
for streams in (1, 2, 4, 8):
    hrs.sweep_segments(*args, hrs.EPS_GRID, segs, streams=streams)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        hrs.sweep_segments(*args, hrs.EPS_GRID, segs, streams=streams)
        ts.append(time.perf_counter() - t0)
    print(f"streams={streams} wall_ms={1e3 * min(ts):.3f} median={1e3 * np.median(ts):.3f}", flush=True)
t0 = time.perf_counter()
for _ in range(100):
    hrs.standin_panel  # noqa
x = torch.empty((200, 19433), dtype=torch.float64, device="cuda")
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(1000):
    torch.empty((200, 19433), dtype=torch.float64, device="cuda")
print("torch.empty us", (time.perf_counter() - t0) * 1e3, flush=True)
runs = hrs.sweep_segments(*args, hrs.EPS_GRID, segs).reshape(23, 200, 6)
t0 = time.perf_counter()
for _ in range(20):
    hrs.sweep_summaries(hrs.EPS_GRID, runs)
print("summaries ms", (time.perf_counter() - t0) / 20 * 1e3, flush=True)
