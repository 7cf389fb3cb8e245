"""Diagnostic: per-replicate parity of a few cells through simulate() and the grid, vs the oracle."""
import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "distributed-correlation_amd"), os.path.join(os.getcwd(), "tests")]
import numpy as np
import torch
from dcor.sim import CellSpec, simulate, grid_launch
from oracle import oracle as orc
from helpers import close

def rep_ok(got, ref):
    return [bool(close(got[r], ref[r], 1e-12, 1e-13)) for r in range(len(got))]

cells = [CellSpec(n=1600, rho=0.0, eps1=1.0, eps2=1.0, seed=1000052),
         CellSpec(n=800, rho=0.0, eps1=1.0, eps2=1.0, seed=1000051),
         CellSpec(n=1600, rho=0.3, eps1=1.5, eps2=0.5, seed=1000053),
         CellSpec(n=1600, rho=0.3, eps1=0.5, eps2=0.5, seed=1000054),
         CellSpec(n=20000, rho=0.5, eps1=1.0, eps2=1.0, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1000055),
         CellSpec(n=20000, rho=0.5, eps1=0.5, eps2=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1000056),
         CellSpec(n=20000, rho=0.5, eps1=1.5, eps2=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1000057)]
R = 12
for c in cells:
    got = simulate(c, R).cpu().numpy()
    ref = orc.sim_reps(c.to_c(), 0, R)
    ok = rep_ok(got, ref)
    print("sim", c.n, c.eps1, c.eps2, "ok", sum(ok), "/", R, "first bad", ok.index(False) if False in ok else None,
          flush=True)
    if False in ok:
        r = ok.index(False)
        print("   got", got[r], "\n   ref", ref[r], flush=True)
# grid: the n = 1600 (1, 1) cell alone, then with an m = 200 cell in the same launch
for extra in ([], [CellSpec(n=1600, rho=0.3, eps1=0.2, eps2=0.2, seed=1000060)]):
    cs = [cells[0]] + extra
    out, acc = grid_launch(cs, 0, R)
    torch.cuda.synchronize()
    rec = out.cpu().numpy().reshape(len(cs), R, 6)
    ref = orc.sim_reps(cells[0].to_c(), 0, R)
    ok = rep_ok(rec[0], ref)
    print("grid extra", len(extra), "ok", sum(ok), "/", R, flush=True)
