"""Generate tests/golden/explicit_cases.npz: seeded explicit-input cases (inputs + the
numpy restatement's outputs) for ci_NI_signbatch, ci_INT_signflip, correlation_NI_subG
(sim + HRS), ci_INT_subG (sim + HRS), mixquant, priv_standardize and dp_sd.

The reference ships no golden vectors and R is absent, so these are the
build's own restatement outputs (parity unpinned); they pin the oracle and the GPU path
to each other and guard against regressions.  Run: python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy_ref as R  # noqa: E402
from helpers import sign_case, subg_case, unit_laplace  # noqa: E402

EPS = [(0.5, 0.5), (1.0, 1.0), (1.5, 0.5), (0.5, 1.5), (0.2, 0.2)]
NS = [10, 57, 400, 1999]


def main():
    out = {}
    g = np.random.default_rng(20251205)
    i = 0
    for n in NS:
        for (e1, e2) in EPS:
            cs = sign_case(g, n, e1, e2, rho=float(g.uniform(-0.9, 0.9)))
            p = f"sign{i}_"
            for key in ("X", "Y", "lap_ni_sc", "lap_x", "lap_y", "lap_int_sc", "flips", "mix_z", "mix_l"):
                out[p + key] = cs[key]
            out[p + "scalars"] = np.array([n, e1, e2, cs["lap_z"]])
            ni = R.ci_ni_signbatch(cs["X"], cs["Y"], e1, e2, 0.05, True, cs["lap_ni_sc"], cs["lap_x"], cs["lap_y"])
            out[p + "ni"] = np.array(ni if ni is not None else [np.nan] * 3)
            out[p + "int"] = np.array([R.ci_int_signflip(cs["X"], cs["Y"], e1, e2, 0.05, md, True,
                                                         cs["lap_int_sc"], cs["flips"], cs["lap_z"],
                                                         cs["mix_z"], cs["mix_l"]) for md in (0, 1, 2)])
            i += 1
    out["n_sign"] = np.array([i])
    i = 0
    for n in NS:
        for (e1, e2) in EPS:
            for hrs in (False, True):
                cs = subg_case(g, n, e1, e2, rho=float(g.uniform(0, 0.95)), nsim=2000 if hrs else 1000, hrs=hrs)
                p = f"subg{i}_"
                for key in ("X", "Y", "lap_x", "lap_y", "lap_local", "mix_z", "mix_l"):
                    out[p + key] = cs[key]
                if hrs:
                    out[p + "perm"] = cs["perm"]
                lam = (2.2, 2.6) if hrs else (np.nan, np.nan)
                out[p + "scalars"] = np.array([n, e1, e2, cs["lap_central"], float(hrs), lam[0], lam[1]])
                out[p + "ni"] = np.array(R.ni_subg(cs["X"], cs["Y"], e1, e2, hrs=hrs,
                                                   lam_x=lam[0] if hrs else None, lam_y=lam[1] if hrs else None,
                                                   perm=cs["perm"], lap_x=cs["lap_x"], lap_y=cs["lap_y"]))
                out[p + "int"] = np.array(R.int_subg(cs["X"], cs["Y"], e1, e2, hrs=hrs,
                                                     lam_s=lam[0] if hrs else None, lam_o=lam[1] if hrs else None,
                                                     lap_local=cs["lap_local"], lap_central=cs["lap_central"],
                                                     mix_z=cs["mix_z"], mix_l=cs["mix_l"]))
                i += 1
    out["n_subg"] = np.array([i])
    # mixquant / priv_standardize / dp_sd
    for j in range(12):
        nsim = [1000, 2000, 7, 1][j % 4]
        z, l = g.standard_normal(nsim), unit_laplace(g, nsim)
        c = float([0.0, 0.3, 5.0, 100.0][j % 4])
        out[f"mq{j}_z"], out[f"mq{j}_l"] = z, l
        out[f"mq{j}_c"] = np.array([c, R.mixquant(z, l, c, 0.975)])
    for j in range(6):
        v = g.normal(0.5, 2.0, [10, 100, 1000][j % 3])
        lap = unit_laplace(g, 2)
        eps = [0.5, 1.0][j % 2]
        L = math.sqrt(2 * math.log(len(v)))
        out[f"ps{j}_v"], out[f"ps{j}_lap"] = v, lap
        out[f"ps{j}_par"] = np.array([eps, L])
        out[f"ps{j}_out"] = R.priv_standardize(v, eps, L, lap)
        x = g.normal(65, 10, [50, 500, 5000][j % 3])
        out[f"sd{j}_x"], out[f"sd{j}_lap"] = x, lap
        out[f"sd{j}_out"] = np.array(R.dp_sd(x, 45.0, 90.0, 0.1, 0.1, lap))
    np.savez_compressed(os.path.join(HERE, "explicit_cases.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
