"""Grid output tables: the merged replicate-level `detail_all` and the per-setting `summ_all`
of the reference grid scripts (vert-cor.R:556-593; ver-cor-subG.R:303-333), plus a CSV writer.

`detail_all` is rbindlist of every cell's run_sim_one detail with the setting columns
n, rho_true, eps1, eps2 appended, in the column order of the first cell's family: vert-cor.R's
run_sim_one frame (vert-cor.R:367-385) for the sign family, ver-cor-subG.R's (:170-172,
201-206) for sub-G.  Cover flags are 0/1/NaN floats here (R: integer for the sign family, whose
frame starts them as NA_integer_; logical for sub-G).  `summ_all` is rbindlist(summ_NI, summ_INT): per
(n, rho_true, eps1, eps2) group (data.table's `by`, groups in first-appearance order),
mse = mean(se2), bias = mean(hat) - mean(rho_true), coverage = mean(cover),
ci_len = mean(ci_len), then the method column.  The summaries come from the device
accumulators (double-double sums), so no replicate needs to leave the GPU; cells that share
a group key are merged the way data.table would pool their rows.  NA propagates as in R's
mean (no na.rm).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import lib

DETAIL_ORDER = ("repl", "ni_hat", "ni_low", "ni_up", "int_hat", "int_low", "int_up", "ni_se2", "int_se2",
                "ni_cover", "int_cover", "ni_ci_len", "int_ci_len", "n", "rho_true", "eps1", "eps2")
DETAIL_ORDER_SIGN = ("repl", "ni_hat", "int_hat", "ni_se2", "int_se2", "ni_low", "ni_up", "int_low", "int_up",
                     "ni_cover", "int_cover", "ni_ci_len", "int_ci_len", "n", "rho_true", "eps1", "eps2")


def detail_order(family: str) -> tuple:
    """detail_all's columns for a grid of `family` ("sign": vert-cor.R, "subG": ver-cor-subG.R)."""
    return DETAIL_ORDER_SIGN if family == "sign" else DETAIL_ORDER
SUMMARY_ORDER = ("n", "rho_true", "eps1", "eps2", "mse", "bias", "coverage", "ci_len", "method")
LOGICAL_COLS = ("ni_cover", "int_cover")


def grid_detail(cells, results) -> dict:
    """rbindlist of the cells' detail frames with the setting columns (vert-cor.R:556-568;
    ver-cor-subG.R:303-314), columns in detail_order(cells[0].family)."""
    order = detail_order(cells[0].family) if cells else DETAIL_ORDER
    parts = []
    for cell, res in zip(cells, results):
        d = res["detail"]
        B = len(d["repl"])
        part = {k: d[k] for k in order[:13]}
        part["n"] = np.full(B, float(cell.n))
        part["rho_true"] = np.full(B, float(cell.rho))
        part["eps1"] = np.full(B, float(cell.eps1))
        part["eps2"] = np.full(B, float(cell.eps2))
        parts.append(part)
    return {k: np.concatenate([p[k] for p in parts]) for k in order}


def _row(key, acc: _lib.Accum, method: str) -> dict:
    """One summ_* row from a (possibly merged) accumulator through dcor_accum_finalize (the same
    arithmetic as the R shim's summ_all).  With a group's rows all sharing rho_true,
    mean(hat) - mean(rho_true) = mean(hat) - rho."""
    s = _lib.Summary()
    lib.dcor_accum_finalize(C.byref(acc), float(key[1]), C.byref(s))
    return {"n": key[0], "rho_true": key[1], "eps1": key[2], "eps2": key[3], "mse": s.mse,
            "bias": s.bias, "coverage": s.coverage, "ci_len": s.ci_length, "method": method}


def grid_summary(cells, results) -> list:
    """summ_all = rbindlist(summ_NI, summ_INT) (vert-cor.R:573-593; ver-cor-subG.R:319-333)
    from the per-cell accumulators of run_cell."""
    groups, order = {}, []
    for cell, res in zip(cells, results):
        key = (float(cell.n), float(cell.rho), float(cell.eps1), float(cell.eps2))
        if key not in groups:
            groups[key] = [_lib.Accum(), _lib.Accum()]
            order.append(key)
        for m in range(2):
            lib.dcor_accum_merge(C.byref(groups[key][m]), C.byref(res["accum"][m]))
    return ([_row(k, groups[k][0], "NI") for k in order] +
            [_row(k, groups[k][1], "INT") for k in order])


def _fmt(v) -> str:
    if isinstance(v, str):
        return '"' + v.replace('"', '""') + '"'
    if v is None or (isinstance(v, float) and math.isnan(v)):
        return "NA"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    f = float(v)
    if f.is_integer() and abs(f) < 1e15:
        return str(int(f))
    return repr(f)  # shortest round-trip form: read back bit for bit


def write_csv(table, path: str) -> None:
    """Write a column dict (detail_all) or a list of row dicts (summ_all) as CSV the way R's
    write.csv(row.names = FALSE) does: NA for missing, TRUE/FALSE for the cover flags."""
    if isinstance(table, dict):
        cols = list(table)   # grid_detail's family order
        nrow = len(table[cols[0]]) if cols else 0
        get = lambda c, i: table[c][i]
    else:
        cols = [c for c in SUMMARY_ORDER if table and c in table[0]]
        nrow = len(table)
        get = lambda c, i: table[i][c]
    with open(path, "w") as f:
        f.write(",".join(f'"{c}"' for c in cols) + "\n")
        for i in range(nrow):
            vals = []
            for c in cols:
                v = get(c, i)
                if c in LOGICAL_COLS:
                    vals.append("NA" if (v != v) else ("TRUE" if v else "FALSE"))
                else:
                    vals.append(_fmt(v))
            f.write(",".join(vals) + "\n")


def run_grid_tables(cells, B: int, detail: bool = True, devices=None) -> dict:
    """Run a grid through the batched engine (dcor.sim.run_grid: one dcor_grid_run_multi call
    over `devices`) and return {'detail_all' (if detail), 'summ_all'}."""
    from .sim import run_grid
    results = run_grid(cells, B, detail=detail, devices=devices)
    out = {"summ_all": grid_summary(cells, results)}
    if detail:
        out["detail_all"] = grid_detail(cells, results)
    return out
