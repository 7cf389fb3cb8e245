"""Tie batches of the one-pass sign path per VG cell (vert-cor.R's grid, Philox): the share of
batches whose record codes tie a private centre's code and are recomputed exactly."""
import ctypes as C
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-correlation_amd"))
from dcor import _lib  # noqa: E402
from dcor.sim import vert_cor_grid  # noqa: E402

cells = vert_cor_grid()
B = 250
tot_t = tot_b = 0
rows = []
for cs in cells:
    c = cs.to_c()
    m = {(0.5, 0.5): 32, (1.0, 1.0): 8, (1.5, 0.5): 11}[(cs.eps1, cs.eps2)]
    k = cs.n // m
    ties = np.zeros(B, dtype=np.int64)
    _lib.check(_lib.lib.dcor_diag_sign_ties(C.byref(c), 0, B, ties.ctypes.data_as(C.POINTER(C.c_int64))))
    tot_t += int(ties.sum())
    tot_b += B * k
    rows.append((cs.n, m, cs.rho, cs.eps1, cs.eps2, int(ties.sum()) / (B * k)))
rows.sort(key=lambda r: -r[-1])
for r in rows[:4]:
    print("n=%d m=%d rho=%.2f eps=(%.1f,%.1f) tie share %.4f" % r)
print("all Gaussian sign cells: tie batches %d of %d (%.4f)" % (tot_t, tot_b, tot_t / max(tot_b, 1)))
