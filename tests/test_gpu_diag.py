"""GPU tests of the measurement entries bench.py's roofline rests on (dcor_diag_sign_pass,
dcor_diag_sign_ties): every pass and ceiling runs on the headline cell, a ceiling -- the pass's own
instruction stream with its memory side removed -- is not slower than its pass, and the ceilings
leave the results of the real passes untouched."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dc():
    import torch
    assert torch.cuda.is_available()
    import dcor
    return dcor


def test_measure_passes_orders(dc):
    sys.path.insert(0, ROOT)
    from bench import measure_passes
    from dcor.sim import headline_cell
    ms = measure_passes(headline_cell(), 512, rep_begin=1000, iters=3)
    assert all(v > 0 for v in ms.values()), ms
    assert ms["pass1_ceiling"] <= 1.05 * ms["pass1"], ms
    assert ms["pass2_ceiling"] <= 1.05 * ms["pass2"], ms
    assert ms["pass1_ceiling"] <= 1.05 * ms["pass1_ceiling_plus_queue"], ms


def test_diag_refuses_other_cells(dc):
    from dcor import _lib
    from dcor.sim import CellSpec, headline_cell
    small = headline_cell(2000).to_c()        # wave kernels: passes 1-3 only, in the workgroup kernels
    assert _lib.lib.dcor_diag_sign_pass(C.byref(small), 0, 8, 11, None) == _lib.DCOR_EINVAL
    bern = CellSpec(n=100_000, rho=0.5, eps1=1.0, eps2=1.0, dgp="bernoulli", mu=(0.0, 0.0),
                    sigma=(1.0, 1.0), seed=7).to_c()
    assert _lib.lib.dcor_diag_sign_pass(C.byref(bern), 0, 8, 1, None) == _lib.DCOR_EINVAL
    m11 = CellSpec(n=100_000, rho=0.5, eps1=1.5, eps2=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=7).to_c()
    assert _lib.lib.dcor_diag_sign_pass(C.byref(m11), 0, 8, 11, None) == _lib.DCOR_EINVAL   # ceilings: m = 8
    h = headline_cell().to_c()
    assert _lib.lib.dcor_diag_sign_pass(C.byref(h), 0, 8, 7, None) == _lib.DCOR_EINVAL


def test_ceilings_do_not_disturb_results(dc):
    """The ceiling kernels write nothing a simulate() call reads: running them between two identical
    calls leaves the second call's records bit-identical to the first's."""
    from dcor import _lib
    from dcor.sim import headline_cell, simulate
    cell = headline_cell()
    a = simulate(cell, 2048, 4096).cpu().numpy()
    c = cell.to_c()
    for which in (1, 2, 3, 11, 12, 13, 14, 15):
        _lib.check(_lib.lib.dcor_diag_sign_pass(C.byref(c), 4096, 256, which, None))
    b = simulate(cell, 2048, 4096).cpu().numpy()
    assert np.array_equal(a.view(np.int64), b.view(np.int64))


def test_diag_ties_on_small_cells(dc):
    """dcor_diag_sign_ties on a wave-kernel cell (n = 1000, m = 32: the reference grid's most
    tie-prone cell) runs its replicates in the workgroup kernels and counts tie batches per
    replicate: some, and at most every batch; its passes leave simulate()'s results untouched."""
    from dcor import _lib
    from dcor.sim import CellSpec, simulate
    cell = CellSpec(n=1000, rho=0.5, eps1=0.5, eps2=0.5, mu=(0.5, 0.5), sigma=(2.0, 2.0), seed=1_000_003)
    a = simulate(cell, 256, 0).cpu().numpy()
    c = cell.to_c()
    ties = np.zeros(256, dtype=np.int64)
    _lib.check(_lib.lib.dcor_diag_sign_ties(C.byref(c), 0, 256, ties.ctypes.data_as(C.POINTER(C.c_int64))))
    k = 1000 // 32
    assert 0 < ties.sum() and ties.max() <= k, ties
    b = simulate(cell, 256, 0).cpu().numpy()
    assert np.array_equal(a.view(np.int64), b.view(np.int64))
