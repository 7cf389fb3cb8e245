"""dcor -- MI355X (gfx950) engine for the Monte-Carlo hot path of
abhinavc3/distributed-correlation (DP correlation estimation across two servers).

Host-side mirror of the reference's R function surface over the C-ABI in
include/dcor.h (libdcor.so).  Import fails loudly if the gfx950 library is missing.
"""
from ._lib import (DcorError, KLessThanOne, LIB_PATH, get_variant, lib, set_variant, variants)  # noqa: F401
from .api import (ci_INT_signflip, ci_INT_subG, ci_NI_signbatch, correlation_INT_signflip,  # noqa: F401
                  correlation_NI_subG, dp_mean, dp_sd, lambda_from_priv, lambda_INT_n, lambda_n,
                  lambda_receiver_from_noise, mixquant, priv_standardize, qnorm, rLap, set_seed,
                  standardize_dp)
from .sim import (CellSpec, headline_cell, paper_grid, run_cell, run_grid, run_sim_one,  # noqa: F401
                  run_sim_one_subG, simulate, subg_grid, vert_cor_grid)

__version__ = "0.1.0"
from . import rstream  # noqa: F401,E402
