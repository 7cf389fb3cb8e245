"""HRS BMI-vs-Age real-data study (real-data-sims.R) on the engine: panel ingest, DP
standardisation, the calibrated lambdas, and the replicate sweep of BASELINE config C5.

The reference loads `hrs_long_panel.rds`, keeps wave 2 complete cases of (agey_e, bmi)
(real-data-sims.R:13, 38-41), standardises both columns with a DP mean / sd
(real-data-sims.R:73-106, 273-287) and runs the NI and INT estimators on the standardised
panel (real-data-sims.R:290-323), then sweeps eps over seq(.25, 2.5, .1) with R = 200
replicates each (real-data-sims.R:345-448).

Ingesting the HRS panel itself waits for a data-licensing decision by the
project owner, so the repository ships no HRS microdata, nothing computed from them, and no
reader for them.  `standin_panel(n, rho)` is a generic synthetic panel of the same kind
(whole-year ages, one-decimal BMIs): each column is centred on its clip interval
(real-data-sims.R:260-261) with sd = interval width / 4; n and rho are the caller's.
"""
from __future__ import annotations

import math

import numpy as np

# real-data-sims.R:260-270
AGE_LO, AGE_HI = 45.0, 90.0
BMI_LO, BMI_HI = 15.0, 35.0
EPS_MEAN, EPS_M2 = 0.10, 0.10
EPS_CORR = 2.0
EPS_GRID = tuple(round(0.25 + 0.1 * i, 10) for i in range(23))  # seq(0.25, 2.5, by = 0.1)
R_PER_EPS = 200
NI_SEED, INT_SEED = 231, 322                                     # set.seed (:289, :312)


def standin_panel(n: int, rho: float, seed: int = 2):
    """Synthetic raw (age, bmi): whole-year ages and one-decimal BMIs from a bivariate normal
    centred on the clip intervals with sd = width / 4 and correlation rho."""
    g = np.random.default_rng(seed)
    za = g.standard_normal(n)
    zb = rho * za + math.sqrt(1.0 - rho * rho) * g.standard_normal(n)
    age = np.round(0.5 * (AGE_LO + AGE_HI) + 0.25 * (AGE_HI - AGE_LO) * za)
    bmi = np.round(0.5 * (BMI_LO + BMI_HI) + 0.25 * (BMI_HI - BMI_LO) * zb, 1)
    return age, bmi


def standardize_panel(age, bmi, lap=None, rng=None):
    """dp_sd of both columns, standardize_dp, lambda_from_priv (real-data-sims.R:273-287).
    lap: optional unit Laplace draws [age mean, age m2, bmi mean, bmi m2]."""
    from . import api
    lap = np.asarray(api.unit_laplace(4, rng) if lap is None else lap, dtype=np.float64)
    age_priv = api.dp_sd(age, AGE_LO, AGE_HI, EPS_MEAN, EPS_M2, lap=lap[:2])
    bmi_priv = api.dp_sd(bmi, BMI_LO, BMI_HI, EPS_MEAN, EPS_M2, lap=lap[2:])
    age_z = api.standardize_dp(age, age_priv, AGE_LO, AGE_HI)
    bmi_z = api.standardize_dp(bmi, bmi_priv, BMI_LO, BMI_HI)
    ok = ~(np.isnan(age_z) | np.isnan(bmi_z))                      # drop_na (:282)
    return {"age_z": np.ascontiguousarray(age_z[ok]), "bmi_z": np.ascontiguousarray(bmi_z[ok]),
            "age_priv": age_priv, "bmi_priv": bmi_priv,
            "lambda_age_z": api.lambda_from_priv(AGE_LO, AGE_HI, age_priv),
            "lambda_bmi_z": api.lambda_from_priv(BMI_LO, BMI_HI, bmi_priv)}
