## dcor_hrs.R -- the real-data-sims.R surface on the MI355X engine: its DP building blocks and
## its variants of the sub-G estimators (pairwise-complete inputs, lambda overrides, random
## batches, the receiver bound from the sender's noise, mixquant with nsim = 2000).  Source after
## dcor.R; like real-data-sims.R it redefines rLap, lambda_n, lambda_INT_n, mixquant,
## correlation_NI_subG and ci_INT_subG.  See dcor.R for the conventions.

rLap <- function(n, scale) {   # :58-61 (inverse CDF on runif(n, -0.5, 0.5))
  u <- runif(n, -0.5, 0.5)
  -scale * sign(u) * log(1 - 2 * abs(u))
}

.unit_lap_hrs <- function(n) rLap(n, 1)   # scale * unit is bit-identical to rLap(n, scale)

dp_mean <- function(x, lo, hi, eps) {   # :64-70
  x <- x[!is.na(x)]
  if (!length(x)) return(NA_real_)
  .Call("dcor_R_dp_mean", as.double(x), as.double(lo), as.double(hi), as.double(eps),
        .unit_lap_hrs(1))
}

dp_sd <- function(x, lo, hi, eps1, eps2) {   # :73-84
  x <- x[!is.na(x)]
  if (!length(x)) return(NA_real_)
  lap <- c(.unit_lap_hrs(1), .unit_lap_hrs(1))   # dp_mean's draw, then the second moment's
  o <- .Call("dcor_R_dp_sd", as.double(x), as.double(lo), as.double(hi), as.double(eps1),
             as.double(eps2), lap)
  list(mean = o[1], sd = o[2])
}

standardize_dp <- function(x, priv, lo, hi, eps = 1e-8)   # :87-90
  .Call("dcor_R_standardize_dp", as.double(x), as.double(lo), as.double(hi),
        as.double(priv$mean), as.double(priv$sd), as.double(eps))

standardize_age_bmi <- function(age, bmi,
                                age_priv, bmi_priv,
                                age_lo, age_hi, bmi_lo, bmi_hi,
                                eps = 1e-8) {   # :92-100
  z <- list(age_z = standardize_dp(age, age_priv, age_lo, age_hi, eps),
            bmi_z = standardize_dp(bmi, bmi_priv, bmi_lo, bmi_hi, eps))
  if (requireNamespace("tibble", quietly = TRUE)) tibble::as_tibble(z) else as.data.frame(z)
}

lambda_from_priv <- function(lo, hi, priv, eps_sd = 1e-8)   # :103-106
  .Call("dcor_R_lambda_from_priv", as.double(lo), as.double(hi), as.double(priv$mean),
        as.double(priv$sd), as.double(eps_sd))

lambda_n <- function(n, eta = 1) .Call("dcor_R_lambda_n", as.double(n), as.double(eta))   # :109

correlation_NI_subG <- function(X, Y, eps1, eps2,
                                eta1 = 1, eta2 = 1,
                                alpha = 0.05,
                                lambda_X = NULL, lambda_Y = NULL) {   # :115-147
  ok <- !(is.na(X) | is.na(Y))
  X <- X[ok]; Y <- Y[ok]
  n <- length(X); stopifnot(n == length(Y), n >= 2)
  m <- ceiling(8 / (eps1 * eps2)); if (m > n) m <- n
  k <- floor(n / m); if (k < 2) { k <- 2; m <- floor(n / k) }
  idx <- sample.int(n, k * m)                            # :131
  lap_x <- .unit_lap_hrs(k); lap_y <- .unit_lap_hrs(k)   # :136-137
  o <- .Call("dcor_R_correlation_NI_subG", as.double(X), as.double(Y), as.double(eps1),
             as.double(eps2), as.double(eta1), as.double(eta2), as.double(alpha), TRUE,
             if (is.null(lambda_X)) NA_real_ else as.double(lambda_X),
             if (is.null(lambda_Y)) NA_real_ else as.double(lambda_Y),
             as.integer(idx - 1L), lap_x, lap_y)
  list(rho_hat = o[1], ci = o[2:3], k = k, m = m,
       lambda_X = if (!is.null(lambda_X)) lambda_X else lambda_n(n, eta1),
       lambda_Y = if (!is.null(lambda_Y)) lambda_Y else lambda_n(n, eta2))
}

lambda_INT_n <- function(n, eta_s = 1, eta_r = 1, eps_s = 1)   # :154-158
  .Call("dcor_R_lambda_INT_n", as.double(n), as.double(eta_s), as.double(eta_r), as.double(eps_s))

mixquant <- function(c, p, nsim = 2000L) {   # :161-164
  mx <- .mix_draws(nsim)
  .Call("dcor_R_mixquant", mx$z, mx$l, as.double(c), as.double(p))
}

lambda_receiver_from_noise <- function(lambda_sender, lambda_other,
                                       eps_sender, delta_per_sample)   # :170-174
  .Call("dcor_R_lambda_receiver_from_noise", as.double(lambda_sender), as.double(lambda_other),
        as.double(eps_sender), as.double(delta_per_sample))

ci_INT_subG <- function(X, Y, eps1, eps2,
                        eta1 = 1, eta2 = 1,
                        alpha = 0.05,
                        mode  = c("auto","normal","laplace"),
                        lambda_sender   = NULL,
                        lambda_other    = NULL,
                        lambda_receiver = NULL,
                        delta_clip      = NULL
) {   # :176-252
  ok <- !(is.na(X) | is.na(Y))
  X <- X[ok]; Y <- Y[ok]
  n <- length(X); stopifnot(n == length(Y), n >= 2)
  sender_is_X <- (eps1 >= eps2)
  eps_s <- if (sender_is_X) eps1 else eps2
  eta_s <- if (sender_is_X) eta1 else eta2
  eta_r <- if (sender_is_X) eta2 else eta1
  if (is.null(delta_clip)) delta_clip <- 1 / n                                 # :199
  if (is.null(lambda_sender) || is.null(lambda_other)) {                      # :202-208
    lam <- lambda_INT_n(n, eta_s = eta_s, eta_r = eta_r, eps_s = eps_s)
    if (is.null(lambda_sender)) lambda_sender <- lam[1]
    if (is.null(lambda_other)) lambda_other <- lambda_n(n, if (sender_is_X) eta2 else eta1)
  }
  if (is.null(lambda_receiver))                                                # :211-218
    lambda_receiver <- lambda_receiver_from_noise(lambda_sender, lambda_other, eps_s, delta_clip)
  lap_local <- .unit_lap_hrs(n)   # rLap(n, 2 lambda_sender / eps_s) (:224 / :228)
  lap_c <- .unit_lap_hrs(1)       # rLap(1, 2 lambda_receiver / (n eps_r)) (:233)
  lam <- as.double(c(lambda_sender, lambda_other, lambda_receiver, delta_clip))
  # sd(Uc) == 0 takes the closed-form width and draws nothing more (:236-238); otherwise
  # mixquant(cstar, 1 - alpha/2) draws its 2000 values (:240-241)
  sd_uc <- .Call("dcor_R_int_subg_sd_uc", as.double(X), as.double(Y), as.double(eps1),
                 as.double(eps2), as.double(eta1), as.double(eta2), lam, lap_local)
  mx <- if (sd_uc == 0) list(z = 0, l = 0) else .mix_draws(2000L)
  o <- .Call("dcor_R_ci_INT_subG", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(eta1), as.double(eta2), as.double(alpha), TRUE, lam[1], lam[2], lam[3],
             lam[4], lap_local, lap_c, mx$z, mx$l)
  list(rho_hat = o[1], ci = o[2:3], roles = if (sender_is_X) "X→Y" else "Y→X",
       lambda_sender = lambda_sender, lambda_other = lambda_other,
       lambda_receiver = lambda_receiver, delta_clip = delta_clip)
}
