## dcor.R -- drop-in R surface of the MI355X engine.
##
## Same names, arguments, defaults and return values as the reference's closures
## (vert-cor.R, ver-cor-subG.R, real-data-sims.R).  Each function draws its noise with the
## reference's own RNG calls, in the reference's order, at unit scale (extraDistr::rlaplace(.,0,1),
## rbinom, rnorm, rexp), so it consumes .Random.seed exactly like the reference, and hands the
## draws to the GPU through .Call; the engine scales them (scale * unit is bit-identical to
## rlaplace(., 0, scale)).  run_sim_one's grid path replaces mclapply with one .Call that runs
## replicates on the GPU from Philox streams keyed by the cell seed.
##
## dyn.load("dcor_r.so") first (see INTEGRATION.md).  R is absent from the build image, so this
## file is untested there; tests/ exercise the same C entry points through ctypes.

.unit_lap <- function(n) extraDistr::rlaplace(n, mu = 0, sigma = 1)

lambda_n <- function(n, eta = 1) .Call("dcor_R_lambda_n", as.double(n), as.double(eta))

lambda_INT_n <- function(n, eta_s = 1, eta_r = 1, eps_s = 1)
  .Call("dcor_R_lambda_INT_n", as.double(n), as.double(eta_s), as.double(eta_r), as.double(eps_s))

mixquant <- function(c, p, nsim = 1000) {
  # ver-cor-subG.R:8-13: draw order rnorm, rexp, rbinom
  z <- rnorm(nsim); e <- rexp(nsim); b <- rbinom(nsim, 1, 0.5)
  .Call("dcor_R_mixquant", z, e * (2 * b - 1), as.double(c), as.double(p))
}

.mix_draws <- function(nsim) {
  z <- rnorm(nsim); e <- rexp(nsim); b <- rbinom(nsim, 1, 0.5)
  list(z = z, l = e * (2 * b - 1))
}

priv_standardize <- function(vec, eps_norm, L_raw = 6) {
  lap <- .unit_lap(2)   # mu draw, then m2 draw (vert-cor.R:335-340)
  .Call("dcor_R_priv_standardize", as.double(vec), as.double(eps_norm), as.double(L_raw), lap)
}

ci_NI_signbatch <- function(X, Y, eps1, eps2, alpha = 0.05, normalise = T) {
  n <- length(X)
  m <- ceiling(8 / (eps1 * eps2)); k <- floor(n / m)
  stopifnot(k >= 1)
  lap_sc <- if (normalise == T) .unit_lap(4) else NULL   # X: mu, m2; Y: mu, m2
  lap_x <- .unit_lap(k); lap_y <- .unit_lap(k)
  o <- .Call("dcor_R_ci_NI_signbatch", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(alpha), as.logical(normalise), lap_sc, lap_x, lap_y)
  list(rho_hat = o[1], ci = o[2:3])
}

ci_INT_signflip <- function(X, Y, eps1, eps2, alpha = 0.05,
                            mode = c("auto", "normal", "laplace"), normalise = T) {
  stopifnot(length(X) == length(Y), eps1 > 0, eps2 > 0)
  n <- length(X); mode <- match.arg(mode)
  lap_sc <- if (normalise == T) .unit_lap(4) else NULL
  sender_is_X <- (eps1 >= eps2)
  eps_s <- if (sender_is_X) eps1 else eps2
  eps_r <- if (sender_is_X) eps2 else eps1
  p <- exp(eps_s) / (exp(eps_s) + 1)
  S <- rbinom(n, 1, p)
  lap_z <- .unit_lap(1)
  resolved <- if (mode == "auto") (if (sqrt(n) * eps_r > 0.5) "normal" else "laplace") else mode
  mx <- if (resolved == "normal") .mix_draws(1000) else list(z = 0, l = 0)
  o <- .Call("dcor_R_ci_INT_signflip", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(alpha), match(resolved, c("auto", "normal", "laplace")) - 1L,
             as.logical(normalise), lap_sc, as.integer(S), lap_z, mx$z, mx$l)
  list(rho_hat = o[1], ci = o[2:3], mode = resolved, roles = if (sender_is_X) "X→Y" else "Y→X")
}

correlation_NI_subG <- function(X, Y, eps1, eps2, eta1 = 1, eta2 = 1, alpha = 0.05,
                                lambda_X = NULL, lambda_Y = NULL, hrs = FALSE) {
  if (hrs) { ok <- !(is.na(X) | is.na(Y)); X <- X[ok]; Y <- Y[ok] }
  n <- length(X); stopifnot(n == length(Y))
  m <- ceiling(8 / (eps1 * eps2)); if (m > n) m <- n
  k <- floor(n / m)
  if (hrs) { if (k < 2) { k <- 2; m <- floor(n / k) } } else stopifnot(k >= 1)
  perm <- if (hrs) sample.int(n, k * m) - 1L else NULL
  lap_x <- .unit_lap(k); lap_y <- .unit_lap(k)
  o <- .Call("dcor_R_correlation_NI_subG", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(eta1), as.double(eta2), as.double(alpha), as.logical(hrs),
             if (is.null(lambda_X)) NA_real_ else as.double(lambda_X),
             if (is.null(lambda_Y)) NA_real_ else as.double(lambda_Y), perm, lap_x, lap_y)
  res <- list(rho_hat = o[1], ci = o[2:3])
  if (hrs) res <- c(res, list(k = k, m = m,
                              lambda_X = if (is.null(lambda_X)) lambda_n(n, eta1) else lambda_X,
                              lambda_Y = if (is.null(lambda_Y)) lambda_n(n, eta2) else lambda_Y))
  res
}

ci_INT_subG <- function(X, Y, eps1, eps2, eta1 = 1, eta2 = 1, alpha = 0.05,
                        mode = c("auto", "normal", "laplace"),
                        lambda_sender = NULL, lambda_other = NULL, lambda_receiver = NULL,
                        delta_clip = NULL, hrs = FALSE) {
  if (hrs) { ok <- !(is.na(X) | is.na(Y)); X <- X[ok]; Y <- Y[ok] }
  n <- length(X); stopifnot(n == length(Y))
  nsim <- if (hrs) 2000L else 1000
  lap_local <- .unit_lap(n); lap_c <- .unit_lap(1)
  mx <- .mix_draws(nsim)   # the sd(Uc)==0 branch (HRS) draws nothing there; see INTEGRATION.md
  nz <- function(v) if (is.null(v)) NA_real_ else as.double(v)
  o <- .Call("dcor_R_ci_INT_subG", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(eta1), as.double(eta2), as.double(alpha), as.logical(hrs), nz(lambda_sender),
             nz(lambda_other), nz(lambda_receiver), nz(delta_clip), lap_local, lap_c, mx$z, mx$l)
  list(rho_hat = o[1], ci = o[2:3], mode = mode, roles = if (eps1 >= eps2) "X→Y" else "Y→X")
}

dp_sd <- function(x, lo, hi, eps1, eps2) {
  x <- x[!is.na(x)]
  if (!length(x)) return(NA_real_)
  lap <- c(.unit_lap(1), .unit_lap(1))
  o <- .Call("dcor_R_dp_sd", as.double(x), as.double(lo), as.double(hi), as.double(eps1),
             as.double(eps2), lap)
  list(mean = o[1], sd = o[2])
}

## Fused grid: run_sim_one over many cells in one .Call (replaces mclapply).
## family: "sign" (vert-cor.R) or "subG" (ver-cor-subG.R);
## dgp: "gaussian"/"bernoulli"/"bounded_factor"/"mix_gaussian" (gen_mix_gaussian, whose
## arguments come in `mix`, defaults as ver-cor-subG.R:113-116).
## rng: "philox" (counter-based streams, shardable by replicate) or "R" (R's own
## Mersenne-Twister stream from set.seed(1e6 + i) per cell: the reference's per-seed numbers).
dcor_grid <- function(design, B = 250, alpha = 0.05, mu = c(0, 0), sigma = c(1, 1),
                      family = "sign", dgp = "gaussian", ci_mode = "auto", normalise = TRUE,
                      detail = FALSE,
                      mix = list(mu0 = c(0, 0), sigma0 = c(1, 1), mu1 = c(3, 3),
                                 sigma1 = c(2, 0.5), pi_mix = 0.5),
                      rng = c("philox", "R")) {
  rng <- match.arg(rng)
  nc <- nrow(design)
  fam <- rep(match(family, c("sign", "subG")) - 1L, length.out = nc)
  dg <- rep(match(dgp, c("gaussian", "bernoulli", "bounded_factor", "mix_gaussian")) - 1L,
            length.out = nc)
  mixv <- as.double(c(mix$mu0, mix$sigma0, mix$mu1, mix$sigma1, mix$pi_mix))
  r <- .Call("dcor_R_grid_run", fam, dg, as.double(design$n), as.double(design$rho),
             as.double(design$eps1), as.double(design$eps2), rep(as.double(alpha), nc),
             rep(mu[1], nc), rep(mu[2], nc), rep(sigma[1], nc), rep(sigma[2], nc),
             rep(as.logical(normalise), nc),
             rep(match(ci_mode, c("auto", "normal", "laplace")) - 1L, nc),
             as.double(1e6 + seq_len(nc)), as.double(B), as.logical(detail), mixv,
             identical(rng, "R"))
  s <- matrix(r[[1]], ncol = 5, byrow = TRUE,
              dimnames = list(NULL, c("mse", "bias", "var", "coverage", "ci_length")))
  summ <- data.frame(design[rep(seq_len(nc), each = 2), , drop = FALSE],
                     method = rep(c("NI", "INT"), nc), s, row.names = NULL)
  list(summary = summ, detail = if (detail) r[[2]] else NULL)
}
