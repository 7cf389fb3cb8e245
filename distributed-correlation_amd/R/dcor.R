## dcor.R -- drop-in R surface of the MI355X engine: the vert-cor.R functions, plus the grid.
##
## Three files mirror the reference's three scripts, which redefine each other's names
## (run_sim_one, mixquant, correlation_NI_subG, ci_INT_subG, rLap, lambda_n; SURVEY.md §1):
##   dcor.R        vert-cor.R        (source this first: it also holds the shared internals)
##   dcor_subG.R   ver-cor-subG.R    (source after dcor.R, as ver-cor-subG.R after vert-cor.R)
##   dcor_hrs.R    real-data-sims.R  (its DP helpers and HRS estimator variants)
## Every function keeps the reference's name, formals, defaults and return value.  Each makes
## the reference's own RNG calls in the reference's order (extraDistr::rlaplace, rbinom, rnorm,
## rexp, runif, sample.int), so .Random.seed advances exactly as under the reference, and hands
## the draws to the GPU through .Call, where the arithmetic runs in R's operation order.
##
## run_sim_one runs its replicates on the GPU in one .Call.  options(dcor.rng = "philox")
## (default) draws them from the engine's counter-based Philox streams keyed by `seed`; "R"
## replays R's own stream from set.seed(seed), i.e. the reference's replicates (up to libm's
## rounding of log, DESIGN.md).  A DGP the engine does not know runs the reference's loop with
## the GPU estimators below.  dcor_grid() replaces the mclapply grid blocks with one .Call over
## any number of GPUs.  HIP does not survive fork(): call the engine from the parent process,
## never from mclapply children (the library fails with DCOR_EFORK there).
##
## dyn.load("dcor_r.so") first (INTEGRATION.md).  R is absent from the build image: this file
## is parsed by tests/test_r_surface.py (formals against the reference's) and its .Call
## targets are executed through a stub R runtime by tests/test_r_shim.py.

.unit_lap <- function(n) extraDistr::rlaplace(n, mu = 0, sigma = 1)

.mix_draws <- function(nsim) {
  # mixquant's draws in R's evaluation order: rnorm, rexp, rbinom (vert-cor.R:47)
  z <- rnorm(nsim); e <- rexp(nsim); b <- rbinom(nsim, 1, 0.5)
  list(z = z, l = e * (2 * b - 1))
}

.dcor_rng <- function() {
  r <- getOption("dcor.rng", "philox")
  if (!r %in% c("philox", "R")) stop("options(dcor.rng) must be \"philox\" or \"R\"")
  r
}

.dcor_devices <- function() as.integer(getOption("dcor.devices", integer(0)))

## One grid through the engine.  cells: data.frame with one row per cell (columns family, dgp,
## n, rho, eps1, eps2, alpha, mu1, mu2, s1, s2, normalise, ci_mode, seed, nsim and, for
## gen_mix_gaussian, mix = c(mu0, sigma0, mu1, sigma1, pi_mix)).  Returns the summaries
## [cell][method][mse, bias, var, coverage, ci_length] and, with detail, the replicate records.
.dcor_run <- function(cells, B, detail, rng = .dcor_rng(), mix = c(0, 0, 1, 1, 3, 3, 2, 0.5, 0.5),
                      devices = .dcor_devices()) {
  nc <- nrow(cells)
  .Call("dcor_R_grid_run",
        as.integer(cells$family), as.integer(cells$dgp), as.double(cells$n), as.double(cells$rho),
        as.double(cells$eps1), as.double(cells$eps2), as.double(cells$alpha),
        as.double(cells$mu1), as.double(cells$mu2), as.double(cells$s1), as.double(cells$s2),
        as.logical(cells$normalise), as.integer(cells$ci_mode), as.double(cells$seed),
        as.double(B), as.logical(detail), as.double(mix), identical(rng, "R"),
        as.double(cells$nsim), as.integer(devices))
}

.ci_mode_code <- function(m) match(m[1], c("auto", "normal", "laplace")) - 1L

## R's `rho >= lo && rho <= up` per replicate (FALSE wins over NA, NA over TRUE).
.r_cover <- function(rho, lo, up) rho >= lo & rho <= up

## run_sim_one's detail and summary frames from the engine's replicate records.
.sign_frames <- function(rec, rho, B) {
  r <- matrix(rec, ncol = 6, byrow = TRUE)
  ni_hat <- r[, 1]; ni_low <- r[, 2]; ni_up <- r[, 3]
  int_hat <- r[, 4]; int_low <- r[, 5]; int_up <- r[, 6]
  # vert-cor.R:367-385 column order
  out <- data.frame(repl = seq_len(B), ni_hat = ni_hat, int_hat = int_hat,
                    ni_se2 = (ni_hat - rho)^2, int_se2 = (int_hat - rho)^2,
                    ni_low = ni_low, ni_up = ni_up, int_low = int_low, int_up = int_up,
                    # integer 0/1/NA: vert-cor.R:381-382 starts the columns as NA_integer_ and
                    # assigns the logical cover into them (:405, :416)
                    ni_cover = as.integer(.r_cover(rho, ni_low, ni_up)),
                    int_cover = as.integer(.r_cover(rho, int_low, int_up)),
                    ni_ci_len = ni_up - ni_low, int_ci_len = int_up - int_low)
  summarise <- function(est, se2, cover, lo, up)   # vert-cor.R:422-430
    c(mse = mean(se2), bias = mean(est) - rho, var = var(est), coverage = mean(cover),
      ci_length = mean(up - lo))
  summ_df <- rbind(NI = summarise(out$ni_hat, out$ni_se2, out$ni_cover, out$ni_low, out$ni_up),
                   INT = summarise(out$int_hat, out$int_se2, out$int_cover, out$int_low, out$int_up))
  summ_df <- as.data.frame(summ_df)
  summ_df$method <- rownames(summ_df)
  rownames(summ_df) <- NULL
  list(detail = out, summary = summ_df)
}

## =========================================================== vert-cor.R ====
mixquant <- function(c, p) {   # vert-cor.R:44-49 (nsim = 1000)
  mx <- .mix_draws(1000)
  .Call("dcor_R_mixquant", mx$z, mx$l, as.double(c), as.double(p))
}

gen_gaussian <- function(n, rho, mu = c(0, 0)) {   # vert-cor.R:64-73
  z <- rnorm(2 * n)   # MASS::mvrnorm: matrix(rnorm(p * n), n)
  xy <- .Call("dcor_R_mvrnorm", z, as.double(n), as.double(mu), c(1, 1), as.double(rho))
  if (n == 1) drop(xy) else xy
}

gen_bernoulli <- function(n, rho) {   # vert-cor.R:78-98
  stopifnot(abs(rho) <= 1)
  u <- runif(n)
  v <- runif(n)
  xy <- .Call("dcor_R_gen_bernoulli", u, v, as.double(rho))
  colnames(xy) <- c("X", "Y")
  xy
}

rLap <- function(n = 1, scale) extraDistr::rlaplace(n, mu = 0, sigma = scale)   # vert-cor.R:106

correlation_INT_signflip <- function(X, Y, eps1, eps2) {   # vert-cor.R:164-195
  stopifnot(length(X) == length(Y), eps1 > 0, eps2 > 0)
  n <- length(X)
  eps_s <- if (eps1 >= eps2) eps1 else eps2
  p <- exp(eps_s) / (exp(eps_s) + 1)
  S <- rbinom(n, 1, p)
  lap_z <- .unit_lap(1)
  # the point estimate of ci_INT_signflip(normalise = F): no standardisation, no mixquant
  o <- .Call("dcor_R_ci_INT_signflip", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             0.05, 2L, FALSE, NULL, as.integer(S), lap_z, 0, 0)
  o[1]
}

ci_NI_signbatch <- function(X, Y, eps1, eps2, alpha = 0.05, normalise = T) {   # vert-cor.R:204-255
  n <- length(X)
  m <- ceiling(8 / (eps1 * eps2)); k <- floor(n / m)
  stopifnot(k >= 1)
  lap_sc <- if (normalise == T) .unit_lap(4) else NULL   # X: mu, m2; Y: mu, m2 (:214-215)
  lap_x <- .unit_lap(k); lap_y <- .unit_lap(k)            # :230-231
  o <- .Call("dcor_R_ci_NI_signbatch", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(alpha), as.logical(normalise), lap_sc, lap_x, lap_y)
  list(rho_hat = o[1], ci = o[2:3])
}

ci_INT_signflip <- function(X, Y, eps1, eps2, alpha = 0.05,
                            mode = c("auto", "normal", "laplace"), normalise = T) {   # vert-cor.R:260-317
  stopifnot(length(X) == length(Y), eps1 > 0, eps2 > 0)
  n <- length(X); mode <- match.arg(mode)
  lap_sc <- if (normalise == T) .unit_lap(4) else NULL   # :271-272
  sender_is_X <- (eps1 >= eps2)
  eps_s <- if (sender_is_X) eps1 else eps2
  eps_r <- if (sender_is_X) eps2 else eps1
  p <- exp(eps_s) / (exp(eps_s) + 1)
  S <- rbinom(n, 1, p)                                   # :175
  lap_z <- .unit_lap(1)                                  # :188
  resolved <- if (mode == "auto") (if (sqrt(n) * eps_r > 0.5) "normal" else "laplace") else mode
  mx <- if (resolved == "normal") .mix_draws(1000) else list(z = 0, l = 0)   # :302
  o <- .Call("dcor_R_ci_INT_signflip", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(alpha), .ci_mode_code(resolved), as.logical(normalise), lap_sc,
             as.integer(S), lap_z, mx$z, mx$l)
  list(rho_hat = o[1], ci = o[2:3], mode = resolved, roles = if (sender_is_X) "X→Y" else "Y→X")
}

priv_standardize <- function(vec, eps_norm, L_raw = 6) {   # vert-cor.R:322-348
  lap <- .unit_lap(2)   # mu draw, then m2 draw (:335-340)
  .Call("dcor_R_priv_standardize", as.double(vec), as.double(eps_norm), as.double(L_raw), lap)
}

run_sim_one <- function(n, rho, eps1, eps2,
                        mu = c(0, 0), sigma = c(1, 1),
                        B      = 1000,
                        alpha  = 0.05,
                        ci_mode = "auto",
                        normalise = T,
                        seed   = 2025L) {   # vert-cor.R:356-444
  cell <- data.frame(family = 0L, dgp = 0L, n = n, rho = rho, eps1 = eps1, eps2 = eps2,
                     alpha = alpha, mu1 = mu[1], mu2 = mu[2], s1 = sigma[1], s2 = sigma[2],
                     normalise = normalise == T, ci_mode = .ci_mode_code(ci_mode), seed = seed,
                     nsim = 1000)
  r <- .dcor_run(cell, B, detail = TRUE)
  .sign_frames(r[[2]], rho, B)
}

## ================================================================= grid ====
## Every cell of `design` (data.frame with n, rho, eps1, eps2; one row per cell) for B
## replicates in one .Call: replaces the expand.grid + mclapply blocks of vert-cor.R:486-554
## and ver-cor-subG.R:245-296, and the merge + summary blocks after them: `detail_all` (with
## detail = TRUE) and `summ_all` are the tables of vert-cor.R:556-597 / ver-cor-subG.R:301-333
## (columns, order, cover type and data.table's group order), so the figure code after them runs
## unchanged.  Cell i is seeded 1e6 + i as there.  family "sign" / "subG";
## dgp "gaussian" / "bernoulli" / "bounded_factor" / "mix_gaussian" (gen_mix_gaussian's
## arguments in `mix`).  rng "philox" shards replicates over `devices` (0-based HIP ids; all
## visible GPUs by default); "R" replays R's own streams cell by cell.
dcor_grid <- function(design, B = 250, alpha = 0.05, mu = c(0, 0), sigma = c(1, 1),
                      family = "sign", dgp = "gaussian", ci_mode = "auto", normalise = TRUE,
                      detail = FALSE,
                      mix = list(mu0 = c(0, 0), sigma0 = c(1, 1), mu1 = c(3, 3),
                                 sigma1 = c(2, 0.5), pi_mix = 0.5),
                      rng = c("philox", "R"), devices = .dcor_devices()) {
  rng <- match.arg(rng)
  nc <- nrow(design)
  cells <- data.frame(family = rep(match(family, c("sign", "subG")) - 1L, length.out = nc),
                      dgp = rep(match(dgp, c("gaussian", "bernoulli", "bounded_factor",
                                             "mix_gaussian")) - 1L, length.out = nc),
                      n = design$n, rho = design$rho, eps1 = design$eps1, eps2 = design$eps2,
                      alpha = alpha, mu1 = mu[1], mu2 = mu[2], s1 = sigma[1], s2 = sigma[2],
                      normalise = normalise, ci_mode = .ci_mode_code(ci_mode),
                      seed = 1e6 + seq_len(nc), nsim = 1000)
  mixv <- as.double(c(mix$mu0, mix$sigma0, mix$mu1, mix$sigma1, mix$pi_mix))
  r <- .dcor_run(cells, B, detail = detail, rng = rng, mix = mixv, devices = devices)
  s <- matrix(r[[1]], ncol = 5, byrow = TRUE,
              dimnames = list(NULL, c("mse", "bias", "var", "coverage", "ci_length")))
  summ <- data.frame(design[rep(seq_len(nc), each = 2), , drop = FALSE],
                     method = rep(c("NI", "INT"), nc), s, row.names = NULL)
  as_dt <- function(x) if (!is.null(x) && requireNamespace("data.table", quietly = TRUE))
    data.table::setDT(x) else x
  list(summary = summ, detail = if (detail) r[[2]] else NULL,
       detail_all = as_dt(r[[3]]), summ_all = as_dt(r[[4]]))
}
