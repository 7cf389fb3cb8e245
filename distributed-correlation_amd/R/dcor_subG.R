## dcor_subG.R -- the ver-cor-subG.R surface on the MI355X engine.  Source after dcor.R (as
## ver-cor-subG.R is sourced after vert-cor.R: it uses rLap, ci_NI_signbatch and
## ci_INT_signflip from there).  Same names, formals, defaults, RNG calls and return values as
## ver-cor-subG.R; see dcor.R for the conventions.

lambda_n <- function(n, eta = 1) .Call("dcor_R_lambda_n", as.double(n), as.double(eta))   # :1

lambda_INT_n <- function(n, eta_s = 1, eta_r = 1, eps_s = 1)                              # :3-7
  .Call("dcor_R_lambda_INT_n", as.double(n), as.double(eta_s), as.double(eta_r), as.double(eps_s))

mixquant <- function(c, p) {   # :8-13 (nsim = 1000)
  mx <- .mix_draws(1000)
  .Call("dcor_R_mixquant", mx$z, mx$l, as.double(c), as.double(p))
}

correlation_NI_subG <- function(X, Y, eps1, eps2,
                                eta1 = 1, eta2 = 1,
                                alpha = 0.05) {   # :25-62
  n <- length(X); stopifnot(n == length(Y))
  m <- ceiling(8 / (eps1 * eps2)); if (m > n) m <- n
  k <- floor(n / m); stopifnot(k >= 1)
  lap_x <- .unit_lap(k); lap_y <- .unit_lap(k)   # rLap(k) for X, then for Y (:48-49)
  o <- .Call("dcor_R_correlation_NI_subG", as.double(X), as.double(Y), as.double(eps1),
             as.double(eps2), as.double(eta1), as.double(eta2), as.double(alpha), FALSE,
             NA_real_, NA_real_, NULL, lap_x, lap_y)
  list(rho_hat = o[1], ci = o[2:3])
}

ci_INT_subG <- function(X, Y, eps1, eps2,
                        eta1 = 1, eta2 = 1,
                        alpha = 0.05,
                        mode  = c("auto","normal","laplace")) {   # :67-108
  n <- length(X); stopifnot(n == length(Y))
  lap_local <- .unit_lap(n)   # rLap(n, 2 lambda_s / eps_s) (:89 / :94)
  lap_c <- .unit_lap(1)       # rLap(1, 2 lambda_r / (n eps_r)) (:91 / :96)
  mx <- .mix_draws(1000)      # mixquant (:101)
  o <- .Call("dcor_R_ci_INT_subG", as.double(X), as.double(Y), as.double(eps1), as.double(eps2),
             as.double(eta1), as.double(eta2), as.double(alpha), FALSE, NA_real_, NA_real_,
             NA_real_, NA_real_, lap_local, lap_c, mx$z, mx$l)
  list(rho_hat = o[1], ci = o[2:3], mode = mode, roles = if (eps1 >= eps2) "X→Y" else "Y→X")
}

gen_mix_gaussian <- function(n, rho,
                             mu0    = c(0, 0), sigma0 = c(1, 1),
                             mu1    = c(3, 3), sigma1 = c(2, 0.5),
                             pi_mix = 0.5) {   # :115-136
  labels <- rbinom(n, 1, pi_mix)
  n0 <- sum(labels == 0);   n1 <- n - n0
  z0 <- rnorm(2 * n0)   # MASS::mvrnorm(n0, ...): matrix(rnorm(2 n0), n0)
  z1 <- rnorm(2 * n1)   # MASS::mvrnorm(n1, ...)
  idx <- sample.int(n)  # shuffle rows
  .Call("dcor_R_mix_gaussian", z0, as.double(n0), z1, as.double(n1), as.integer(idx - 1L),
        as.double(rho), as.double(mu0), as.double(sigma0), as.double(mu1), as.double(sigma1))
}

gen_bounded_factor <- function(n, rho) {   # :141-154
  cU <- sqrt(3 * rho)
  cE <- sqrt(3 * (1 - rho))
  U  <- runif(n, -cU,  cU)
  E1 <- runif(n, -cE,  cE)
  E2 <- runif(n, -cE,  cE)
  .Call("dcor_R_gen_bounded_factor", U, E1, E2)
}

## The engine's DGP code of a dgp_fun (and its arguments), or NA for a DGP it does not know.
.dgp_code <- function(dgp_fun, dgp_args) {
  if (identical(dgp_fun, gen_bounded_factor) && !length(dgp_args)) return(2L)
  if (identical(dgp_fun, gen_bernoulli) && !length(dgp_args)) return(1L)
  if (identical(dgp_fun, gen_mix_gaussian) &&
      all(names(dgp_args) %in% c("mu0", "sigma0", "mu1", "sigma1", "pi_mix"))) return(3L)
  if (identical(dgp_fun, gen_gaussian) && all(names(dgp_args) %in% "mu")) return(0L)
  NA_integer_
}

run_sim_one <- function(n, rho,
                        eps1, eps2,
                        dgp_fun  = gen_bounded_factor,
                        dgp_args = list(),
                        B        = 1000,
                        alpha    = 0.05,
                        use_subG = TRUE,
                        ci_mode  = "auto",
                        seed     = 2025L) {   # :159-222
  code <- .dgp_code(dgp_fun, dgp_args)
  if (!is.na(code)) {
    mix <- modifyList(list(mu0 = c(0, 0), sigma0 = c(1, 1), mu1 = c(3, 3), sigma1 = c(2, 0.5),
                           pi_mix = 0.5), if (code == 3L) dgp_args else list())
    mu <- if (code == 0L && !is.null(dgp_args$mu)) dgp_args$mu else c(0, 0)
    cell <- data.frame(family = if (use_subG) 1L else 0L, dgp = code, n = n, rho = rho,
                       eps1 = eps1, eps2 = eps2, alpha = alpha, mu1 = mu[1], mu2 = mu[2],
                       s1 = 1, s2 = 1, normalise = TRUE, ci_mode = .ci_mode_code(ci_mode),
                       seed = seed, nsim = 1000)
    r <- .dcor_run(cell, B, detail = TRUE,
                   mix = c(mix$mu0, mix$sigma0, mix$mu1, mix$sigma1, mix$pi_mix))
    rec <- matrix(r[[2]], ncol = 6, byrow = TRUE)
    out <- data.frame(repl = seq_len(B), ni_hat = rec[, 1], ni_low = rec[, 2], ni_up = rec[, 3],
                      int_hat = rec[, 4], int_low = rec[, 5], int_up = rec[, 6])
  } else {
    # a DGP the engine does not know: the reference's loop (:169-198), GPU estimators
    set.seed(seed)
    out <- data.frame(repl = seq_len(B), ni_hat = NA, ni_low = NA, ni_up = NA,
                      int_hat = NA, int_low = NA, int_up = NA)
    for (b in seq_len(B)) {
      XY <- do.call(dgp_fun, c(list(n = n, rho = rho), dgp_args))
      X <- XY[, 1]; Y <- XY[, 2]
      ni <- if (use_subG) correlation_NI_subG(X, Y, eps1, eps2, alpha = alpha)
            else ci_NI_signbatch(X, Y, eps1, eps2, alpha = alpha, normalise = TRUE)
      out$ni_hat[b] <- ni$rho_hat
      out$ni_low[b] <- ni$ci[1];  out$ni_up[b] <- ni$ci[2]
      int <- if (use_subG) ci_INT_subG(X, Y, eps1, eps2, alpha = alpha)
             else ci_INT_signflip(X, Y, eps1, eps2, alpha = alpha, mode = ci_mode, normalise = TRUE)
      out$int_hat[b] <- int$rho_hat
      out$int_low[b] <- int$ci[1]; out$int_up[b] <- int$ci[2]
    }
  }
  # :200-221
  out$ni_se2  <- (out$ni_hat  - rho)^2
  out$int_se2 <- (out$int_hat - rho)^2
  out$ni_cover  <- .r_cover(rho, out$ni_low, out$ni_up)
  out$int_cover <- .r_cover(rho, out$int_low, out$int_up)
  out$ni_ci_len <- out$ni_up  - out$ni_low
  out$int_ci_len<- out$int_up - out$int_low
  summarise <- function(est, se2, cov, len)
    c(mse = mean(se2), bias = mean(est) - rho, var = var(est),
      coverage = mean(cov), ci_length = mean(len))
  summary <- rbind(NI  = summarise(out$ni_hat,  out$ni_se2, out$ni_cover,  out$ni_ci_len),
                   INT = summarise(out$int_hat, out$int_se2, out$int_cover, out$int_ci_len))
  summary <- data.frame(method = rownames(summary), summary, row.names = NULL)
  list(detail = out, summary = summary)
}
