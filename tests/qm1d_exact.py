"""Exact stationary covariance of the linear (potID 0) QM1D chain under the
Euler-Maruyama update, for the two orderings (test utility, numpy/scipy only).

  drift   M f = (f[i+1] + f[i-1] - 2 f[i]) / a2 - 2 f[i]   (tau_kernel.cl:111-117,
          V'' = 2 for harmOscPot; the Dirichlet ghosts only shift the mean)
  noise   sqrt(2 h / a) xi                                   (tau_kernel.cl:112)

  Jacobi        f' = (I + h M) f + s xi                   -> Sigma = A Sigma A^T + s^2 I
  Gauss-Seidel  (I - h L) f' = (I + h (M - L)) f + s xi  (L = strict lower part of M;
                the reference's order under a serialising runtime)

The two differ at O(h): at dtau/dt^2 = 0.2 the mid-chain variance is 0.366
(Jacobi) vs 0.442 (Gauss-Seidel) against 0.353 for dtau -> 0.
"""
import numpy as np
import scipy.linalg as sl


def drift_matrix(N, a):
    fa = np.float32(a)
    a2 = float(np.float32(fa * fa))   # pown((float)deltat, 2)
    lap = (np.diag(np.ones(N - 1), 1) + np.diag(np.ones(N - 1), -1) - 2 * np.eye(N)) / a2
    return lap - 2 * np.eye(N)


def stationary_cov(N, a, h, order="jacobi", C=1.0):
    M = drift_matrix(N, a)
    s2 = C * C * 2 * h / a
    if order == "jacobi":
        return sl.solve_discrete_lyapunov(np.eye(N) + h * M, s2 * np.eye(N))
    low = np.tril(M, -1)
    Q = np.linalg.inv(np.eye(N) - h * low)
    B = Q @ (np.eye(N) + h * (M - low))
    return sl.solve_discrete_lyapunov(B, s2 * Q @ Q.T)


def block_error(samples, nblocks=10):
    s = np.asarray(samples)
    n = len(s) // nblocks * nblocks
    b = s[:n].reshape(nblocks, -1).mean(axis=1)
    return b.mean(), b.std(ddof=1) / np.sqrt(nblocks)
