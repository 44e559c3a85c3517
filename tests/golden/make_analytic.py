"""Generate tests/golden/analytic_kats.json (closed-form known answers).

Run:  python tests/golden/make_analytic.py
Pure numpy; does not touch the reference or the oracle.
"""
import json
import os

import numpy as np


def ho_fixed_point(N=100, a=0.1, eta=0.8):
    """Fixed point of the C=0 gradient flow of tau_kernel.cl:68-117 for potID 0:
    (f[i+1]+f[i-1]-2 f[i])/a2 - 2 f[i] = 0 with ghosts f[-1] = -eta, f[N] = +eta
    (harmOscSol = 0, boundary(+-1) = +-eta), a2 = fp32(a)^2 rounded to fp32."""
    fa = np.float32(a)
    a2 = float(np.float32(fa * fa))
    A = np.zeros((N, N))
    b = np.zeros(N)
    for i in range(N):
        A[i, i] = -2.0 / a2 - 2.0
        if i > 0:
            A[i, i - 1] = 1.0 / a2
        else:
            b[i] -= -eta / a2
        if i < N - 1:
            A[i, i + 1] = 1.0 / a2
        else:
            b[i] -= eta / a2
    return np.linalg.solve(A, b)


def free_var_1d(h, V2=2.0, nk=1 << 16):
    """Stationary <f^2> of the Euler-Maruyama chain f' = f + h(lap f - V2 f) + sqrt(2h) xi
    (a = 1) in the bulk: integral dk/2pi [lam (1 - h lam/2)]^-1, lam = V2 + 2 - 2 cos k."""
    k = 2 * np.pi * (np.arange(nk) + 0.5) / nk
    lam = V2 + 2 - 2 * np.cos(k)
    return float(np.mean(1.0 / (lam * (1 - h * lam / 2))))


def free_var_3d(L, m2, h):
    """<phi^2> of the periodic L^3 free field under the same Euler step (lambda = 0)."""
    k = 2 * np.pi * np.arange(L) / L
    s = 2 - 2 * np.cos(k)
    lam = m2 + s[:, None, None] + s[None, :, None] + s[None, None, :]
    return float(np.mean(1.0 / (lam * (1 - h * lam / 2))))


def main():
    fp = ho_fixed_point()
    out = {
        "_provenance": "closed form, tests/golden/make_analytic.py (numpy only)",
        "ho_fixed_point": {"N": 100, "a": 0.1, "pot": 0, "C": 0.0, "f": fp.tolist()},
        "free_var_1d": {"a": 1.0, "V2": 2.0, "h": 0.01, "value": free_var_1d(0.01)},
        "free_var_3d_L16": {"L": 16, "m2": 1.0, "h": 0.01, "value": free_var_3d(16, 1.0, 0.01)},
        "free_var_3d_L32": {"L": 32, "m2": 1.0, "h": 0.01, "value": free_var_3d(32, 1.0, 0.01)},
        "free_var_3d_L64": {"L": 64, "m2": 1.0, "h": 0.01, "value": free_var_3d(64, 1.0, 0.01)},
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "analytic_kats.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(out["free_var_1d"], out["free_var_3d_L64"])


if __name__ == "__main__":
    main()
