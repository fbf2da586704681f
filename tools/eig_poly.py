"""Coefficients of cos((2/3) acos(u)) on u in [0, 1] as a polynomial in t = 2u - 1 (the
eigenvalue's trigonometric step in csrc/of3d_dev.hpp: cos_two_thirds_acos), and a check of
the eigenvalue formula that uses it against the acos form and numpy's eigvalsh.

    python tools/eig_poly.py          # prints the coefficients and the comparison

Degree 16: max error 1.4e-15 on [0, 1] (Chebyshev fit at 40001 Chebyshev points, converted to
monomials in t; |coefficients| <= 0.77, so Horner in t is stable)."""
import numpy as np
from numpy.polynomial import chebyshev as C

DEG = 16


def coefficients(deg=DEG):
    u = np.cos(np.linspace(0, np.pi, 40001)) * 0.5 + 0.5
    c = C.chebfit(2 * u - 1, np.cos(2.0 / 3.0 * np.arccos(u)), deg)
    return C.cheb2poly(c)  # monomial coefficients in t, lowest first


def horner(m, t):
    v = np.zeros_like(t)
    for a in m[::-1]:
        v = v * t + a
    return v


def eigmin3(a, b, c, d, e, f, m=None):
    """The device eigmin3 in numpy (m: polynomial form; None: the acos form it replaces)."""
    p1 = d * d + e * e + f * f
    q = (a + b + c) * (1 / 3)
    aq, bq, cq = a - q, b - q, c - q
    p2 = aq * aq + bq * bq + cq * cq + 2 * p1
    p = np.sqrt(p2 * (1 / 6))
    ip = 1 / p
    B11, B22, B33, B12, B13, B23 = aq * ip, bq * ip, cq * ip, d * ip, e * ip, f * ip
    detB = B11 * (B22 * B33 - B23 * B23) - B12 * (B12 * B33 - B23 * B13) + B13 * (B12 * B23 - B22 * B13)
    r = np.clip(0.5 * detB, -1, 1)
    if m is None:
        lam = q - 2 * p * np.cos(np.pi / 3 - np.arccos(r) / 3)
    else:
        lam = q - 2 * p * horner(m, 2 * np.sqrt((1 - r) * 0.5) - 1)
    return np.where(p1 == 0, np.minimum(a, np.minimum(b, c)), lam)


def main():
    m = coefficients()
    uu = np.linspace(0, 1, 200001)
    print("degree %d, max |poly - cos(2/3 acos u)| = %.2e" % (DEG, np.abs(horner(m, 2 * uu - 1) - np.cos(2 / 3 * np.arccos(uu))).max()))
    print("coefficients (t^0 first):")
    for x in m:
        print("    %r" % float(x))
    rng = np.random.default_rng(1)
    n = 400000
    Q, _ = np.linalg.qr(rng.standard_normal((n, 3, 3)))
    lam = rng.standard_normal((n, 3)) * rng.choice([1e-3, 1, 1e6], size=(n, 1))
    k = n // 4
    lam[:k, 1] = lam[:k, 0] * (1 + rng.standard_normal(k) * 1e-9)  # near-degenerate pairs
    lam[k:2 * k, 2] = lam[k:2 * k, 0]  # exact pairs (before rounding)
    A = np.einsum("nij,nj,nkj->nik", Q, lam, Q)
    args = (A[:, 0, 0], A[:, 1, 1], A[:, 2, 2], A[:, 0, 1], A[:, 0, 2], A[:, 1, 2])
    ref = np.linalg.eigvalsh(A)
    lmax = np.abs(ref).max(axis=1)
    for name, mm in (("acos form", None), ("polynomial form", m)):
        err = np.abs(eigmin3(*args, m=mm) - ref[:, 0]) / lmax
        print("%-16s max err / lambda_max %.3e" % (name, err.max()))


if __name__ == "__main__":
    main()
