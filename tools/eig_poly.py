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


def deflate(aq, bq, cq, d, e, f, w):
    """csrc/of3d_dev.hpp eigmin3_deflate: the smaller eigenvalue of the near-degenerate pair of
    B = (T - qI) / p from the 2x2 block on the plane orthogonal to lambda_max's eigenvector
    (scaled: entries O(1) whatever the tensor's magnitude; the caller multiplies by p)."""
    mu = 2 * (1 - (2 / 9) * w)
    m00, m11, m22 = aq - mu, bq - mu, cq - mu
    cr = [np.stack([d * f - e * m11, e * d - m00 * f, m00 * m11 - d * d], -1),
          np.stack([d * m22 - e * f, e * e - m00 * m22, m00 * f - d * e], -1),
          np.stack([m11 * m22 - f * f, f * e - d * m22, d * f - m11 * e], -1)]
    nr = [(c * c).sum(-1) for c in cr]
    v, nn = cr[0], nr[0]
    for c, k in zip(cr[1:], nr[1:]):  # the device's sequential "if (n > nn)" picks
        pick = k > nn
        v, nn = np.where(pick[..., None], c, v), np.where(pick, k, nn)
    v = v / np.sqrt(nn)[..., None]
    vx, vy, vz = v[..., 0], v[..., 1], v[..., 2]
    big = np.abs(vx) > np.abs(vy)
    s = 1 / np.sqrt(np.where(big, vx * vx + vz * vz, vy * vy + vz * vz))
    u = np.stack([np.where(big, -vz * s, 0.0), np.where(big, 0.0, vz * s), np.where(big, vx * s, -vy * s)], -1)
    wv = np.cross(v, u)
    E = np.stack([np.stack([aq, d, e], -1), np.stack([d, bq, f], -1), np.stack([e, f, cq], -1)], -2)
    e1 = np.einsum("...ij,...j->...i", E, u)
    e2 = np.einsum("...ij,...j->...i", E, wv)
    al, be, ga = (u * e1).sum(-1), (wv * e2).sum(-1), (u * e2).sum(-1)
    h = (al - be) * 0.5
    return (al + be) * 0.5 - np.sqrt(h * h + ga * ga)


DEFLATE_W = 1e-6  # the device's threshold on w = (1 - r) / 2 (fp64-rel instances)


def eigmin3(a, b, c, d, e, f, m=None, refine=False):
    """The device eigmin3 in numpy (m: polynomial form; None: the acos form it replaces;
    refine: the fp64-rel instances' deflation for w < DEFLATE_W)."""
    a, b, c, d, e, f = (np.asarray(v, np.float64) for v in (a, b, c, d, e, f))
    p1 = d * d + e * e + f * f
    q = (a + b + c) * (1 / 3)
    aq, bq, cq = a - q, b - q, c - q
    p2 = aq * aq + bq * bq + cq * cq + 2 * p1
    with np.errstate(divide="ignore", invalid="ignore"):
        p = np.sqrt(p2 * (1 / 6))
        ip = 1 / p
        B11, B22, B33, B12, B13, B23 = aq * ip, bq * ip, cq * ip, d * ip, e * ip, f * ip
        detB = B11 * (B22 * B33 - B23 * B23) - B12 * (B12 * B33 - B23 * B13) + B13 * (B12 * B23 - B22 * B13)
        r = np.clip(0.5 * detB, -1, 1)
        w = np.maximum((1 - r) * 0.5, 1e-290)
        if m is None:
            lam = q - 2 * p * np.cos(np.pi / 3 - np.arccos(r) / 3)
        else:
            lam = q - 2 * p * horner(m, 2 * np.sqrt(w) - 1)
        if refine:
            sel = (w < DEFLATE_W) & (p1 != 0)
            if sel.any():
                lam = lam.copy()
                lam[sel] = q[sel] + p[sel] * deflate(B11[sel], B22[sel], B33[sel], B12[sel], B13[sel], B23[sel],
                                                     w[sel])
    return np.where(p1 == 0, np.minimum(a, np.minimum(b, c)), lam)


def test_set(n=400000, seed=1, psd=False, extreme=False):
    """Symmetric 3x3 tensors with random orientation: generic spectra (three scales), and
    five hard sets — near-degenerate pairs, exact pairs (before rounding), a near-degenerate
    smallest pair, near-isotropic, rank 1.  extreme: magnitudes 1e-100 / 1e100 too (fp64 only:
    float32 cannot hold them).  Returns (the six entries, eigvalsh)."""
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, 3, 3)))
    scales = [1e-3, 1, 1e6] + ([1e-100, 1e100] if extreme else [])
    lam = rng.standard_normal((n, 3)) * rng.choice(scales, size=(n, 1))
    if psd:
        lam = np.abs(lam)
    k = n // 6
    lam[:k, 1] = lam[:k, 0] * (1 + rng.standard_normal(k) * 1e-9)  # near-degenerate pairs
    lam[k:2 * k, 2] = lam[k:2 * k, 0]  # exact pairs (before rounding)
    srt = np.sort(lam[2 * k:3 * k], axis=1)
    srt[:, 1] = srt[:, 0] * (1 + np.abs(rng.standard_normal(k)) * 10.0 ** rng.uniform(-16, -2, k))
    lam[2 * k:3 * k] = srt  # the smallest pair near-degenerate, at every distance
    lam[3 * k:4 * k, 1:] = lam[3 * k:4 * k, :1] * (1 + rng.standard_normal((k, 2)) * 1e-6)  # near-isotropic
    lam[4 * k:5 * k, 1:] = 0  # rank 1
    A = np.einsum("nij,nj,nkj->nik", Q, lam, Q)
    return (A[:, 0, 0], A[:, 1, 1], A[:, 2, 2], A[:, 0, 1], A[:, 0, 2], A[:, 1, 2]), np.linalg.eigvalsh(A)


def main():
    m = coefficients()
    uu = np.linspace(0, 1, 200001)
    print("degree %d, max |poly - cos(2/3 acos u)| = %.2e" % (DEG, np.abs(horner(m, 2 * uu - 1) - np.cos(2 / 3 * np.arccos(uu))).max()))
    print("coefficients (t^0 first):")
    for x in m:
        print("    %r" % float(x))
    for psd in (False, True):
        args, ref = test_set(psd=psd)
        lmax = np.abs(ref).max(axis=1)
        for name, mm, rf in (("acos form", None, False), ("polynomial form", m, False),
                             ("polynomial + deflation (fp64 rel)", m, True)):
            err = np.abs(eigmin3(*args, m=mm, refine=rf) - ref[:, 0]) / lmax
            print("%-4s %-36s max err / lambda_max %.3e" % ("psd" if psd else "any", name, err.max()))


if __name__ == "__main__":
    main()
