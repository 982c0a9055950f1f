"""The two conservative 8x8-quadrant bounds of the blends, restated on the CPU (float32, step for step):

* k_emit's per-(Gaussian, tile row) band bound (csrc/gsr_common.h span_prep / span_quads / quads_of_tile), which
  the unpacked tile keys carry as each instance's 4-bit quadrant mask (the quadrant-wave forward gathers only its
  quadrant's candidates from it, the C5 tile-wave backward culls from it);
* the blends' per-(candidate, quadrant) test on the staged conic (csrc/gsr_kernels.h quadrant_hit: the minimum of
  the conic's quadratic form over the quadrant's pixel-centre rectangle).

They are different tests: the outputs do not depend on them agreeing, only on each keeping every
quadrant that holds a pixel whose blend condition (power <= 0 and alpha = min(0.99, o exp(power)) >= 1/255, the
kernels' fp32 exponent) holds.  Checked here on rotated, needle-like, faint, large and tile-edge ellipses; the
number of quadrants one bound keeps and the other drops is reported (both beyond every blending pixel).
"""
import numpy as np
import pytest

f32 = np.float32
ALPHA_MIN = f32(1.0 / 255.0)


def span_prep(px, py, a, b, c, o):
    D = f32(a * c) - f32(b * b)
    mode = 0 if not (o >= f32(ALPHA_MIN * f32(0.9999))) else (1 if not (a > 0 and c > 0 and D > 0) else 2)
    tau = max(f32(0.0), f32(np.log(f32(f32(255.0) * o))))
    thr = f32(2.0) * f32(f32(tau * f32(1.002)) + f32(2e-3))
    ia = f32(1.0) / a
    ue = f32(np.sqrt(f32(f32(thr * c) * (f32(1.0) / D)))) if mode == 2 else f32(0)
    ve = f32(f32(b * ue) * (f32(1.0) / c)) if mode == 2 else f32(0)
    return dict(px=px, py=py, b=b, D=D, ia=ia, thra=f32(thr * a), ue=ue, ve=ve, mode=mode)


def span_quads(p, v1):
    if p["mode"] != 2:
        return (0x7fff << 16) if p["mode"] == 1 else 0
    v0 = f32(v1 - f32(7.0))
    umax, umin = f32(-3.0e38), f32(3.0e38)
    if v0 <= -p["ve"] <= v1:
        umax = p["ue"]
    if v0 <= p["ve"] <= v1:
        umin = -p["ue"]
    for v in (v0, v1):
        e = f32(p["thra"] - f32(p["D"] * f32(v * v)))
        if e >= 0:
            r, m = f32(np.sqrt(e)), f32(-p["b"] * v)
            umax = max(umax, f32(f32(m + r) * p["ia"]))
            umin = min(umin, f32(f32(m - r) * p["ia"]))
    if not umax >= umin:
        return 0
    lo = min(max(f32(f32(f32(f32(p["px"] - f32(7.0)) - umax) - f32(0.05)) * f32(0.125)), f32(-1.0)), f32(32767.0))
    hi = min(max(f32(f32(f32(p["px"] - umin) + f32(0.05)) * f32(0.125)), f32(-1.0)), f32(32767.0))
    c0 = max(0, int(np.ceil(lo)))
    c1 = max(c0, min(int(np.floor(hi)) + 1, 0x7fff))
    return c0 | c1 << 16


def quads_of_tile(up, dn, tx):
    c = 2 * tx
    inside = lambda r, x: (r & 0xffff) <= x < (r >> 16)  # noqa: E731
    return int(inside(up, c)) | int(inside(up, c + 1)) << 1 | int(inside(dn, c)) << 2 | int(inside(dn, c + 1)) << 3


def fma(x, y, z):
    """fmaf for float32 operands: the product is exact in float64, one rounding of the sum (to f32 via f64)."""
    return f32(np.float64(x) * np.float64(y) + np.float64(z))


def quad_form(a, b, c, u, v):
    """csrc/gsr_kernels.h quad_form: fmaf(a u, u, fmaf(2 b u, v, c v v))."""
    return fma(f32(a * u), u, fma(f32(f32(f32(2.0) * b) * u), v, f32(f32(c * v) * v)))


def quadrant_hit(px, py, a, b, c, o, qx, qy):
    if not (o >= f32(ALPHA_MIN * f32(0.9999))):
        return False
    if not (a > 0 and c > 0 and f32(a * c) - f32(b * b) > 0):
        return True
    tau = max(f32(0.0), f32(np.log(f32(f32(255.0) * o))))
    thr = f32(2.0) * f32(f32(tau * f32(1.002)) + f32(2e-3))
    u1 = f32(px - qx)
    u0 = f32(u1 - f32(7.0))
    v1 = f32(py - qy)
    v0 = f32(v1 - f32(7.0))
    if u0 <= 0 <= u1 and v0 <= 0 <= v1:
        return True
    ia, ic = f32(1.0) / a, f32(1.0) / c
    cl = lambda x, lo, hi: min(max(x, lo), hi)  # noqa: E731
    q = min(quad_form(a, b, c, u0, cl(f32(f32(-b * u0) * ic), v0, v1)),
            quad_form(a, b, c, u1, cl(f32(f32(-b * u1) * ic), v0, v1)),
            quad_form(a, b, c, cl(f32(f32(-b * v0) * ia), u0, u1), v0),
            quad_form(a, b, c, cl(f32(f32(-b * v1) * ia), u0, u1), v1))
    return f32(q * f32(0.998)) <= thr


def blends(px, py, a, b, c, o, x, y):
    """The blends' condition at pixel (x, y) (csrc/gsr_common.h gauss_power, fp32)."""
    dx, dy = f32(px - f32(x)), f32(py - f32(y))
    q = f32(f32(f32(c * dy) * dy) + f32(f32(a * dx) * dx))
    power = f32(f32(f32(-0.5) * q) - f32(f32(b * dx) * dy))
    alpha = min(f32(0.99), f32(o * f32(np.exp(power))))
    return power <= 0 and alpha >= ALPHA_MIN


def conic(sx, sy, theta):
    """The 2D conic (inverse covariance) of a rotated ellipse with the EWA low-pass (+0.3) of the preprocess."""
    R = np.array([[np.cos(theta), -np.sin(theta)], [np.sin(theta), np.cos(theta)]])
    cov = R @ np.diag([sx * sx, sy * sy]) @ R.T + 0.3 * np.eye(2)
    inv = np.linalg.inv(cov)
    return f32(inv[0, 0]), f32(inv[0, 1]), f32(inv[1, 1])


def cases():
    rng = np.random.default_rng(12)
    out = []
    for kind in ("round", "rotated", "needle", "faint", "large", "edge"):
        for _ in range(40):
            px, py = f32(rng.uniform(8, 56)), f32(rng.uniform(8, 56))
            if kind == "edge":  # centres on / next to quadrant and tile boundaries
                px = f32(rng.integers(1, 7) * 8 + rng.choice([-0.5, -0.01, 0.0, 0.01, 0.5]))
                py = f32(rng.integers(1, 7) * 8 + rng.choice([-0.5, -0.01, 0.0, 0.01, 0.5]))
            sx, sy, th, o = rng.uniform(0.5, 4), rng.uniform(0.5, 4), rng.uniform(0, np.pi), rng.uniform(0.05, 0.95)
            if kind == "round":
                sy, th = sx, 0.0
            elif kind == "needle":
                sx, sy = rng.uniform(6, 20), rng.uniform(0.05, 0.3)
            elif kind == "faint":
                o = rng.uniform(1.0 / 255.0, 1.5 / 255.0)
            elif kind == "large":
                sx, sy, o = rng.uniform(6, 15), rng.uniform(6, 15), rng.uniform(0.9, 0.99)
            a, b, c = conic(sx, sy, th)
            out.append((kind, px, py, a, b, c, f32(o)))
    return out


@pytest.mark.parametrize("kind", ["round", "rotated", "needle", "faint", "large", "edge"])
def test_quadrant_bounds_keep_every_blending_quadrant(kind):
    grid = 4  # 4 x 4 tiles of 16 x 16 pixels around the Gaussians (64 x 64 pixels)
    ys, xs = np.mgrid[0:16 * grid, 0:16 * grid]
    differ = kept_band = kept_hit = exact = 0
    for k, px, py, a, b, c, o in cases():
        if k != kind:
            continue
        sp = span_prep(px, py, a, b, c, o)
        for ty in range(grid):
            v1 = f32(py - f32(ty * 16))
            up, dn = span_quads(sp, v1), span_quads(sp, f32(v1 - f32(8.0)))
            for tx in range(grid):
                band = quads_of_tile(up, dn, tx)
                for q in range(4):
                    qx, qy = tx * 16 + (q & 1) * 8, ty * 16 + (q >> 1) * 8
                    pix = [(x, y) for y in range(qy, qy + 8) for x in range(qx, qx + 8)]
                    any_blend = any(blends(px, py, a, b, c, o, x, y) for x, y in pix)
                    hit = quadrant_hit(px, py, a, b, c, o, f32(qx), f32(qy))
                    inb = bool((band >> q) & 1)
                    if any_blend:
                        exact += 1
                        assert inb, (kind, px, py, a, b, c, o, tx, ty, q, "span_quads drops a blending quadrant")
                        assert hit, (kind, px, py, a, b, c, o, tx, ty, q, "quadrant_hit drops a blending quadrant")
                    kept_band += inb
                    kept_hit += hit
                    differ += inb != hit
    del ys, xs
    assert exact > 0
    print(f"{kind}: blending quadrants {exact}, kept by span_quads {kept_band}, by quadrant_hit {kept_hit}, "
          f"kept by one only {differ}")
