"""The culling rule of gs_common.h (rect_min_within / quadrant_mask), restated in numpy and checked
against the four-edge rule it replaced and a sampled minimum: the minimum of a positive-definite quadratic q over a rectangle that
does not hold its centre lies on an edge facing the centre, so evaluating one edge per axis (the
facing one, or any when the centre lies within that axis's range) finds it.  CPU only: the kernels'
own culling is covered by the GPU parity suite (culling only skips work, results are unchanged)."""
import numpy as np

import pytest


def _q(cx, cy, cz, dx, dy):
    return cx * dx * dx + 2.0 * cy * dx * dy + cz * dy * dy


def _rule_min(cx, cy, cz, dxl, dxh, dyl, dyh):
    """gs_common.h: the centre-inside case, else one edge per axis with the 1-D minimiser clamped."""
    if dxl <= 0.0 <= dxh and dyl <= 0.0 <= dyh:
        return 0.0
    dxe = dxl if dxl > 0.0 else dxh
    dye = dyl if dyl > 0.0 else dyh
    a = _q(cx, cy, cz, dxe, np.clip(-cy / cz * dxe, dyl, dyh))
    b = _q(cx, cy, cz, np.clip(-cy / cx * dye, dxl, dxh), dye)
    return min(a, b)


def _four_edge_min(cx, cy, cz, dxl, dxh, dyl, dyh):
    """The round-4 rule (every edge, each with its clamped 1-D minimiser): the exact minimum."""
    if dxl <= 0.0 <= dxh and dyl <= 0.0 <= dyh:
        return 0.0
    return min(_q(cx, cy, cz, dxl, np.clip(-cy / cz * dxl, dyl, dyh)), _q(cx, cy, cz, dxh, np.clip(-cy / cz * dxh, dyl, dyh)),
               _q(cx, cy, cz, np.clip(-cy / cx * dyl, dxl, dxh), dyl), _q(cx, cy, cz, np.clip(-cy / cx * dyh, dxl, dxh), dyh))


def _brute_min(cx, cy, cz, dxl, dxh, dyl, dyh, n=401):
    xs = np.linspace(dxl, dxh, n)
    ys = np.linspace(dyl, dyh, n)
    X, Y = np.meshgrid(xs, ys)
    # the rectangle's boundary exactly (the minimum of a convex function off its centre is there)
    edges = [
        _q(cx, cy, cz, np.full(n, dxl), ys), _q(cx, cy, cz, np.full(n, dxh), ys),
        _q(cx, cy, cz, xs, np.full(n, dyl)), _q(cx, cy, cz, xs, np.full(n, dyh)),
    ]
    return min(float(_q(cx, cy, cz, X, Y).min()), min(float(e.min()) for e in edges))


@pytest.mark.parametrize("seed", range(4))
def test_facing_edge_rule_finds_the_rectangle_minimum(seed):
    rng = np.random.default_rng(seed)
    for _ in range(400):
        # a random positive-definite conic (anisotropic, rotated) and a random 8x8-pixel rectangle
        s1, s2 = np.exp(rng.uniform(-4.0, 2.0, 2))
        th = rng.uniform(0.0, np.pi)
        c, s = np.cos(th), np.sin(th)
        R = np.array([[c, -s], [s, c]])
        Q = R @ np.diag([1.0 / s1 ** 2, 1.0 / s2 ** 2]) @ R.T
        cx, cy, cz = Q[0, 0], Q[0, 1], Q[1, 1]
        x0, y0 = rng.uniform(-30.0, 30.0, 2)
        dxl, dyl = x0, y0
        dxh, dyh = x0 + 7.0, y0 + 7.0
        rule = _rule_min(cx, cy, cz, dxl, dxh, dyl, dyh)
        exact = _four_edge_min(cx, cy, cz, dxl, dxh, dyl, dyh)
        brute = _brute_min(cx, cy, cz, dxl, dxh, dyl, dyh, n=101)
        # two facing edges give the four-edge minimum (same value, the same expressions), and
        # no sampled rectangle point lies below it
        assert rule == exact, (rule, exact)
        assert rule <= brute * (1.0 + 1e-12) + 1e-12, (rule, brute)


def test_non_facing_edges_cannot_undercut():
    """Where the centre lies within an axis's range, the rule evaluates an arbitrary edge of that
    axis: any point of the rectangle is >= the minimum, so the result is still the minimum (the
    other axis's facing edge attains it)."""
    cx, cy, cz = 0.05, 0.01, 0.08
    # centre inside the x range, below the rectangle in y
    r = _rule_min(cx, cy, cz, -3.0, 4.0, 2.0, 9.0)
    assert r <= _brute_min(cx, cy, cz, -3.0, 4.0, 2.0, 9.0) <= r * (1.0 + 1e-4)
