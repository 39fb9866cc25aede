"""tanh_fast (csrc/hf_device.h), the PureGNN / PINN one-launch rollouts' tanh:
its f32 arithmetic restated in numpy float32 from the coefficients in the
header, checked against float64 tanh (no GPU needed).  The hardware v_exp_f32
and v_rcp_f32 are modelled as correctly rounded, then perturbed by one ulp
(their documented accuracy), so the bounds cover both: <= 1 ulp below
|x| = 0.55, above it <= 2 ulp with exp and rcp correctly rounded and <= 4
ulp with both one ulp off in the worst directions (near |x| = 0.55, where
1 - 2r loses a bit)."""
import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(__file__), "..", "gnn-plasma-flux_amd", "csrc", "hf_device.h")


def _coeffs():
    with open(HDR) as f:
        src = f.read()
    body = src[src.index("float tanh_fast(float x)"):]
    body = body[:body.index("\n}\n")]
    num = r"(-?\d+\.\d+)f"
    scale = np.float32(re.search(r"ax \* " + num, body).group(1))
    poly = [np.float32(v) for v in re.findall(r"p = (?:__builtin_fmaf\(p, x2, )?" + num, body)]
    thr = np.float32(re.search(r"ax < " + num, body).group(1))
    assert len(poly) == 5, poly
    return scale, poly, thr


def _tanh_fast(x, exp_ulp=0, rcp_ulp=0):
    with np.errstate(all="ignore"):  # inf / NaN inputs: both branches are evaluated, as on the GPU
        return _tanh_fast_eval(x, exp_ulp, rcp_ulp)


def _tanh_fast_eval(x, exp_ulp, rcp_ulp):
    scale, (p0, p1, p2, p3, p4), thr = _coeffs()
    x = x.astype(np.float32)
    ax = np.abs(x)
    arg = (ax * scale).astype(np.float32)
    e = np.exp2(arg.astype(np.float64)).astype(np.float32)  # -> inf for large |x|, as on the GPU
    e = (e.astype(np.float64) * (1 + exp_ulp * 2.0 ** -23)).astype(np.float32)
    d = (np.float32(1) + e).astype(np.float32)
    r = (1.0 / d.astype(np.float64)).astype(np.float32)
    r = (r.astype(np.float64) * (1 + rcp_ulp * 2.0 ** -23)).astype(np.float32)
    big = (np.float64(-2.0) * r.astype(np.float64) + 1.0).astype(np.float32)  # fma(-2, r, 1): one rounding
    x2 = (x * x).astype(np.float32)
    p = np.full_like(x2, p0)
    for k in (p1, p2, p3, p4):                                          # fma: one rounding each
        p = (p.astype(np.float64) * x2.astype(np.float64) + np.float64(k)).astype(np.float32)
    small = ((x * x2).astype(np.float32).astype(np.float64) * p.astype(np.float64) + x.astype(np.float64)).astype(np.float32)
    return np.where(ax < thr, small, np.copysign(big, x)), thr


def test_tanh_fast_accuracy():
    x = np.concatenate([np.linspace(-12, 12, 400001), np.linspace(-0.6, 0.6, 200001),
                        np.float32([0.0, -0.0, 1e-30, -1e-6, 0.55, -0.55])]).astype(np.float32)
    ref = np.tanh(x.astype(np.float64))
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    for eu in (-1, 0, 1):
        for ru in (-1, 0, 1):
            y, thr = _tanh_fast(x, eu, ru)
            err = np.abs(y.astype(np.float64) - ref) / np.maximum(ulp, np.spacing(np.float32(1e-38)))
            assert thr == np.float32(0.55)
            assert err[np.abs(x) < thr].max() <= 1.0          # the polynomial branch
            assert err[np.abs(x) >= thr].max() <= (2.0 if eu == ru == 0 else 4.0)  # the exp / rcp branch
    y, _ = _tanh_fast(np.float32([np.nan, np.inf, -np.inf, 40.0, -40.0]))
    assert np.isnan(y[0]) and y[1] == 1 and y[2] == -1 and y[3] == 1 and y[4] == -1


def test_tanh_fast2_same_arithmetic():
    """tanh_fast2 (the packed pair) carries tanh_fast's constants in the same
    order and the same threshold, so the two are the same f32 arithmetic (the
    GPU A/B in profiles/r05_puregnn_tanh2_ab.txt found the rollouts bitwise
    equal)."""
    with open(HDR) as f:
        src = f.read()
    num = r"(-?\d+\.\d+)f"

    def body(sig):
        b = src[src.index(sig):]
        return b[:b.index("\n}\n")]

    one, two = body("float tanh_fast(float x)"), body("hf_f2 tanh_fast2(hf_f2 x)")
    poly1 = re.findall(r"p = (?:__builtin_fmaf\(p, x2, )?" + num, one)
    poly2 = re.findall(r"p = (?:__builtin_elementwise_fma\(p, x2, )?hf_f2\(" + num, two)
    assert len(poly1) == 5 and poly2 == poly1
    assert re.findall(r"ax \* " + num, one) == re.findall(r"ax \* " + num, two)
    assert re.findall(r"ax < " + num, one) * 2 == re.findall(r"ax\.[xy] < " + num, two)
    assert set(re.findall(num, one)) == set(re.findall(num, two))
