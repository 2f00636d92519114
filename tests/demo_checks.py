"""Where a DeMo sign is unambiguous (test infrastructure).

The decode applies p -= lr * sign(g_hat).  Two correct fp32 implementations
(the reference's torch einsum, our MFMA kernels) can disagree on a sign only
where g_hat is ~0 relative to the tensor, or where a node's top-k set was
decided by a near-tie (then the transmitted coefficients differ).  Everywhere
else -- the FIRM elements -- signs must agree exactly, and each disagreement
would be an element off by 2*lr, so the tests assert exact equality there and
that the firm set covers nearly every element (so the check is not vacuous).
"""
import numpy as np

from oracle import demo as odemo


def chunk_mask_to_elements(ok_chunks, shape, chunk):
    """Per-chunk bools [gy*gx] (or [gy, gx]) -> per-element bools of `shape`."""
    R, C, n1, n2 = odemo.tensor_view(shape, chunk)
    okc = np.asarray(ok_chunks).reshape(R // n1, C // n2)
    return np.repeat(np.repeat(okc, n1, axis=0), n2, axis=1).reshape(shape)


def firm(g_hat, margins, shape, chunk=64, rel=1e-5, margin_rel=1e-5):
    """Elements whose sign is decided: |g_hat| > rel * max|g_hat| and every
    node's top-k set in that chunk is unambiguous (k-th margin > margin_rel
    times the node's largest coefficient; margins as oracle.demo.demo_step(...,
    detail=True) returns them, with the coefficient scale alongside)."""
    g = np.abs(np.asarray(g_hat, dtype=np.float64))
    out = g > rel * max(g.max(), 1e-30)
    for m, scale in margins:
        out &= chunk_mask_to_elements(np.asarray(m) > margin_rel * scale, shape, chunk)
    return out


def chunk_max_abs(x, shape, chunk=64):
    """Per element: max |x| over the element's DeMo chunk (the chunk's scale)."""
    R, C, n1, n2 = odemo.tensor_view(shape, chunk)
    a = np.abs(np.asarray(x, np.float64)).reshape(R // n1, n1, C // n2, n2)
    m = a.max(axis=(1, 3))
    return np.repeat(np.repeat(m, n1, axis=0), n2, axis=1).reshape(shape)


def residual_close(got_d, ref_d, x, margin, shape, chunk=64, rel=1e-6, loose=2e-5, what=""):
    """The residual delta (demo.py:174-180) where the node's top-k set is firm
    (k-th margin > 1e-5 of its largest coefficient): within rel x the chunk's
    scale (max |x| of the encoded input x = decay*delta + lr*grad).  In chunks
    decided by a near-tie the two implementations may keep different
    coefficients: there only the tensor-scale bar `loose` applies."""
    m, scale = margin
    firm_el = chunk_mask_to_elements(np.asarray(m) > 1e-5 * scale, shape, chunk)
    err = np.abs(np.asarray(got_d, np.float64) - np.asarray(ref_d, np.float64))
    lim = rel * chunk_max_abs(x, shape, chunk)
    bad = np.flatnonzero((err > lim) & firm_el)
    assert bad.size == 0, (f"{what}: residual delta off by > {rel} x chunk scale at {bad.size} firm elements, "
                           f"worst {float((err / np.maximum(lim / rel, 1e-30))[firm_el].max()):.3g}")
    if (~firm_el).any():
        assert err[~firm_el].max() <= loose * np.abs(np.asarray(x)).max(), what
    return float(firm_el.mean())


def node_margins(deltas, grads, shape, lr, decay, topk=32, chunk=64):
    """(per-chunk k-th margin, coefficient scale) of each node's encoded delta."""
    out = []
    for d, g in zip(deltas, grads):
        x = np.asarray(d, np.float64) * decay + lr * np.asarray(g, np.float64)
        Y = odemo.encode(x, shape, chunk)
        out.append((odemo.kth_margin(Y, topk), np.abs(Y).max()))
    return out


class SignTally:
    """Exact sign equality on the firm elements of each tensor, and (at the
    end) a floor on the firm fraction over all tensors checked."""

    def __init__(self):
        self.firm = 0
        self.total = 0

    def check(self, got_sign, want_sign, firm_mask, what=""):
        got_sign, want_sign = np.asarray(got_sign), np.asarray(want_sign)
        assert np.isin(got_sign, (-1.0, 0.0, 1.0)).all(), what
        bad = np.flatnonzero((got_sign != want_sign) & firm_mask)
        assert bad.size == 0, f"{what}: {bad.size} firm sign mismatches (of {firm_mask.sum()}), first at {bad[:5]}"
        self.firm += int(firm_mask.sum())
        self.total += firm_mask.size

    def done(self, min_firm=0.98):
        frac = self.firm / max(self.total, 1)
        assert frac >= min_firm, f"only {frac:.4f} of the elements are firm (floor {min_firm})"
        return frac


def bf16_round(x):
    """fp32 -> nearest-even bf16, returned widened to fp32 (what a bf16 store keeps)."""
    u = np.ascontiguousarray(np.asarray(x, np.float32)).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32).view(np.float32)


def bf16_ulp(x):
    """Spacing of bf16 values at |x| (8 significand bits)."""
    a = np.maximum(np.abs(np.asarray(x, np.float64)), 2.0 ** -126)
    return 2.0 ** (np.floor(np.log2(a)) - 7)


class Bf16Agreement:
    """Statistical parity with the reference's bf16 DeMo (tests/golden/demo_steps_bf16.npz).

    The reference computes the DCT in bf16 and resolves the k-th-largest ties
    that bf16 coefficients produce in a large share of chunks in the order of
    torch's CPU selection algorithm, so two correct implementations disagree on
    the top-k set of those chunks and on the signs they feed.  Bars, calibrated on
    the fp64 oracle (an exact-rounding numpy restatement of the reference's bf16
    arithmetic measured 0.939-1.000 per tensor):
    - signs in {-1, 0, 1}; agreement >= min_tensor per tensor and >= min_all overall;
    - where the signs agree, p equals the reference's p within one bf16 ulp of
      the larger of p before and after, plus |bf16(lr) - lr| (torch's CPU add_
      casts alpha to the tensor's dtype: lr 0.01 steps by 0.010009765625 there,
      which shows where p - lr cancels);
    - the residual delta: median |error| <= delta_rel * max|reference delta|.
    """

    def __init__(self, min_tensor=0.93, min_all=0.96, delta_rel=1e-2):
        self.min_tensor, self.min_all, self.delta_rel = min_tensor, min_all, delta_rel
        self.agree = 0
        self.total = 0
        self.worst = 1.0

    def check(self, sign, p_after, deltas, z, step, i):
        what = f"step {step} tensor {i}"
        sign = np.asarray(sign, np.float32)
        assert np.isin(sign, (-1.0, 0.0, 1.0)).all(), what
        ref_s = z[f"sign_{step}_{i}"]
        ok = sign == ref_s
        frac = ok.mean()
        self.worst = min(self.worst, frac)
        assert frac >= self.min_tensor, f"{what}: sign agreement {frac:.4f} < {self.min_tensor}"
        ref_p, p0, lr = z[f"p_after_{step}_{i}"], z[f"p_before_{step}_{i}"], float(z["lr"])
        err = np.abs(np.asarray(p_after, np.float64) - ref_p)
        alpha_err = abs(float(bf16_round(np.float32([lr]))[0]) - lr)
        lim = bf16_ulp(np.maximum(np.abs(ref_p), np.abs(p0))) * 1.0001 + alpha_err
        bad = np.flatnonzero((err > lim) & ok)
        assert bad.size == 0, f"{what}: p differs by > 1 bf16 ulp at {bad.size} agreeing elements, first {bad[:5]}"
        for k, d in enumerate(deltas):
            ref_d = z[f"delta_after_{step}_{i}"][k]
            med = np.median(np.abs(np.asarray(d, np.float64) - ref_d))
            assert med <= self.delta_rel * np.abs(ref_d).max(), f"{what} node {k}: delta median error {med:.3g}"
        self.agree += int(ok.sum())
        self.total += ok.size

    def done(self):
        frac = self.agree / max(self.total, 1)
        assert frac >= self.min_all, f"overall bf16 sign agreement {frac:.4f} < {self.min_all}"
        return frac, self.worst
