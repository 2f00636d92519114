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
