"""Test infrastructure: FMLoss::CalcGrad (fm_loss.h:148-203) with every sum in float64 over
the reference's own float32 terms.

The reference sums a key's gradient sequentially in float (spmv.h:139-171, spmm.h:127-159).
A hot key (C5, Zipf(1.1): tens of thousands of occurrences per batch) cannot be summed that way
on a GPU in bounded time, so the device sums its chunks in double and rounds once.  Both the
device and the reference are then compared with these float64 sums, with the error measured
against the condition scale of each sum (sum of |terms|): the reference's own float rounding
is the only difference that remains between the two."""
import numpy as np


def exact_calcgrad(blk, col, W, wp, vp, d, pred, U):
    """-> (grad f64 in the layout of W, scale f64: sum of |terms| of each element)"""
    offs = blk.offs.astype(np.int64)
    B = blk.size
    nnz = blk.nnz
    col = np.asarray(col, np.int64)
    x = np.ones(nnz, np.float32) if blk.vals is None else blk.vals
    y = np.where(blk.labels > 0, 1.0, -1.0)
    # p = -y / (1 + exp(y pred)), the exponential rounded once (as the device computes it)
    p = (-y / (1.0 + np.exp(y * pred.astype(np.float64)))).astype(np.float32)
    row = np.repeat(np.arange(B), np.diff(offs))
    px = (p[row] * x).astype(np.float32)
    pxx = (p[row] * (x * x).astype(np.float32)).astype(np.float32)
    nz = p[row] != 0
    gw = np.zeros(U)
    np.add.at(gw, col[nz], px[nz].astype(np.float64))
    xxp = np.zeros(U)
    np.add.at(xxp, col[nz], pxx[nz].astype(np.float64))
    absw = np.zeros(U)
    np.add.at(absw, col[nz], np.abs(px[nz]).astype(np.float64))
    out = np.zeros(len(W))
    scale = np.zeros(len(W))
    wp = np.arange(U) if wp is None else np.asarray(wp)
    has_w = wp >= 0
    out[wp[has_w]] = gw[has_w]
    scale[wp[has_w]] = absw[has_w]
    if d > 0:
        # X*V per row in float32, in the reference's (row, nnz) order (fm_loss.h:95-106)
        XV = np.zeros((B, d), np.float32)
        maxlen = int(np.max(np.diff(offs))) if B else 0
        for j in range(maxlen):
            rows = np.nonzero(offs[:-1] + j < offs[1:])[0]
            q = offs[rows] + j
            v = vp[col[q]]
            ok = v >= 0
            r2, q2, v2 = rows[ok], q[ok], v[ok]
            Vv = W[v2[:, None] + np.arange(d)]
            XV[r2] = (XV[r2] + (Vv * x[q2][:, None]).astype(np.float32)).astype(np.float32)
        XVp = (XV * p[:, None]).astype(np.float32)
        T = (XVp[row] * x[:, None]).astype(np.float32)
        S = np.zeros((U, d))
        np.add.at(S, col, T.astype(np.float64))
        SA = np.zeros((U, d))
        np.add.at(SA, col, np.abs(T).astype(np.float64))
        hv = vp >= 0
        Vk = W[vp[hv][:, None] + np.arange(d)].astype(np.float64)
        idx = vp[hv][:, None] + np.arange(d)
        out[idx] = -Vk * xxp[hv][:, None] + S[hv]
        scale[idx] = np.abs(Vk * xxp[hv][:, None]) + SA[hv]
    return out, scale
