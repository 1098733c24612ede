"""Parity at the BASELINE configs' own sizes (C2, C3, C5), through the C-ABI.

The other GPU parity tests run small batches; these run the batch shapes the benchmark and
the survey quote: C3 at the bench's B = 100,000 rows x 39 binary nnz over 2^24 keys (3.9 M
nnz), C2 at B = 10^4 x 40 valued nnz over 2^20 keys with FTRL L1 and no V, C5 at B = 10^4
Zipf(1.1) rows at V_dim = 128 with lazy V.  The checker is the oracle (the C restatement of
the reference, oracle/oracle.cc) on the same inputs, plus size-independent properties of the
Localizer (strictly ascending unique keys, counts summing to nnz, uniq[col] == the nnz's key).
"""
import numpy as np
import pytest
import torch

from difacto_amd import data as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5  # north_star: per-minibatch predictions within 1e-5 relative (fp32)


@pytest.fixture(scope="module")
def H():
    from difacto_amd import hotpath
    return hotpath


def close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    floor = 1e-6 * max(1.0, float(np.max(np.abs(b))) if b.size else 1.0)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(a), np.abs(b)) + floor)


def _rev(a):
    return np.array([O.reverse_bytes(int(x)) for x in a], dtype=np.uint64)


def _auc_expect(label, opred, oauc):
    return O.auc_stable_ties(label, opred) if O.has_ties(opred) else oauc


def test_localizer_full_c3(H):
    """Localizer::Compact of a bench-sized batch: bit-exact against the oracle, and the
    properties that hold at any size"""
    c = H.Context(0, max_keys=1 << 20, V_dim=16)
    blk = D.synthetic(100_000, 39, 1 << 24, seed=4242)
    db = H.DeviceRowBlock(c, blk)
    col, uniq, cnt = H.Localizer(c).compact(db)
    u, n, cl = H.u64(uniq), cnt.cpu().numpy(), H.u32(col)
    ou, oc, ocol = O.localize(blk.offs, blk.ids)
    assert np.array_equal(u, ou)
    assert np.array_equal(n, oc)
    assert np.array_equal(cl, ocol)
    assert np.all(u[1:] > u[:-1])
    assert float(n.astype(np.float64).sum()) == blk.nnz
    # ReverseBytes (base.h:39-51): bytes reversed, then the two nibbles of every byte swapped
    b = np.frombuffer(blk.ids.astype(">u8").tobytes(), dtype="<u8")
    lo, hi = np.uint64(0x0F0F0F0F0F0F0F0F), np.uint64(0xF0F0F0F0F0F0F0F0)
    keys = ((b & lo) << np.uint64(4)) | ((b & hi) >> np.uint64(4))
    assert np.array_equal(keys[:64], _rev(blk.ids[:64]))
    assert np.array_equal(u[cl], keys)
    c.close()


def _run(H, cfg, batches, n_cnt, max_keys, pred_rtol, model_rtol, check_model=True):
    c = H.Context(0, max_keys=max_keys, **cfg)
    up = O.Updater(**cfg)
    for step, blk in enumerate(batches):
        push = step < n_cnt
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=push, want_pred=True)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=push, pred=pred)
        p = H.progress(c)
        assert close(pred.cpu().numpy(), opred, rtol=pred_rtol), step
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), (step, p["loss"], loss)
        assert abs(p["auc"] - _auc_expect(blk.labels, opred, auc)) <= 1e-4 * blk.size, step
        assert p["nrows"] == blk.size
    s = H.Store(c).stats()
    assert s["n_keys"] == up.size() and s["seed"] == up.seed
    if check_model:
        # the model after the last Update, over the last batch's keys (Get: values and lens)
        uniq, _, _ = O.localize(blk.offs, blk.ids)
        v, l = H.Store(c).pull(c.tensor(uniq, torch.int64))
        ov, ol = up.get(uniq)
        if cfg.get("V_dim", 0) > 0:
            assert np.array_equal(l.cpu().numpy(), ol)
        assert close(v.cpu().numpy(), ov, rtol=model_rtol)
    c.close()


def test_fused_full_c3(H):
    """C3 at the bench's shape: an epoch-0 step (count push, every key gets V at
    V_threshold = 0), then training steps over fresh batches"""
    cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    batches = [D.synthetic(100_000, 39, 1 << 24, seed=5000 + s) for s in range(3)]
    _run(H, cfg, batches, n_cnt=1, max_keys=1 << 24, pred_rtol=RTOL, model_rtol=RTOL)


def test_fused_full_c2(H):
    """C2: LR only (V_dim = 0), FTRL with L1, valued rows of 40 nnz over 2^20 keys"""
    cfg = dict(V_dim=0, l1=1, l2=0, lr=.1)
    batches = [D.synthetic(10_000, 40, 1 << 20, binary=False, seed=6000 + s)
               for s in range(6)]
    _run(H, cfg, batches, n_cnt=0, max_keys=1 << 20, pred_rtol=RTOL, model_rtol=RTOL)


def test_fused_full_c5(H):
    """C5: Zipf(1.1) keys over 2^24, V_dim = 128, reference defaults (V_threshold = 10,
    l1 = 1, l1_shrk): V is created lazily for the hot keys.  Hot keys' Xᵀ sums run in
    256-occurrence chunks combined in chunk order (reordered sums), so predictions after the
    first update and the model are compared within tolerance (Determinism)."""
    cfg = dict(V_dim=128, lr=.05, V_lr=.01)
    batches = [D.synthetic(10_000, 39, 1 << 24, zipf=1.1, seed=7000 + s) for s in range(4)]
    _run(H, cfg, batches, n_cnt=2, max_keys=1 << 20, pred_rtol=1e-4, model_rtol=1e-3)
