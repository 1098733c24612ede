"""Round-5 GPU tests: the kernels added this round against the oracle and the kernels they
replace.

* k_fm_fwd_walk (the fat-slot forward at V_dim 8 / 16): each row's slots read kWkNB per trip
  from ids staged in LDS, summed in the reference's (row, nnz) order (fm_loss.h:67-119), so
  predictions must be BIT-identical to the oracle's and to the probe walk's (fat_fwd=0: the
  entry, then V, per nnz), and the trained model the same.  Ragged rows cover the staging
  edges: empty rows, rows longer than a staged chunk (40 ids), a row of 1300 nnz, and rows
  the resident grid's groups reach on their second and third pass (80 k rows).
"""
import numpy as np
import pytest
import torch

from difacto_amd import data as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    from difacto_amd import hotpath
    return hotpath


def _auc_expect(label, opred, oauc):
    return O.auc_stable_ties(label, opred) if O.has_ties(opred) else oauc


def _long_rows(blk, lens, binary, seed):
    """blk with rows of the given lengths appended (ids spread over the key space)"""
    rng = np.random.default_rng(seed)
    ids, offs, vals, labels = [blk.ids], [blk.offs], [blk.vals], [blk.labels]
    end = int(blk.offs[-1])
    for n in lens:
        ids.append(rng.integers(0, 1 << 40, n, dtype=np.uint64))
        end += n
        offs.append(np.array([end], np.uint64))
        if not binary:
            vals.append((1.0 - rng.random(n, dtype=np.float32)).astype(np.float32))
        labels.append(np.array([1.0 if n % 2 else -1.0], np.float32))
    return D.RowBlock(np.concatenate(offs).astype(np.uint64), np.concatenate(ids),
                      None if binary else np.concatenate(vals), np.concatenate(labels))


@pytest.mark.parametrize("rows,d", [(3001, 16), (80001, 16), (3001, 8)])
@pytest.mark.parametrize("binary", [True, False])
def test_walk_forward_bit_identical(H, rows, d, binary):
    cfg = dict(V_dim=d, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    ks, mk = (1 << 15, 1 << 16) if rows < 10000 else (1 << 20, 1 << 21)
    ca = H.Context(0, max_keys=mk, fat_fwd=0, **cfg)  # the probe walk: entry, then V
    cb = H.Context(0, max_keys=mk, **cfg)             # the fat walk (k_fm_fwd_walk)
    up = O.Updater(**cfg)
    for step in range(4):
        blk = D.synthetic(rows, 39, ks, binary=binary, ragged=True, seed=60 + step)
        if step >= 2:  # rows longer than a chunk, one exactly a chunk, one crossing two
            blk = _long_rows(blk, [700, 512, 1300, 0, 3], binary, seed=step)
        pa = torch.zeros(blk.size, dtype=torch.float32, device=ca.device)
        pb = torch.zeros(blk.size, dtype=torch.float32, device=cb.device)
        H.train_step(ca, H.DeviceRowBlock(ca, blk), H.kTraining, push_cnt=(step < 1), pred=pa)
        H.train_step(cb, H.DeviceRowBlock(cb, blk), H.kTraining, push_cnt=(step < 1), pred=pb)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 1), want_pred=True)
        qa, qb = H.progress(ca), H.progress(cb)
        got = pb.cpu().numpy()
        assert np.array_equal(pa.cpu().numpy().view(np.uint32), got.view(np.uint32)), step
        # no key reaches a chunked (> 256 occurrences) gradient sum: the model stays the
        # oracle's, so predictions equal the reference's bit for bit
        assert np.array_equal(got.view(np.uint32), np.asarray(opred, np.float32).view(np.uint32))
        # per-block loss partials: the double sums differ in the last bits only
        assert abs(qa["loss"] - qb["loss"]) <= 1e-12 * abs(qa["loss"]) and qa["auc"] == qb["auc"]
        assert abs(qb["loss"] - loss) <= 1e-4 * abs(loss)
        assert abs(qb["auc"] - _auc_expect(blk.labels, opred, auc)) <= 1e-4 * blk.size
    uniq, _, _ = O.localize(blk.offs, blk.ids)
    va, la = H.Store(ca).pull(ca.tensor(uniq, torch.int64))
    vb, lb = H.Store(cb).pull(cb.tensor(uniq, torch.int64))
    assert np.array_equal(la.cpu().numpy(), lb.cpu().numpy())
    assert np.array_equal(va.cpu().numpy().view(np.uint32), vb.cpu().numpy().view(np.uint32))
    ca.close()
    cb.close()


@pytest.mark.parametrize("d,binary", [(128, True), (16, False), (0, True)])
def test_tile_chunks_hot_keys(H, d, binary):
    """The hottest keys of a skewed batch (more than kTileMinOcc = 128 occurrences per row tile
    of kTileRows = 1024 rows) sum per row tile (fm.hip k_fm_bwd_tchunks, tiles walked XCD by
    XCD), the other long keys per 256 occurrences; partials in double, combined in order.  30 k
    Zipf(1.1) rows give 30 tiles: the top keys (thousands of occurrences) are tile-chunked, keys
    of 300..3840 occurrences are occurrence-chunked.  Valued rows take the deferred gather's
    position -> row indirection in the tile starts (occ_rx).  Bounds as test_c5_model_drift_
    bound: the device's model no farther from the exact (f64-sum) trajectory than the reference
    is (plus 1e-8), device vs reference within DRIFT, loss / AUC within 1e-4, lens exact."""
    DRIFT = 1e-5
    cfg = dict(V_dim=d, lr=.05, V_lr=.01)
    c = H.Context(0, max_keys=1 << 19, **cfg)
    up, ex = O.Updater(**cfg), O.Updater(**cfg, sum64=1)
    nrel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    rows = []
    for step in range(4):
        blk = D.synthetic(30000, 39, 1 << 20, zipf=1.1, binary=binary, seed=500 + step)
        if step == 0:
            cnt = np.bincount(O.localize(blk.offs, blk.ids)[2])
            assert cnt.max() > 128 * 30 and (cnt > 256).sum() > (cnt > 128 * 30).sum() > 3
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 2), want_pred=True)
        ex.train_step(blk.offs, blk.ids, blk.vals, blk.labels, push_cnt=(step < 2))
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 2))
        p = H.progress(c)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), step
        assert abs(p["auc"] - _auc_expect(blk.labels, opred, auc)) <= 1e-4 * blk.size, step
        uniq, _, _ = O.localize(blk.offs, blk.ids)
        v, l = H.Store(c).pull(c.tensor(uniq, torch.int64))
        ov, ol = up.get(uniq)
        xv, _ = ex.get(uniq)
        assert np.array_equal(l.cpu().numpy(), ol), step
        a, b, x = (t.astype(np.float64) for t in (v.cpu().numpy(), ov, xv))
        rows.append((nrel(a, b), nrel(a, x), nrel(b, x)))
    print("tile chunks d=%d: per-step drift (device-ref, device-exact, ref-exact):" % d,
          ["%.2e/%.2e/%.2e" % r for r in rows])
    assert max(r[0] for r in rows) <= DRIFT, rows
    assert all(r[1] <= r[2] + 1e-8 for r in rows), rows
    c.close()


@pytest.mark.parametrize("binary", [True, False])
def test_split_one_owner_tile_chunks_equal_fused(H, binary):
    """The split owner plans and sums tile chunks as the fused step does (its rows are the
    concatenated workers' rows, tiled the same way): at N = 1 on Zipf(1.1) batches of 6 k rows
    (6 tiles; the top keys tile-chunked) predictions, AUC and the model equal the fused step's
    exactly, the loss to its double sum's order."""
    from difacto_amd import dist as DI
    kw = dict(V_dim=16, V_threshold=2, lr=.05, V_lr=.02)
    cs = H.Context(0, max_keys=1 << 18, **kw)
    cf = H.Context(0, max_keys=1 << 18, **kw)
    sh = [DI.Shard(cs, 1)]
    comm = DI.LoopbackComm(1)
    blocks = []
    for s in range(4):
        blk = D.synthetic(6000, 39, 1 << 18, zipf=1.1, binary=binary, seed=620 + s)
        blocks.append(blk)
        ds, df = H.DeviceRowBlock(cs, blk), H.DeviceRowBlock(cf, blk)
        ps = torch.zeros(blk.size, dtype=torch.float32, device=cs.device)
        pf = torch.zeros(blk.size, dtype=torch.float32, device=cf.device)
        DI.split_step(sh, [ds], comm, H.kTraining, push_cnt=s < 2, preds=[ps])
        H.train_step(cf, df, H.kTraining, push_cnt=s < 2, pred=pf)
        assert np.array_equal(ps.cpu().numpy(), pf.cpu().numpy()), s
        a, b = H.progress(cs), H.progress(cf)
        assert a["loss"] == pytest.approx(b["loss"], rel=1e-12) and a["auc"] == b["auc"], s
    cs.sync()
    cf.sync()
    assert H.Store(cs).stats() == H.Store(cf).stats()
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0] for b in blocks]))
    cnt = np.bincount(O.localize(blocks[-1].offs, blocks[-1].ids)[2])
    hot = O.localize(blocks[-1].offs, blocks[-1].ids)[0][np.argsort(-cnt)[:40]]
    for k in np.concatenate([hot, keys[::11]]):
        ea, eb = H.Store(cs).entry(k), H.Store(cf).entry(k)
        assert (ea is None) == (eb is None)
        if ea is None:
            continue
        assert np.array_equal(ea[0], eb[0]), k
        assert (ea[1] is None) == (eb[1] is None)
        if ea[1] is not None:
            assert np.array_equal(ea[1], eb[1]), k
    cs.close()
    cf.close()
