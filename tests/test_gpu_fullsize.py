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

K_CHUNK_OCC = 128  # csrc/internal.h kChunkOcc: longer segments are summed in chunks

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


def _run(H, cfg, batches, n_cnt, max_keys, pred_rtol, model_rtol, check_model=True,
         exact=False, drift=None):
    """exact: no key reaches a chunked (> kChunkOcc = 128 occurrences, csrc/internal.h) gradient
    sum, so predictions and the model must equal the oracle's bit for bit (sums in the
    reference's order, glibc expf); asserted per batch, so a change of the chunk threshold fails
    here by name rather than as an unexplained bit mismatch.
    drift: after every step the model over the batch's keys is compared as a vector with the
    reference's and with the exact trajectory's (the oracle with every gradient column summed in
    double, sum64): ||device - ref|| / ||ref|| <= drift, and the device no farther from the exact
    trajectory than the reference is (test_gpu_r3.py test_c5_model_drift_bound's form)"""
    c = H.Context(0, max_keys=max_keys, **cfg)
    up = O.Updater(**cfg)
    ex = O.Updater(**cfg, sum64=1) if drift is not None else None
    nrel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
    rows = []
    for step, blk in enumerate(batches):
        if exact:
            _, cnt = np.unique(blk.ids, return_counts=True)
            assert int(cnt.max()) <= K_CHUNK_OCC, (step, int(cnt.max()))
        push = step < n_cnt
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=push, want_pred=True)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=push, pred=pred)
        p = H.progress(c)
        rt = pred_rtol[step] if isinstance(pred_rtol, (list, tuple)) else pred_rtol
        assert close(pred.cpu().numpy(), opred, rtol=rt), step
        if exact:
            assert np.array_equal(pred.cpu().numpy().view(np.uint32),
                                  np.asarray(opred, np.float32).view(np.uint32)), step
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), (step, p["loss"], loss)
        assert abs(p["auc"] - _auc_expect(blk.labels, opred, auc)) <= 1e-4 * blk.size, step
        assert p["nrows"] == blk.size
        if ex is not None:
            ex.train_step(blk.offs, blk.ids, blk.vals, blk.labels, push_cnt=push)
            uniq, _, _ = O.localize(blk.offs, blk.ids)
            v, l = H.Store(c).pull(c.tensor(uniq, torch.int64))
            ov, ol = up.get(uniq)
            xv, xl = ex.get(uniq)
            assert np.array_equal(l.cpu().numpy(), ol) and np.array_equal(xl, ol), step
            a, b, x = (t.astype(np.float64) for t in (v.cpu().numpy(), ov, xv))
            rows.append((nrel(a, b), nrel(a, x), nrel(b, x)))
    if ex is not None:
        print("full-size model drift ||.||/||.|| (device-ref, device-exact, ref-exact):",
              ["%.2e/%.2e/%.2e" % r for r in rows])
        assert max(r[0] for r in rows) <= drift, rows
        assert all(r[1] <= r[2] + 1e-8 for r in rows), rows
    s = H.Store(c).stats()
    assert s["n_keys"] == up.size() and s["seed"] == up.seed
    if check_model:
        # the model after the last Update, over the last batch's keys (Get: values and lens)
        uniq, _, _ = O.localize(blk.offs, blk.ids)
        v, l = H.Store(c).pull(c.tensor(uniq, torch.int64))
        ov, ol = up.get(uniq)
        if cfg.get("V_dim", 0) > 0:
            assert np.array_equal(l.cpu().numpy(), ol)
        if model_rtol is not None:
            assert close(v.cpu().numpy(), ov, rtol=model_rtol)
        if exact:
            assert np.array_equal(v.cpu().numpy().view(np.uint32),
                                  np.asarray(ov, np.float32).view(np.uint32))
    c.close()


def test_fused_full_c3(H):
    """C3 at the bench's shape: an epoch-0 step (count push, every key gets V at
    V_threshold = 0), then training steps over fresh batches"""
    cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    batches = [D.synthetic(100_000, 39, 1 << 24, seed=5000 + s) for s in range(3)]
    _run(H, cfg, batches, n_cnt=1, max_keys=1 << 24, pred_rtol=RTOL, model_rtol=RTOL,
         exact=True)


def test_fused_full_c2(H):
    """C2: LR only (V_dim = 0), FTRL with L1, valued rows of 40 nnz over 2^20 keys"""
    cfg = dict(V_dim=0, l1=1, l2=0, lr=.1)
    batches = [D.synthetic(10_000, 40, 1 << 20, binary=False, seed=6000 + s)
               for s in range(6)]
    _run(H, cfg, batches, n_cnt=0, max_keys=1 << 20, pred_rtol=RTOL, model_rtol=RTOL,
         exact=True)


def test_fused_full_c5(H):
    """C5: Zipf(1.1) keys over 2^24, V_dim = 128, reference defaults (V_threshold = 10,
    l1 = 1, l1_shrk): V is created lazily for the hot keys.  Hot keys' Xᵀ sums run in
    256-occurrence chunks combined in chunk order (reordered sums), so predictions after the
    first update and the model are compared within tolerance (Determinism).  The
    model is held to the drift bound every step (the device within 1e-5 of the reference as a
    vector, and no farther from the exact f64-sum trajectory than the reference is), not to an
    elementwise tolerance: FTRL's L1 threshold turns a last-bit difference of z into w = 0 (round
    6; was close()'s elementwise 1e-3)."""
    cfg = dict(V_dim=128, lr=.05, V_lr=.01)
    batches = [D.synthetic(10_000, 39, 1 << 24, zipf=1.1, seed=7000 + s) for s in range(4)]
    # step 0 reads the oracle's own (empty) model: north_star's 1e-5; after the first chunked
    # update the models differ by the reference's float rounding of hot keys' sums
    _run(H, cfg, batches, n_cnt=2, max_keys=1 << 20, pred_rtol=[RTOL, 1e-4, 1e-4, 1e-4],
         model_rtol=None, drift=1e-5)


def test_calcgrad_c5_chunked(H):
    """C5 per-minibatch gradients through the skewed-key chunk path (dfx_fm_calcgrad builds the
    fused step's chunk plan): B = 10^4 rows of 39 Zipf(1.1) keys over [1, 2^24], V_dim = 128,
    a third of the keys without V.  The hottest key has ~45k occurrences in the batch.

    Keys of <= 256 occurrences are summed in the reference's order (bit-exact up to expf);
    longer ones in 256-occurrence chunks combined in double.  Against float64 sums of the
    reference's own terms (tests/exact_sums.py) the device is within 1e-6 of each element's
    condition scale (sum of |terms|); the reference itself (the oracle) is up to ~3e-5 of that
    scale away — its own sequential float rounding over ~45k terms — so the device and the
    reference agree within 1e-5 relative except where a sum cancels far below its terms (84 of
    8.07 M elements on the GPU box), and their distance is always the reference's rounding plus
    at most 1e-6 of the scale (measured: DESIGN.md, Determinism)."""
    from tests.exact_sums import exact_calcgrad
    d = 128
    blk = D.synthetic(10_000, 39, 1 << 24, zipf=1.1, seed=7100)
    ou, _, ocol = O.localize(blk.offs, blk.ids)
    U = len(ou)
    assert np.bincount(ocol).max() > 40 * 256  # a hot key far beyond one chunk
    rng = np.random.default_rng(5)
    lens = np.where(rng.random(U) < 0.33, 1, d + 1).astype(np.int32)
    wp, vp = O.get_pos(lens)
    W = (rng.standard_normal(int(lens.sum())) * 0.05).astype(np.float32)
    c = H.Context(0)
    db = H.DeviceRowBlock(c, blk)
    col, _, _ = H.Localizer(c).compact(db)
    assert np.array_equal(H.u32(col), ocol)
    loss = H.FMLoss(c, d)
    tW, twp, tvp = c.tensor(W, torch.float32), c.tensor(wp, torch.int32), c.tensor(vp, torch.int32)
    pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
    loss.predict(db, col, tW, twp, tvp, pred, U)
    opred = O.fm_predict(blk.offs, ocol, blk.vals, W, wp, vp, d)
    assert np.array_equal(pred.cpu().numpy(), opred)
    grad = torch.zeros(len(W), dtype=torch.float32, device=c.device)
    loss.calc_grad(db, col, tW, twp, tvp, pred, grad, U)
    g = grad.cpu().numpy().astype(np.float64)
    og = O.fm_calcgrad(blk.offs, ocol, blk.vals, blk.labels, None, W, wp, vp, U, d, opred)
    ex, sc = exact_calcgrad(blk, ocol, W, wp, vp, d, opred, U)
    sc = np.maximum(sc, 1e-30)
    dev_exact = np.abs(g - ex) / sc
    ref_exact = np.abs(og - ex) / sc
    dev_ref = np.abs(g - og)
    rel = dev_ref / np.maximum(np.maximum(np.abs(g), np.abs(og)), 1e-30)
    print("C5 calcgrad: device vs f64 %.3g of scale, reference vs f64 %.3g, device vs reference "
          "%.3g of scale; %d of %d elements beyond 1e-5 relative (cancelling sums)"
          % (dev_exact.max(), ref_exact.max(), (dev_ref / sc).max(), int((rel > RTOL).sum()),
             len(g)))
    # the device sums every gradient to within 1e-6 of its condition scale ...
    assert dev_exact.max() <= 1e-6
    # ... so its distance from the reference is the reference's own float rounding (measured
    # up to ~3e-5 of the scale on hot keys of ~45k occurrences), plus at most that 1e-6
    assert np.all(dev_ref <= ref_exact * sc + 1e-6 * sc)
    # and beyond 1e-5 relative only where a sum cancels far below its terms
    assert int((rel > RTOL).sum()) <= 1e-4 * len(g)
    c.close()


@pytest.mark.timeout(300)
def test_c4_one_shard_full_table():
    """C4 at its own scale on one GPU: one of 8 key-range servers of a 2^30-key model holds
    2^27 keys at V_dim = 64 — its table (2^28 slots of 32 B = 8 GiB, load 0.5) and V pool
    (2^27 rows of [V | Vaux] = 64 GiB) allocated and filled through the sharded owner phases:
    count pushes (fea_cnt 11 > V_threshold 10), then a gradient push that moves every w off
    zero, whose InitV gives every key its V row.  Checks the key and V-row counts, the rand_r
    advance (3 draws per coordinate per key), and the table's probe lengths."""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    from oracle import oracle as O
    N, g, d = 8, 1, 64
    n_keys = 1 << 27
    kw = dict(V_dim=d, V_threshold=10, l1=0, lr=.1, V_lr=.01, seed=3, push_agg="sum")
    c = H.Context(0, max_keys=n_keys, max_vrows=n_keys, **kw)
    sh = DI.Shard(c, N)
    dev = c.device
    chunk = 1 << 24
    stride = (1 << 61) // n_keys  # keys spread over server g's range [g 2^61, (g+1) 2^61)
    S = sh.S
    for i in range(0, n_keys, chunk):
        idx = torch.arange(i, i + chunk, dtype=torch.int64, device=dev)
        keys = (g << 61) + idx * stride + (idx * 7919) % stride
        cnt = torch.full((chunk,), 11.0, dtype=torch.float32, device=dev)
        sh.owner_begin(keys, [chunk] + [0] * (N - 1), cnt, 0)
        # this server's InitV ranking (none yet: w is still 0)
        allc = torch.zeros(N, dtype=torch.int64, device=dev)
        allc[g] = sh.initv_local(0)[0]
        sh.initv_draw(allc, g, 0)
        grads = torch.zeros(chunk * S, dtype=torch.float32, device=dev)
        grads.view(chunk, S)[:, d] = -1.0  # gw: w leaves zero, FTRL with l1 = 0
        sh.owner_push(grads, 0)
        allc = torch.zeros(N, dtype=torch.int64, device=dev)
        allc[g] = sh.initv_local(0)[0]
        sh.initv_draw(allc, g, 0)
        del grads, cnt, keys, idx
    st = H.Store(c).stats()
    assert st["n_keys"] == n_keys
    assert st["n_vrows"] == n_keys
    # rand_r: 3 LCG steps per draw, d draws per InitV, one InitV per key (glibc rand_r)
    A, C, m, a_, c_ = 1, 0, 3 * d * n_keys, 1103515245, 12345
    while m:  # the LCG jumped m steps: s -> A s + C (mod 2^32)
        if m & 1:
            A, C = (a_ * A) % (1 << 32), (a_ * C + c_) % (1 << 32)
        a_, c_ = (a_ * a_) % (1 << 32), (a_ * c_ + c_) % (1 << 32)
        m >>= 1
    assert st["seed"] == (A * 3 + C) % (1 << 32)
    mean, mx, cap = H.Store(c).probe_stats()
    assert cap == 2 * n_keys
    assert mean < 1.0 and mx < 64, (mean, mx)
    # a few keys' state against the updater rule: w after one FTRL step from zero, V drawn
    for i in (0, n_keys // 3, n_keys - 1):
        k = (g << 61) + i * stride + (i * 7919) % stride
        e = H.Store(c).entry(k)
        assert e is not None and e[1] is not None
        assert e[0][3] == 11.0 and e[0][0] != 0.0
    c.close()


@pytest.mark.timeout(300)
def test_c4_eight_ranges_at_scale():
    """C4-shaped twin of test_sharded_eight_ranges_at_scale: V_dim 64, 39 binary nnz per row,
    keys drawn from 2^30, 8 loopback key-range servers each sized for its 2^27-key share of the
    2^30 key space (a 1/8-range table: the range-aware ordered hash), against AggOracle (the
    single reference updater on the concatenated batches)"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    from oracle import dist_oracle as DO
    N, rows, kb, d = 8, 10_000, 30, 64
    kw = dict(V_dim=d, V_threshold=0, lr=0.1, V_lr=0.01, l1=0.0, seed=9)
    ctxs = [H.Context(0, max_keys=1 << 22, max_vrows=1 << 22, push_agg="sum", **kw)
            for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    so = DO.AggOracle(N, **kw)
    for s in range(3):
        step = [D.synthetic(rows, 39, 1 << kb, seed=1900 + 17 * s + r) for r in range(N)]
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        preds = [torch.zeros(rows, dtype=torch.float32, device=ctxs[r].device) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=(s == 0), preds=preds)
        out = so.step(step, push_cnt=(s == 0))
        for r in range(N):
            assert close(preds[r].cpu().numpy(), out[r][2]), (s, r)
            pr = H.progress(ctxs[r])
            assert pr["loss"] == pytest.approx(out[r][0], rel=1e-4), (s, r)
    stats = [H.Store(c).stats() for c in ctxs]
    assert sum(st["n_keys"] for st in stats) == so.one.size()
    assert all(st["seed"] == so.one.seed for st in stats)
    for c in ctxs:
        mean, mx, _ = H.Store(c).probe_stats()
        assert mean < 1.0 and mx < 64, (mean, mx)
        c.close()
