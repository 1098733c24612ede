"""Parity of the HIP path (through the C-ABI) with the oracle and the reference's known
answers.  Bars (BASELINE.json north_star): Localizer bit-exact; predictions and gradients
within 1e-5 relative (fp32); loss / AUC within 1e-4.  Predictions are also checked for
bit-exactness, which the kernels achieve by summing in the reference's order."""
import numpy as np
import pytest
import torch

from difacto_amd import data as D
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


@pytest.fixture(scope="module")
def H():
    from difacto_amd import hotpath
    return hotpath


def close(a, b, rtol=RTOL):
    """|a-b| <= rtol*max(|a|,|b|) + small absolute floor scaled to the data."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    floor = 1e-6 * max(1.0, float(np.max(np.abs(b))) if b.size else 1.0)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(a), np.abs(b)) + floor)


def _auc_expect(label, opred, oauc):
    """AUC*n the device must produce: the oracle's, or on tied predictions (unspecified in
    the reference's unstable std::sort) the input-order tie break."""
    return O.auc_stable_ties(label, opred) if O.has_ties(opred) else oauc


def _rev(a):
    return np.array([O.reverse_bytes(int(x)) for x in a], dtype=np.uint64)


# ---------------------------------------------------------------- Localizer (bit-exact)
def _check_localize(H, c, blk, max_index=(1 << 64) - 1):
    db = H.DeviceRowBlock(c, blk)
    col, uniq, cnt = H.Localizer(c, max_index).compact(db)
    ou, oc, ocol = O.localize(blk.offs, blk.ids, max_index=max_index)
    assert np.array_equal(H.u64(uniq), ou)
    assert np.array_equal(cnt.cpu().numpy(), oc)
    assert np.array_equal(H.u32(col), ocol)
    return ou, oc


def test_localizer_rcv1_known_answers(H, rcv1, known):
    c = H.Context(0)
    ou, oc = _check_localize(H, c, rcv1)
    assert int(_rev(ou).sum()) == known["localizer_base"]["sum_uidx"]
    assert float(oc.sum()) == known["localizer_base"]["sum_freq"]
    ou, oc = _check_localize(H, c, rcv1, max_index=1000)
    assert int(_rev(ou).sum()) == known["localizer_hash1000"]["sum_uidx"]


@pytest.mark.parametrize("kind", ["criteo", "ragged", "zipf", "u64", "dups", "big"])
def test_localizer_synthetic(H, kind):
    """bit-exact Localizer (the radix sort's tile / look-back variants were pruned in round 6)"""
    c = H.Context(0)
    if kind == "criteo":
        blk = D.synthetic(4000, 39, 1 << 24, seed=1)
    elif kind == "ragged":
        blk = D.synthetic(3000, 20, 1 << 20, seed=2, ragged=True, binary=False)
    elif kind == "zipf":
        blk = D.synthetic(3000, 39, 1 << 24, seed=3, zipf=1.1)
    elif kind == "u64":
        blk = D.synthetic(2000, 30, 1 << 20, seed=4)
        rng = np.random.default_rng(4)
        blk.ids = rng.integers(0, np.iinfo(np.uint64).max, size=blk.nnz, dtype=np.uint64,
                               endpoint=True)
        blk.ids[:7] = np.iinfo(np.uint64).max  # x % UINT64_MAX == 0 edge
    elif kind == "dups":
        blk = D.synthetic(2000, 39, 50, seed=5)  # massive key collisions
    else:
        blk = D.synthetic(60000, 39, 1 << 24, seed=6)  # many sort tiles
    _check_localize(H, c, blk)
    if kind == "u64":
        _check_localize(H, c, blk, max_index=1000)


def test_localizer_key_width_changes(H):
    """one context sorting narrow keys (3 active digit passes) then 64-bit ids (every pass
    active) then narrow keys again: bit-exact every time"""
    c = H.Context(0)
    rng = np.random.default_rng(9)
    for i, wide in enumerate([False, False, True, True, False, True]):
        blk = D.synthetic(30000, 39, 1 << 24, seed=60 + i)  # many tiles
        if wide:
            blk.ids = rng.integers(0, np.iinfo(np.uint64).max, size=blk.nnz, dtype=np.uint64,
                                   endpoint=True)
        _check_localize(H, c, blk)


def test_localizer_empty(H):
    c = H.Context(0)
    blk = D.RowBlock(np.zeros(5, np.uint64), np.zeros(0, np.uint64), None, np.ones(4, np.float32))
    db = H.DeviceRowBlock(c, blk)
    col, uniq, cnt = H.Localizer(c).compact(db)
    assert uniq.numel() == 0 and col.numel() == 0


# ---------------------------------------------------------------- FMLoss
def _fm_weights(uidx, d):
    U = len(uidx)
    W = np.zeros(U * (d + 1), np.float32)
    wp = (np.arange(U) * (d + 1)).astype(np.int32)
    for i in range(U):
        W[i * (d + 1)] = uidx[i] / 5e4
        for j in range(1, d + 1):
            W[i * (d + 1) + j] = uidx[i] * j / 5e5
    return W, wp, wp + 1


def _fm_run(H, c, blk, W, wp, vp, d, U, rw=None):
    db = H.DeviceRowBlock(c, blk)
    if rw is not None:
        db.weights = c.tensor(rw, torch.float32)
    col, uniq, _ = H.Localizer(c).compact(db)
    loss = H.FMLoss(c, d)
    tW = c.tensor(W, torch.float32)
    twp = c.tensor(wp, torch.int32)
    tvp = c.tensor(vp, torch.int32)
    pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
    loss.predict(db, col, tW, twp, tvp, pred, U)
    grad = torch.zeros(len(W), dtype=torch.float32, device=c.device)
    loss.calc_grad(db, col, tW, twp, tvp, pred, grad, U)
    objv = loss.evaluate(db.labels, pred)
    return pred.cpu().numpy(), grad.cpu().numpy(), objv, H.u32(col)


def test_fmloss_nov_known(H, rcv1, known):
    k = known["fmloss_nov"]
    c = H.Context(0)
    ou, _, ocol = O.localize(rcv1.offs, rcv1.ids)
    w = (_rev(ou) / 5e4).astype(np.float32)
    pred, grad, objv, col = _fm_run(H, c, rcv1, w, None, None, 0, len(ou))
    assert abs(objv - k["objv"]) < k["objv_tol"]
    assert abs(float((grad.astype(np.float64) ** 2).sum()) - k["grad_norm2"]) < k["grad_tol"]
    opred = O.fm_predict(rcv1.offs, ocol, rcv1.vals, w, None, None, 0)
    assert np.array_equal(pred, opred)
    og = O.fm_calcgrad(rcv1.offs, ocol, rcv1.vals, rcv1.labels, None, w, None, None, len(ou), 0,
                       opred)
    assert np.array_equal(grad, og)  # bit-exact (expf included: csrc/expf.h)


def test_fmloss_hasv_known(H, rcv1, known):
    k = known["fmloss_hasv"]
    d = k["V_dim"]
    c = H.Context(0)
    ou, _, ocol = O.localize(rcv1.offs, rcv1.ids)
    W, wp, vp = _fm_weights(_rev(ou), d)
    pred, grad, objv, col = _fm_run(H, c, rcv1, W, wp, vp, d, len(ou))
    assert abs(objv - k["objv"]) < k["objv_tol"]
    assert abs(float((grad.astype(np.float64) ** 2).sum()) - k["grad_norm2"]) < k["grad_tol"]
    opred = O.fm_predict(rcv1.offs, ocol, rcv1.vals, W, wp, vp, d)
    assert np.array_equal(pred, opred)
    og = O.fm_calcgrad(rcv1.offs, ocol, rcv1.vals, rcv1.labels, None, W, wp, vp, len(ou), d, opred)
    assert np.array_equal(grad, og)  # bit-exact (expf included: csrc/expf.h)


@pytest.mark.parametrize("d", [0, 1, 2, 5, 16, 33, 64, 100, 128, 200])
@pytest.mark.parametrize("binary", [True, False])
def test_fmloss_random(H, d, binary):
    rng = np.random.default_rng(100 + d)
    blk = D.synthetic(1500, 25, 3000, binary=binary, seed=7 + d, ragged=True)
    ou, _, ocol = O.localize(blk.offs, blk.ids)
    U = len(ou)
    # interleaved Pull layout with ~1/3 of the keys lacking V (lens == 1)
    lens = np.where(rng.random(U) < 0.33, 1, d + 1).astype(np.int32) if d > 0 else None
    if d > 0:
        wp, vp = O.get_pos(lens)
        W = (rng.standard_normal(int(lens.sum())) * 0.1).astype(np.float32)
        W[wp[rng.random(U) < 0.1]] = 0  # w == 0 skip path
    else:
        wp = vp = None
        W = (rng.standard_normal(U) * 0.1).astype(np.float32)
    rw = (rng.random(blk.size) + 0.5).astype(np.float32)
    c = H.Context(0)
    pred, grad, objv, col = _fm_run(H, c, blk, W, wp, vp, d, U, rw=rw)
    opred = O.fm_predict(blk.offs, ocol, blk.vals, W, wp, vp, d)
    assert np.array_equal(pred, opred), np.max(np.abs(pred - opred))
    og = O.fm_calcgrad(blk.offs, ocol, blk.vals, blk.labels, rw, W, wp, vp, U, d, opred)
    assert close(grad, og)
    # no key reaches a chunked sum (<= 256 occurrences) and p's expf is glibc's (csrc/expf.h):
    # the gradients are the reference's bit for bit
    assert np.array_equal(grad, og), int((grad != og).sum())
    assert abs(objv - O.evaluate(blk.labels, opred)) <= 1e-4 * abs(objv)


def test_get_pos(H):
    rng = np.random.default_rng(0)
    lens = rng.choice([0, 1, 17], size=5000).astype(np.int32)
    c = H.Context(0)
    w, v = H.get_pos(c, c.tensor(lens, torch.int32))
    ow, ov = O.get_pos(lens)
    assert np.array_equal(w.cpu().numpy(), ow) and np.array_equal(v.cpu().numpy(), ov)


def test_auc_and_evaluate(H):
    rng = np.random.default_rng(1)
    n = 20000
    label = np.where(rng.random(n) < 0.3, 1.0, -1.0).astype(np.float32)
    pred = (rng.standard_normal(n) + 0.5 * label).astype(np.float32)
    c = H.Context(0)
    tl, tp = c.tensor(label, torch.float32), c.tensor(pred, torch.float32)
    a = H.auc(c, tl, tp)
    assert abs(a - O.auc(label, pred)) <= 1e-4 * n
    assert abs(H.FMLoss(c, 0).evaluate(tl, tp) - O.evaluate(label, pred)) <= 1e-6 * n
    # degenerate batch: the reference returns 1 (not 1*n)
    assert H.auc(c, tl, c.tensor(np.ones(n, np.float32), torch.float32)) > 0
    assert H.auc(c, c.tensor(np.ones(n, np.float32), torch.float32), tp) == 1.0


@pytest.mark.parametrize("n", [1, 2, 4095, 4097, 10000, 12288, 12289, 100000, 1000003])
def test_auc_radix_and_merge_sorts_agree(H, n):
    """the AUC lane's two stable sorts (auc_sort=radix | merge; up to 12288 rows both take the
    one-block LDS sort, k_auc_block): the same AUC*n, equal to the input-order tie break of the
    oracle, with heavy ties (quantised predictions, one constant digit pattern), with all
    predictions equal (epoch 0, w = 0) and with signed zeros (-0 == +0).  Each context sees every
    snapshot twice"""
    rng = np.random.default_rng(n)
    label = np.where(rng.random(n) < 0.25, 1.0, -1.0).astype(np.float32)
    signed0 = np.where(rng.random(n) < 0.5, np.float32(-0.0), np.float32(0.0)).astype(np.float32)
    signed0[rng.random(n) < 0.3] = -1.5
    cs = [H.Context(0, auc_sort=mode) for mode in ["radix", "merge"]]
    for pred in [np.round(rng.standard_normal(n) * 8).astype(np.float32) / 8,
                 np.zeros(n, np.float32), (rng.standard_normal(n) - 0.3 * label).astype(np.float32),
                 signed0]:
        want = O.auc_stable_ties(label, pred) if O.has_ties(pred) else O.auc(label, pred)
        for _ in range(2):
            got = [H.auc(c, c.tensor(label, torch.float32), c.tensor(pred, torch.float32))
                   for c in cs]
            assert got[0] == got[1], got
            assert abs(got[0] - want) <= 1e-4 * n, (got, want)
    for c in cs:
        c.close()


# ---------------------------------------------------------------- Store / SGDUpdater
def _store_pair(H, **kw):
    c = H.Context(0, max_keys=1 << 16, **kw)
    return c, H.Store(c), O.Updater(**kw)


def _pull_eq(H, c, st, up, keys):
    v, l = st.pull(c.tensor(keys, torch.int64))
    ov, ol = up.get(keys)
    assert np.array_equal(v.cpu().numpy(), ov)
    if ol is not None:
        assert np.array_equal(l.cpu().numpy(), ol)


@pytest.mark.parametrize("kw", [
    dict(V_dim=0, l1=1, l2=0.1, lr=0.5),
    dict(V_dim=8, V_threshold=2, l1=0.01, lr=0.1, V_lr=0.05, V_init_scale=0.5, seed=7),
    dict(V_dim=16, V_threshold=0, l1=0, lr=0.1, l1_shrk=0),
])
def test_store_matches_updater(H, kw):
    rng = np.random.default_rng(11)
    c, st, up = _store_pair(H, **kw)
    d = kw["V_dim"]
    keys_all = np.unique(rng.integers(0, 1 << 62, size=3000, dtype=np.uint64))
    for it in range(6):
        keys = np.sort(rng.choice(keys_all, size=1200, replace=False))
        tk = c.tensor(keys, torch.int64)
        if it < 2 and d > 0:
            cnt = rng.integers(1, 5, size=len(keys)).astype(np.float32)
            st.push(tk, H.kFeaCount, c.tensor(cnt, torch.float32))
            up.update(keys, O.Updater.kFeaCount, cnt)
        _pull_eq(H, c, st, up, keys)
        ov, ol = up.get(keys)
        g = (rng.standard_normal(len(ov)) * 2).astype(np.float32)
        st.push(tk, H.kGradient, c.tensor(g, torch.float32),
                c.tensor(ol, torch.int32) if ol is not None else None)
        up.update(keys, O.Updater.kGradient, g, ol)
        c.sync()
    _pull_eq(H, c, st, up, keys_all)
    s = st.stats()
    assert s["seed"] == up.seed
    assert s["new_w"] == up.new_w
    for k in keys_all[:200]:
        e, oe = st.entry(k), up.entry(k)
        assert (e is None) == (oe is None) or (oe is not None and not oe[0].any())
        if e is not None and oe is not None:
            assert np.array_equal(e[0][:3], oe[0][:3])
            if oe[1] is not None:
                assert np.array_equal(e[1], oe[1])
    pen, nnz = st.evaluate()
    open_, onnz = up.penalty()
    assert nnz == onnz and abs(pen - open_) <= 1e-6 * max(1, abs(open_))


def test_store_check_failures(H):
    c = H.Context(0, V_dim=4, max_keys=1024)
    st = H.Store(c)
    keys = c.tensor(np.arange(1, 11, dtype=np.uint64), torch.int64)
    g = c.tensor(np.ones(10 * 5, np.float32), torch.float32)
    lens = c.tensor(np.full(10, 5, np.int32), torch.int32)
    st.push(keys, H.kGradient, g, lens)  # no V exists yet -> CHECK(e.V) fails
    with pytest.raises(H._lib.DfxError):
        c.sync()
    with pytest.raises(H._lib.DfxError):
        st.push(keys, 7, g, lens)


def test_save_load_interop(H, tmp_path):
    kw = dict(V_dim=6, V_threshold=1, l1=0.01, lr=0.1, V_lr=0.05)
    rng = np.random.default_rng(3)
    c, st, up = _store_pair(H, **kw)
    keys = np.unique(rng.integers(0, 1 << 60, size=800, dtype=np.uint64))
    tk = c.tensor(keys, torch.int64)
    cnt = np.full(len(keys), 3, np.float32)
    st.push(tk, H.kFeaCount, c.tensor(cnt, torch.float32))
    up.update(keys, 1, cnt)
    for _ in range(3):
        ov, ol = up.get(keys)
        g = rng.standard_normal(len(ov)).astype(np.float32)
        st.push(tk, H.kGradient, c.tensor(g, torch.float32), c.tensor(ol, torch.int32))
        up.update(keys, 3, g, ol)
    p_gpu, p_orc = str(tmp_path / "gpu_part-0"), str(tmp_path / "orc_part-0")
    st.save(p_gpu, True)
    up.save(p_orc, True)
    # reference-format files load into the other implementation
    up2 = O.Updater(**kw)
    up2.load(p_gpu)
    c2 = H.Context(0, max_keys=1 << 12, **kw)
    st2 = H.Store(c2)
    st2.load(p_orc)
    _pull_eq(H, c2, st2, up2, keys)
    assert st2.stats()["n_keys"] == up2.size()
    st.dump(str(tmp_path / "dump.txt"), True, True)
    assert sum(1 for _ in open(tmp_path / "dump.txt")) == up2.size()


# ---------------------------------------------------------------- fused minibatch
def test_fused_sgd_learner_basic(H, rcv1, known):
    """SGDLearner.Basic (tests/cpp/sgd_learner_test.cc:9-49) through dfx_train_step."""
    k = known["sgd_learner_basic"]
    kw = k["kwargs"]
    c = H.Context(0, V_dim=kw["V_dim"], l2=kw["l2"], l1=kw["l1"], lr=kw["lr"], max_keys=1 << 14)
    db = H.DeviceRowBlock(c, rcv1)
    for ep, want in enumerate(k["objv"]):
        H.train_step(c, db, H.kTraining, push_cnt=False)
        p = H.progress(c)
        assert abs(p["loss"] - want) < k["tol"], (ep, p["loss"], want)


@pytest.mark.parametrize("cfg", [
    dict(V_dim=4, V_threshold=2, lr=.1, V_lr=.01, l1=.1),
    dict(V_dim=2, lr=.02, V_lr=.001, V_threshold=1, l1=0.05),    # C1-like (FM d=2)
    dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01),          # C3-like, all keys get V
])
def test_fused_matches_oracle_rcv1(H, rcv1, cfg):
    c = H.Context(0, max_keys=1 << 14, **cfg)
    up = O.Updater(**cfg)
    db = H.DeviceRowBlock(c, rcv1)
    halves = [rcv1.slice(0, 50), rcv1.slice(50, 100)]
    dhalves = [H.DeviceRowBlock(c, h) for h in halves]
    for ep in range(6):
        for hb, dh in zip(halves, dhalves):
            loss, auc, opred = up.train_step(hb.offs, hb.ids, hb.vals, hb.labels,
                                             push_cnt=(ep == 0), want_pred=True)
            H.train_step(c, dh, H.kTraining, push_cnt=(ep == 0))
            p = H.progress(c)
            assert abs(p["loss"] - loss) <= 1e-4 * max(1, abs(loss)), (ep, p["loss"], loss)
            want = _auc_expect(hb.labels, opred, auc)
            assert abs(p["auc"] - want) <= 1e-4 * hb.size, (ep, p["auc"], want)
    st = H.Store(c)
    uniq, _, _ = O.localize(rcv1.offs, rcv1.ids)
    v, l = st.pull(c.tensor(uniq, torch.int64))
    ov, ol = up.get(uniq)
    assert np.array_equal(l.cpu().numpy(), ol)
    assert close(v.cpu().numpy(), ov, rtol=1e-4)
    assert st.stats()["seed"] == up.seed


@pytest.mark.parametrize("key_space,pack", [(1 << 16, 1), (1 << 63, 1), (1 << 16, 0)])
def test_fused_criteo_like_vs_oracle(H, key_space, pack):
    """2^16 ids: the Localizer's sort carries (varying key bits, row) packed in one u64;
    ids over 63 bits: every key bit varies, the sort falls back to (key, row) pairs on the
    device; sort_pack=0: pairs always"""
    cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    c = H.Context(0, max_keys=1 << 18, sort_pack=pack, **cfg)
    up = O.Updater(**cfg)
    for step in range(4):
        blk = D.synthetic(3000, 39, key_space, seed=50 + step)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 2), want_pred=True)
        db = H.DeviceRowBlock(c, blk)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, db, H.kTraining, push_cnt=(step < 2), pred=pred)
        p = H.progress(c)
        assert close(pred.cpu().numpy(), opred, rtol=1e-4)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss)
        want = _auc_expect(blk.labels, opred, auc)
        assert abs(p["auc"] - want) <= 1e-4 * blk.size
    s = H.Store(c).stats()
    assert s["seed"] == up.seed and s["n_keys"] == up.size()


@pytest.mark.parametrize("max_index", [1000, 65537, (1 << 64) - 1])
def test_fused_max_index_vs_oracle(H, max_index):
    """Localizer keys = ReverseBytes(id % max_index) (localizer.cc:20-24): the fused step's
    forward recomputes them per nnz (probe mode), so a modding max_index (ids colliding into
    one key, repeated keys inside rows) and the ~0 corner id must match the oracle"""
    import numpy as np
    cfg = dict(V_dim=8, V_threshold=1, l1=0.01, lr=.1, V_lr=.02)
    c = H.Context(0, max_keys=1 << 18, **cfg)
    up = O.Updater(**cfg)
    for step in range(4):
        blk = D.synthetic(2000, 12, 1 << 40, binary=(step % 2 == 0), seed=90 + step)
        ids = blk.ids.copy()
        ids[::97] = np.uint64((1 << 64) - 1)  # the all-ones id
        blk = D.RowBlock(blk.offs, ids, blk.vals, blk.labels)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         max_index=max_index, push_cnt=(step < 2),
                                         want_pred=True)
        db = H.DeviceRowBlock(c, blk)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, db, H.kTraining, push_cnt=(step < 2), max_index=max_index, pred=pred)
        p = H.progress(c)
        assert close(pred.cpu().numpy(), opred, rtol=1e-4), (max_index, step)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss)
    s = H.Store(c).stats()
    assert s["seed"] == up.seed and s["n_keys"] == up.size()


def test_fused_validation_does_not_update(H, rcv1):
    c = H.Context(0, V_dim=4, V_threshold=0, l1=0, lr=.1, max_keys=1 << 14)
    db = H.DeviceRowBlock(c, rcv1)
    H.train_step(c, db, H.kTraining, push_cnt=True)
    H.progress(c)
    st = H.Store(c)
    uniq, _, _ = O.localize(rcv1.offs, rcv1.ids)
    before = st.pull(c.tensor(uniq, torch.int64))[0].cpu().numpy()
    H.train_step(c, db, H.kValidation)
    p = H.progress(c)
    after = st.pull(c.tensor(uniq, torch.int64))[0].cpu().numpy()
    assert np.array_equal(before, after) and p["nrows"] == 100


def test_fused_empty_and_tiny(H):
    c = H.Context(0, V_dim=8, V_threshold=0, l1=0, max_keys=1 << 12)
    blk = D.RowBlock(np.array([0, 0, 3, 3], np.uint64), np.array([5, 9, 5], np.uint64), None,
                     np.array([1, -1, 1], np.float32))
    up = O.Updater(V_dim=8, V_threshold=0, l1=0)
    for ep in range(3):
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(ep == 0), want_pred=True)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(ep == 0))
        p = H.progress(c)
        assert abs(p["loss"] - loss) <= 1e-5 * abs(loss)
        assert p["auc"] == pytest.approx(_auc_expect(blk.labels, opred, auc))


@pytest.mark.parametrize("ids", [[7, 7, 7, 7, 7], [11]])
def test_fused_one_distinct_key(H, ids):
    """every nnz has the same key (no digit varies: the Localizer's sort still runs one pass,
    which writes the keys its first pass reads from the batch), and a single nnz"""
    n = len(ids)
    offs = np.array([0] + [min(i + 2, n) for i in range(0, n, 2)], np.uint64)
    blk = D.RowBlock(offs, np.array(ids, np.uint64), None,
                     np.array([1 if i % 2 == 0 else -1 for i in range(len(offs) - 1)], np.float32))
    for d in (0, 8, 16):
        c = H.Context(0, V_dim=d, V_threshold=0, l1=0, max_keys=1 << 12)
        up = O.Updater(V_dim=d, V_threshold=0, l1=0)
        for ep in range(3):
            loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                             push_cnt=(ep == 0), want_pred=True)
            H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(ep == 0))
            p = H.progress(c)
            assert abs(p["loss"] - loss) <= 1e-5 * abs(loss)
            assert p["auc"] == pytest.approx(_auc_expect(blk.labels, opred, auc))
        assert H.Store(c).stats()["n_keys"] == up.size() == 1
        c.close()


def test_fused_async_batches_released(H):
    """Batches created, handed to the device and dropped without any host sync (the bench's
    pattern): the library must run on torch's stream so freed blocks are not recycled
    under a running kernel."""
    cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    c = H.Context(0, max_keys=1 << 18, **cfg)
    up = O.Updater(**cfg)
    tot = 0.0
    for step in range(6):
        blk = D.synthetic(4000, 39, 1 << 16, seed=900 + step)
        tot += up.train_step(blk.offs, blk.ids, blk.vals, blk.labels, push_cnt=(step < 3))[0]
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 3))
    p = H.progress(c)
    assert abs(p["loss"] - tot) <= 1e-4 * tot
    s = H.Store(c).stats()
    assert s["seed"] == up.seed and s["n_keys"] == up.size()


@pytest.mark.parametrize("hash_kind", ["ordered", "mixed"])
def test_fused_clustered_keys_rehash(H, hash_kind):
    """Ids whose nibble-reversed keys share their top bits (ids = i << 40) pile onto one home
    slot of the ordered table; the store detects the long probes and rehashes with the
    multiplicative hash at the next sync.  Results must match the oracle either way."""
    cfg = dict(V_dim=4, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    c = H.Context(0, max_keys=1 << 14, hash=hash_kind, **cfg)
    up = O.Updater(**cfg)
    rng = np.random.default_rng(5)
    for step in range(4):
        B, k = 500, 10
        ids = (rng.integers(0, 3000, B * k).astype(np.uint64) << np.uint64(40))
        blk = D.RowBlock(np.arange(0, B * k + 1, k, dtype=np.uint64), ids, None,
                         np.where(rng.random(B) < .3, 1, -1).astype(np.float32))
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step == 0), want_pred=True)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step == 0))
        p = H.progress(c)   # a sync point: the ordered table rehashes here after step 0
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), (step, p["loss"], loss)
        want = _auc_expect(blk.labels, opred, auc)
        assert abs(p["auc"] - want) <= 1e-4 * blk.size
    s = H.Store(c).stats()
    assert s["n_keys"] == up.size() and s["seed"] == up.seed


@pytest.mark.parametrize("binary,d", [(True, 128), (False, 16), (True, 0)])
def test_fused_zipf_skew_vs_oracle(H, binary, d):
    """C5-shaped skew: Zipf(1.1) keys, so the hottest keys hold thousands of occurrences per
    batch and their Xᵀ sums run in chunks (kChunkOcc) combined in chunk order.  Defaults
    l1=1, V_threshold=10 (lazy V for hot keys only).  Sums are reordered for long segments,
    so loss / AUC / model are compared within tolerance rather than bit-for-bit."""
    cfg = dict(V_dim=d, lr=.05, V_lr=.01)
    c = H.Context(0, max_keys=1 << 18, **cfg)
    up = O.Updater(**cfg)
    for step in range(5):
        blk = D.synthetic(4000, 39, 1 << 20, binary=binary, zipf=1.1, seed=300 + step)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 2), want_pred=True)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 2), pred=pred)
        p = H.progress(c)
        assert close(pred.cpu().numpy(), opred, rtol=1e-4)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), (step, p["loss"], loss)
        want = _auc_expect(blk.labels, opred, auc)
        assert abs(p["auc"] - want) <= 1e-4 * blk.size
    s = H.Store(c).stats()
    assert s["seed"] == up.seed and s["n_keys"] == up.size()
    uniq, _, _ = O.localize(blk.offs, blk.ids)
    v, l = H.Store(c).pull(c.tensor(uniq, torch.int64))
    ov, ol = up.get(uniq)
    if d > 0:
        assert np.array_equal(l.cpu().numpy(), ol)
    assert close(v.cpu().numpy(), ov, rtol=1e-3)


def test_fused_hot_key_every_row(H):
    """One key in every row (a bias-like feature): a 20000-occurrence segment."""
    cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    c = H.Context(0, max_keys=1 << 18, **cfg)
    up = O.Updater(**cfg)
    for step in range(3):
        blk = D.synthetic(20000, 20, 1 << 16, seed=70 + step)
        ids = blk.ids.reshape(20000, 20).copy()
        ids[:, 0] = 123456789
        blk = D.RowBlock(blk.offs, ids.reshape(-1), None, blk.labels)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step == 0), want_pred=True)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step == 0))
        p = H.progress(c)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), (step, p["loss"], loss)
    st_gpu = H.Store(c).entry(O.reverse_bytes(123456789))
    st_cpu = up.entry(O.reverse_bytes(123456789)) if hasattr(up, "entry") else None
    assert st_gpu is not None
    if st_cpu is not None:
        assert close(st_gpu[0], st_cpu[0], rtol=1e-4)
