"""The device store's two slot layouts (common.h Table::es) and its capacity behaviour, through
the C-ABI, against the oracle (SGDUpdater, sgd_updater.cc:34-152):

* split: 32-byte entries, [V | Vaux] rows in a pool allocated by InitV in key order;
* fat (slot_layout=auto at 4 <= V_dim <= 24): the entry and V in one 64/128-byte slot, Vaux in a
  pool row per slot — the forward's lookup and its V read are one line.

Both must give the reference's results bit for bit where the reference order is kept (the store
calls) and within the fused step's tolerances; model files must cross between them; the table
must grow on its own past max_keys (a rehash moves a fat slot's V and Vaux with it); and with
growth off, a full table must never write a failed key's update into another key's slot."""
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


def _pull_eq(c, st, up, keys):
    v, l = st.pull(c.tensor(keys, torch.int64))
    ov, ol = up.get(keys)
    assert np.array_equal(v.cpu().numpy(), ov)
    if ol is not None:
        assert np.array_equal(l.cpu().numpy(), ol)


def _train_store(H, c, st, up, keys, rng, steps=3):
    tk = c.tensor(keys, torch.int64)
    cnt = np.full(len(keys), 3, np.float32)
    st.push(tk, H.kFeaCount, c.tensor(cnt, torch.float32))
    up.update(keys, O.Updater.kFeaCount, cnt)
    for _ in range(steps):
        ov, ol = up.get(keys)
        g = rng.standard_normal(len(ov)).astype(np.float32)
        st.push(tk, H.kGradient, c.tensor(g, torch.float32),
                c.tensor(ol, torch.int32) if ol is not None else None)
        up.update(keys, O.Updater.kGradient, g, ol)


@pytest.mark.parametrize("d,layout", [(8, "fat"), (8, "split"), (16, "fat"), (4, "fat")])
def test_store_layouts_match_updater(H, d, layout):
    kw = dict(V_dim=d, V_threshold=1, l1=0.01, lr=0.1, V_lr=0.05, V_init_scale=0.5, seed=5)
    rng = np.random.default_rng(d)
    c = H.Context(0, max_keys=1 << 14, slot_layout=layout, **kw)
    st, up = H.Store(c), O.Updater(**kw)
    keys = np.unique(rng.integers(0, 1 << 62, size=2000, dtype=np.uint64))
    _train_store(H, c, st, up, keys, rng)
    _pull_eq(c, st, up, keys)
    s = st.stats()
    assert s["seed"] == up.seed and s["n_keys"] == up.size() and s["new_w"] == up.new_w
    for k in keys[:100]:
        e, oe = st.entry(k), up.entry(k)
        assert np.array_equal(e[0][:3], oe[0][:3])
        if oe[1] is not None:
            assert np.array_equal(e[1], oe[1])  # [V | Vaux]


def test_fat_layout_needs_its_vdim(H):
    with pytest.raises(H._lib.DfxError):
        H.Context(0, V_dim=6, slot_layout="fat")
    with pytest.raises(H._lib.DfxError):
        H.Context(0, V_dim=32, slot_layout="fat")


@pytest.mark.parametrize("src,dst", [("fat", "split"), ("split", "fat"), ("fat", "fat")])
def test_model_files_cross_layouts(H, tmp_path, src, dst):
    """SGDUpdater::Save's format (sgd_updater.h:84-106) written by one layout loads into the
    other and into the oracle; the oracle's file loads into both"""
    kw = dict(V_dim=8, V_threshold=1, l1=0.01, lr=0.1, V_lr=0.05)
    rng = np.random.default_rng(9)
    c = H.Context(0, max_keys=1 << 12, slot_layout=src, **kw)
    st, up = H.Store(c), O.Updater(**kw)
    keys = np.unique(rng.integers(0, 1 << 60, size=900, dtype=np.uint64))
    _train_store(H, c, st, up, keys, rng)
    p_gpu, p_orc = str(tmp_path / "gpu_part-0"), str(tmp_path / "orc_part-0")
    st.save(p_gpu, True)
    up.save(p_orc, True)
    for path in (p_gpu, p_orc):
        c2 = H.Context(0, max_keys=1 << 12, slot_layout=dst, **kw)
        st2 = H.Store(c2)
        st2.load(path)
        up2 = O.Updater(**kw)
        up2.load(path)
        _pull_eq(c2, st2, up2, keys)
        assert st2.stats()["n_keys"] == up2.size()
        for k in keys[:50]:
            e, oe = st2.entry(k), up2.entry(k)
            assert np.array_equal(e[0][:3], oe[0][:3])
            if oe[1] is not None:
                assert np.array_equal(e[1], oe[1])
        c2.close()
    st.dump(str(tmp_path / "dump.txt"), True, True)
    assert sum(1 for _ in open(tmp_path / "dump.txt")) == up.size()


@pytest.mark.parametrize("d,layout", [(16, "fat"), (16, "split"), (8, "fat"), (0, "auto")])
def test_fused_steps_grow_the_table(H, d, layout):
    """max_keys=1024 (2048 slots) while the batches bring ~40k keys: the store grows at sync
    points by itself (load kept below 0.5 between steps), and every step still equals the
    reference's: loss / AUC within 1e-4, keys, RNG state and the final model exact-ish"""
    cfg = dict(V_dim=d, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    c = H.Context(0, max_keys=1024, slot_layout=layout, **cfg)
    up = O.Updater(**cfg)
    cap0 = H.Store(c).probe_stats()[2]
    for step in range(6):
        blk = D.synthetic(2000, 20, 1 << 18, seed=300 + step)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 2), want_pred=True)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 2))
        p = H.progress(c)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss), (step, p["loss"], loss)
        want = O.auc_stable_ties(blk.labels, opred) if O.has_ties(opred) else auc
        assert abs(p["auc"] - want) <= 1e-4 * blk.size
    st = H.Store(c)
    s = st.stats()
    assert s["n_keys"] == up.size() and s["seed"] == up.seed
    mean_probe, max_probe, cap = st.probe_stats()
    assert cap > 16 * cap0 and 2 * s["n_keys"] <= cap * 1.0 + 1
    uniq = np.unique(np.concatenate(
        [O.localize(b.offs, b.ids)[0]
         for b in (D.synthetic(2000, 20, 1 << 18, seed=300 + i) for i in range(6))]))
    v, l = st.pull(c.tensor(uniq, torch.int64))
    ov, ol = up.get(uniq)
    if ol is not None:
        assert np.array_equal(l.cpu().numpy(), ol)
    a, b = v.cpu().numpy().astype(np.float64), ov.astype(np.float64)
    assert np.all(np.abs(a - b) <= 1e-4 * np.maximum(np.abs(a), np.abs(b)) + 1e-6)


@pytest.mark.parametrize("layout", ["fat", "split"])
def test_full_table_never_touches_other_keys(H, layout):
    """autogrow=0, a table that cannot hold the pushed keys: the error surfaces at the next sync
    (kErrTableFull), and the keys already stored keep exactly their state — a failed insert
    writes nowhere (round-1's fallback to slot 0 wrote a foreign key's state)"""
    kw = dict(V_dim=8, V_threshold=0, l1=0, lr=0.1, V_lr=0.05)
    rng = np.random.default_rng(4)
    c = H.Context(0, max_keys=1024, max_vrows=1 << 13, autogrow=0, slot_layout=layout,
                  **kw)  # 2048 slots
    st, up = H.Store(c), O.Updater(**kw)
    old = np.unique(rng.integers(1, 1 << 62, size=1500, dtype=np.uint64))
    _train_store(H, c, st, up, old, rng, steps=2)
    c.sync()
    before = st.pull(c.tensor(old, torch.int64))[0].cpu().numpy().copy()
    new = np.setdiff1d(np.unique(rng.integers(1, 1 << 62, size=1200, dtype=np.uint64)), old)
    g = rng.standard_normal(len(new)).astype(np.float32)
    st.push(c.tensor(new, torch.int64), H.kGradient, c.tensor(g, torch.float32),
            c.tensor(np.ones(len(new), np.int32), torch.int32))
    with pytest.raises(H._lib.DfxError):
        c.sync()
    after = st.pull(c.tensor(old, torch.int64))[0].cpu().numpy()
    assert np.array_equal(before, after)


def test_reserved_key_is_rejected(H):
    """key ~0 marks a free slot: the raw-key store calls refuse it (kErrBadKey at the sync)"""
    c = H.Context(0, V_dim=8, max_keys=1024)
    st = H.Store(c)
    keys = c.tensor(np.array([5, (1 << 64) - 1], dtype=np.uint64), torch.int64)
    st.push(keys, H.kFeaCount, c.tensor(np.ones(2, np.float32), torch.float32))
    with pytest.raises(H._lib.DfxError):
        c.sync()


@pytest.mark.parametrize("d", [4, 12, 20, 24])
def test_fused_fat_layout_other_vdims(H, d):
    """fat slots at V_dims whose forward is not the one-trip kernel (d = 4: one lane per row;
    12, 20, 24: lane groups wider than d / 4) walk the fat layout through the generic probe
    forward; each step equals the reference's"""
    cfg = dict(V_dim=d, V_threshold=1, l1=0.01, lr=.1, V_lr=.02)
    c = H.Context(0, max_keys=1 << 16, slot_layout="fat", **cfg)
    up = O.Updater(**cfg)
    for step in range(4):
        blk = D.synthetic(1500, 25, 1 << 14, seed=700 + step)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 1), want_pred=True)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 1), pred=pred)
        p = H.progress(c)
        a, b = pred.cpu().numpy().astype(np.float64), opred.astype(np.float64)
        assert np.all(np.abs(a - b) <= 1e-5 * np.maximum(np.abs(a), np.abs(b)) + 1e-6)
        assert abs(p["loss"] - loss) <= 1e-4 * abs(loss)
    s = H.Store(c).stats()
    assert s["seed"] == up.seed and s["n_keys"] == up.size()
