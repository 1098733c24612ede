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


# ---------------------------------------------------------------- the splitter map
def _hot_ids(kind, rng, n, step):
    if kind == "zipf":      # C5's keys: Zipf(1.1) over 2^24, the top key ~11 % of the nnz
        return D.zipf_keys(rng, n, 1.1, 1 << 24)
    if kind == "one_hot":   # one key in 40 % of the nnz, the rest uniform
        ids = rng.integers(0, 1 << 22, n, dtype=np.uint64)
        ids[rng.random(n) < 0.4] = 12345
        return ids
    if kind == "drift":     # the hot keys change every step: yesterday's splitters misplace them
        return (D.zipf_keys(rng, n, 1.1, 1 << 20) + np.uint64(7919 * step)) % np.uint64(1 << 20)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["zipf", "one_hot", "drift"])
@pytest.mark.parametrize("rows", [60000, 100])
def test_bucket_splitter_map_equals_lsd(H, kind, rows):
    """The bucket Localizer on skewed binary batches (locbucket.hip's splitter map: after a
    batch with a hot key, the next batch's buckets follow that batch's (key, row) quantiles, and
    a hot key's occurrences spread over buckets of their own, its run continued across them)
    against the onesweep radix Localizer (loc_bucket=0): predictions, loss and AUC identical
    every step, the model identical at the end, and within the usual tolerances of the oracle.
    Equal-sized batches so the map engages from the second step; 100-row batches give 4
    buckets, so runs continue over buckets with parts shorter than a chunk; 'drift' moves the
    hot keys under stale splitters (oversize buckets: the global-memory passes)."""
    cfg = dict(V_dim=16, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    cs = [H.Context(0, max_keys=1 << 21, loc_bucket=0, **cfg),
          H.Context(0, max_keys=1 << 21, loc_bucket=1, **cfg)]
    up = O.Updater(**cfg)
    rng = np.random.default_rng(17)
    for step in range(5):
        blk = D.synthetic(rows, 39, 2, binary=True, seed=90 + step)
        blk = D.RowBlock(blk.offs, _hot_ids(kind, rng, blk.nnz, step), None, blk.labels)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, None, blk.labels,
                                         push_cnt=(step < 2), want_pred=True)
        preds, progs = [], []
        for c in cs:
            pr = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
            H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 2), pred=pr)
            preds.append(pr.cpu().numpy().view(np.uint32))
            progs.append(H.progress(c))
        assert np.array_equal(preds[0], preds[1]), step
        assert progs[0]["loss"] == progs[1]["loss"] and progs[0]["auc"] == progs[1]["auc"], step
        assert abs(progs[1]["loss"] - loss) <= 1e-4 * abs(loss), (step, progs[1]["loss"], loss)
        assert abs(progs[1]["auc"] - _auc_expect(blk.labels, opred, auc)) <= 1e-4 * blk.size
    uniq, _, _ = O.localize(blk.offs, blk.ids)
    vs = [H.Store(c).pull(c.tensor(uniq, torch.int64)) for c in cs]
    assert np.array_equal(vs[0][1].cpu().numpy(), vs[1][1].cpu().numpy())
    assert np.array_equal(vs[0][0].cpu().numpy().view(np.uint32),
                          vs[1][0].cpu().numpy().view(np.uint32))
    st = [H.Store(c).stats() for c in cs]
    assert st[0]["n_keys"] == st[1]["n_keys"] == up.size()
    # the hot-key map actually placed batches (else the map's paths — lb_hot_bucket, the
    # continued runs, k_lb_out's skipped heads — would go untested).  Batch t takes
    # the map batch t - 2 built on the same lane workspace: batches 2, 3, 4 of five
    maps = H.prof_counts(cs[1])["lb_map_steps"]
    if kind == "one_hot" or (kind == "zipf" and rows >= 60000):
        assert maps == 3, maps
    for c in cs:
        c.close()


@pytest.mark.parametrize("d", [16, 128])
def test_cold_model_counters_vs_oracle(H, d):
    """A cold model: nearly every backward block has new w's and InitV requests.  The fused
    backward adds its {new_w, n_keys} counts to 32 striped lines (summed by k_step_finalize) and
    raises the InitV gate once; at V_dim 128 pass W leaves its blocks' counts for pass V to add
    (one-word atomics serialise).  The step's statistics must still equal
    SGDUpdater's: n_keys, new_w (sgd_updater.cc: w leaving / returning to zero under l1) and the
    rand_r seed after every InitV draw — over enough keys that every stripe is used."""
    cfg = dict(V_dim=d, V_threshold=0, l1=0.5, lr=.1, V_lr=.02)
    c = H.Context(0, max_keys=1 << 20, **cfg)
    up = O.Updater(**cfg)
    for step in range(3):
        blk = D.synthetic(6000, 39, 1 << 20, binary=True, seed=400 + step)
        loss, auc, opred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels,
                                         push_cnt=(step < 2), want_pred=True)
        pred = torch.zeros(blk.size, dtype=torch.float32, device=c.device)
        H.train_step(c, H.DeviceRowBlock(c, blk), H.kTraining, push_cnt=(step < 2), pred=pred)
        H.progress(c)
        s = H.Store(c).stats()
        assert s["n_keys"] == up.size(), step
        assert s["new_w"] == int(up.new_w), (step, s["new_w"], up.new_w)
        assert s["seed"] == up.seed, step
        assert np.allclose(pred.cpu().numpy(), opred, rtol=1e-4, atol=1e-6), step
    c.close()
