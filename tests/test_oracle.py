"""Pins the CPU restatement (oracle/) against the reference's own known answers.

Every expected value below is read from tests/golden/reference_known_answers.json, which
transcribes the reference's gtest assertions (file:line in that JSON).
"""
import os

import numpy as np
import pytest

from difacto_amd import data as D
from oracle import oracle as O


def _rev(a):
    return np.array([O.reverse_bytes(int(x)) for x in a], dtype=np.uint64)


def test_reverse_bytes_involution():
    # tests/cpp/localizer_test.cc:56-63
    mx = (1 << 64) - 1
    n = 1000
    for i in range(n):
        j = (mx // n) * i
        assert O.reverse_bytes(O.reverse_bytes(j)) == j


def test_localizer_base(rcv1, known):
    k = known["localizer_base"]
    uniq, cnt, col = O.localize(rcv1.offs, rcv1.ids)
    assert int(_rev(uniq).sum()) == k["sum_uidx"]
    assert float(cnt.sum()) == k["sum_freq"]
    assert np.all(np.diff(uniq.astype(np.float64)) >= 0) and np.all(uniq[1:] != uniq[:-1])
    # compacted block keeps every nnz: the remapped column points at its own key
    assert np.array_equal(uniq[col], _rev_keys(rcv1.ids))


def _rev_keys(ids, max_index=(1 << 64) - 1):
    return np.array([O.reverse_bytes(int(i) % max_index) for i in ids], dtype=np.uint64)


def test_localizer_hash(rcv1, known):
    k = known["localizer_hash1000"]
    uniq, cnt, col = O.localize(rcv1.offs, rcv1.ids, max_index=k["max_index"])
    assert int(_rev(uniq).sum()) == k["sum_uidx"]
    assert float(cnt.sum()) == k["sum_freq"]


def _fm_weights(uidx, d):
    U = len(uidx)
    W = np.zeros(U * (d + 1), np.float32)
    wp = (np.arange(U) * (d + 1)).astype(np.int32)
    for i in range(U):
        W[i * (d + 1)] = uidx[i] / 5e4
        for j in range(1, d + 1):
            W[i * (d + 1) + j] = uidx[i] * j / 5e5
    return W, wp, wp + 1


def test_fmloss_nov(rcv1, known):
    k = known["fmloss_nov"]
    uniq, _, col = O.localize(rcv1.offs, rcv1.ids)
    w = (_rev(uniq) / 5e4).astype(np.float32)
    pred = O.fm_predict(rcv1.offs, col, rcv1.vals, w, None, None, 0)
    assert abs(O.evaluate(rcv1.labels, pred) - k["objv"]) < k["objv_tol"]
    g = O.fm_calcgrad(rcv1.offs, col, rcv1.vals, rcv1.labels, None, w, None, None, len(uniq), 0,
                      pred)
    assert abs(float((g.astype(np.float64) ** 2).sum()) - k["grad_norm2"]) < k["grad_tol"]


def test_fmloss_hasv(rcv1, known):
    k = known["fmloss_hasv"]
    d = k["V_dim"]
    uniq, _, col = O.localize(rcv1.offs, rcv1.ids)
    W, wp, vp = _fm_weights(_rev(uniq), d)
    pred = O.fm_predict(rcv1.offs, col, rcv1.vals, W, wp, vp, d)
    assert abs(O.evaluate(rcv1.labels, pred) - k["objv"]) < k["objv_tol"]
    g = O.fm_calcgrad(rcv1.offs, col, rcv1.vals, rcv1.labels, None, W, wp, vp, len(uniq), d, pred)
    assert abs(float((g.astype(np.float64) ** 2).sum()) - k["grad_norm2"]) < k["grad_tol"]


def test_stale_calcgrad_equals_calcgrad_on_one_model(rcv1, known):
    """oracle.cc CalcGradStale (the split store's stale schedule) with the forward's and the
    backward's model the same is CalcGrad term for term; with a different backward model only
    the diag(XXp) V term moves"""
    d = known["fmloss_hasv"]["V_dim"]
    uniq, _, col = O.localize(rcv1.offs, rcv1.ids)
    W, wp, vp = _fm_weights(_rev(uniq), d)
    pred = O.fm_predict(rcv1.offs, col, rcv1.vals, W, wp, vp, d)
    g = O.fm_calcgrad(rcv1.offs, col, rcv1.vals, rcv1.labels, None, W, wp, vp, len(uniq), d, pred)
    gs = O.fm_calcgrad_stale(rcv1.offs, col, rcv1.vals, rcv1.labels, None, W, vp, W, wp, vp,
                             len(uniq), d, pred)
    assert np.array_equal(g.view(np.uint32), gs.view(np.uint32))
    W2 = W.copy()
    W2[vp[vp >= 0][:, None] + np.arange(d)] *= 2  # every V doubled, w unchanged
    g2 = O.fm_calcgrad_stale(rcv1.offs, col, rcv1.vals, rcv1.labels, None, W, vp, W2, wp, vp,
                             len(uniq), d, pred)
    assert np.array_equal(g2[wp], g[wp])
    assert not np.array_equal(g2, g)


def test_sgd_learner_basic(rcv1, known):
    k = known["sgd_learner_basic"]
    kw = k["kwargs"]
    up = O.Updater(V_dim=kw["V_dim"], l2=kw["l2"], l1=kw["l1"], lr=kw["lr"])
    for ep, want in enumerate(k["objv"]):
        loss, _ = up.train_step(rcv1.offs, rcv1.ids, rcv1.vals, rcv1.labels)
        assert abs(loss - want) < k["tol"], (ep, loss, want)


def test_rand_r_is_glibc_lcg():
    """InitV's rand_r (sgd_updater.cc:148): 3 LCG steps per call, a=1103515245, c=12345."""
    seq, _ = O.rand_r_seq(0, 50)
    s = 0
    for want in seq:
        r = 0
        for shift, mod in ((0, 2048), (10, 1024), (10, 1024)):
            s = (s * 1103515245 + 12345) & 0xFFFFFFFF
            r = (r << shift) ^ ((s >> 16) % mod)
        assert r == want


def test_save_load_roundtrip(rcv1, tmp_path):
    up = O.Updater(V_dim=4, V_threshold=2, lr=.1, V_lr=.01, l1=.1)
    for ep in range(3):
        up.train_step(rcv1.offs, rcv1.ids, rcv1.vals, rcv1.labels, push_cnt=(ep == 0))
    path = str(tmp_path / "model")
    up.save(path, True)
    up2 = O.Updater(V_dim=4)
    up2.load(path)
    uniq, _, _ = O.localize(rcv1.offs, rcv1.ids)
    a, la = up.get(uniq)
    b, lb = up2.get(uniq)
    assert np.array_equal(a, b) and np.array_equal(la, lb)


def test_auc_tie_convention_agrees_without_ties():
    rng = np.random.default_rng(5)
    for n in (10, 100, 5000):
        label = np.where(rng.random(n) < 0.3, 1.0, -1.0).astype(np.float32)
        pred = rng.permutation(np.linspace(-3, 3, n)).astype(np.float32)
        assert not O.has_ties(pred)
        assert abs(O.auc_stable_ties(label, pred) - O.auc(label, pred)) <= 1e-4 * n


@pytest.mark.parametrize("nt", [1, 3, 8])
def test_cpu_ref_matches_oracle(nt):
    """oracle/cpu_ref.cc (the CPU baseline: the reference's threading) computes what the pinned
    restatement computes: predictions bitwise for any thread count (row- and column-range
    splits keep every sum's order), the same model size and rand_r state, loss within 1e-4 (the
    reference sums Evaluate as a float reduction), AUC*n equal; also through the two-thread
    IterateData pipeline"""
    from oracle import cpu_ref as C
    cfg = dict(V_dim=8, V_threshold=2, l1=0.5, lr=.1, V_lr=.05)
    up = O.Updater(**cfg)
    ref = C.CpuRef(nt, **cfg)
    for s in range(4):
        blk = D.synthetic(1500, 20, 1 << 12, seed=80 + s, binary=(s % 2 == 0), ragged=(s == 3))
        l1, a1, p1 = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels, push_cnt=s < 2,
                                   want_pred=True)
        l2, a2, p2 = ref.step(blk, push_cnt=s < 2, want_pred=True)
        assert np.array_equal(p1, p2), s
        assert abs(l1 - l2) <= 1e-4 * abs(l1) and (a1 == a2 or O.has_ties(p1)), s
    assert up.size() == ref.size() and up.seed == ref.seed
    blocks = [D.synthetic(800, 20, 1 << 12, seed=90 + s) for s in range(5)]
    tot = 0.0
    for b in blocks:
        tot += up.train_step(b.offs, b.ids, b.vals, b.labels)[0]
    dt, loss, _, n = ref.iterate(blocks)
    assert n == 4000 and dt > 0 and abs(loss - tot) <= 1e-4 * abs(tot)
    assert up.size() == ref.size() and up.seed == ref.seed
    ref.close()


def test_device_expf_equals_glibc():
    """csrc/expf.h (glibc's expf restated for the device: CalcGrad's p, fm_loss.h:159-164)
    equals the host's expf bit for bit on a sample of every 97th float bit pattern (the full
    2^32 sweep: `build/expf_check 1`, 0 differences)"""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "expf_check")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "build/expf_check"], cwd=root)
    r = subprocess.run([exe, "97"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("0 of "), r.stdout
