"""The owner-computes split of FM over key-range shards (csrc/split.hip, dist.split_step)
against the single reference updater on the concatenated batch (one N-GPU step
== one reference step, sgd_learner.cc:201-317, on the N batches in rank order), and at N = 1
against the fused single-GPU step bit for bit.  N shards live on the one GPU and exchange
through LoopbackComm.  Bars: predictions within 1e-5 relative (the forward's sums are regrouped
by owner), loss 1e-5, model values 1e-5; keys, V rows, rand_r state and new_w exact."""
import numpy as np
import pytest
import torch

from difacto_amd import data as D
from oracle import dist_oracle as DO
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def close(a, b, rtol=1e-5):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    floor = 1e-6 * max(1.0, float(np.max(np.abs(b))) if b.size else 1.0)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(a), np.abs(b)) + floor)


CFGS = {
    "fm_v8": dict(V_dim=8, V_threshold=2, lr=0.1, V_lr=0.05, l1=0.2, seed=13),
    "fm_v16": dict(V_dim=16, V_threshold=0, lr=0.1, V_lr=0.01, l1=0.0, seed=3),
    "fm_v5_odd": dict(V_dim=5, V_threshold=2, lr=0.05, l1=0.1, seed=11),
    "logit": dict(V_dim=0, lr=0.2, l1=0.05),
    "fm_v64": dict(V_dim=64, V_threshold=0, lr=0.05, V_lr=0.01, l1=0.0, seed=9),
}


def _run(N, kw, steps, rows=400, nnz=12, key_space=6000, jobs=None, empty=()):
    """N loopback shards through dist.split_step against the oracle's single updater on the
    concatenated batches; returns the contexts (closed by the caller) and the oracle"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    one = O.Updater(**kw)
    seen = []
    for s in range(steps):
        step = [D.synthetic(0 if (s, r) in empty else rows, nnz, key_space,
                            binary=(r % 2 == 0), seed=900 + 37 * s + r, ragged=(s == 2))
                for r in range(N)]
        job = jobs[s] if jobs else H.kTraining
        push = s < 2
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        preds = [torch.zeros(max(step[r].size, 1), dtype=torch.float32, device=ctxs[r].device)
                 for r in range(N)]
        DI.split_step(shards, dbs, comm, job, push_cnt=push, preds=preds)
        cat = D.concat(step)
        loss, _, opred = one.train_step(cat.offs, cat.ids, cat.vals, cat.labels, push_cnt=push,
                                        train=job == H.kTraining, want_pred=True)
        got = 0.0
        b0 = 0
        for r in range(N):
            B = step[r].size
            p = preds[r][:B].cpu().numpy()
            assert close(p, opred[b0:b0 + B]), (N, s, r)
            pr = H.progress(ctxs[r])
            assert pr["nrows"] == B
            got += pr["loss"]
            if B:
                want_auc = (O.auc_stable_ties(step[r].labels, p) if O.has_ties(p)
                            else O.auc(step[r].labels, p))
                assert pr["auc"] == pytest.approx(want_auc, rel=1e-4, abs=1e-6), (N, s, r)
            b0 += B
        assert got == pytest.approx(loss, rel=1e-5), (N, s)
        seen.append(cat)
    return ctxs, one, seen


def _check_model(ctxs, one, seen, N, rtol=1e-5):
    from difacto_amd import hotpath as H
    for c in ctxs:
        c.sync()
    stats = [H.Store(c).stats() for c in ctxs]
    assert sum(st["n_keys"] for st in stats) == one.size()
    assert sum(st["new_w"] for st in stats) == one.new_w
    assert all(st["seed"] == one.seed for st in stats)
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0] for b in seen]))
    n_v = 0
    for k in keys[:: max(1, len(keys) // 600)]:
        g = int(DO.owner_of(np.array([k], np.uint64), N)[0])
        e = one.entry(k)
        got = H.Store(ctxs[g]).entry(k)
        assert (got is None) == (e is None)
        if e is None:
            continue
        assert close(got[0], e[0], rtol), k
        assert (got[1] is None) == (e[1] is None), k
        if e[1] is not None:
            n_v += 1
            assert close(got[1], e[1], rtol), k
    return n_v


@pytest.mark.parametrize("N", [1, 2, 3, 8])
@pytest.mark.parametrize("name", ["fm_v8", "fm_v16", "fm_v5_odd", "logit"])
def test_split_equals_one_step_on_concatenated_batches(name, N):
    kw = CFGS[name]
    ctxs, one, seen = _run(N, kw, steps=5)
    n_v = _check_model(ctxs, one, seen, N)
    if kw.get("V_dim", 0) > 0:
        assert n_v > 0
    for c in ctxs:
        c.close()


def test_split_c4_shaped_eight_owners():
    """V_dim 64 over 8 owners, keys from a 2^30 space (C4's shape at test size)"""
    kw = CFGS["fm_v64"]
    ctxs, one, seen = _run(8, kw, steps=4, rows=300, nnz=39, key_space=1 << 30)
    assert _check_model(ctxs, one, seen, 8) > 0
    for c in ctxs:
        c.close()


def test_split_validation_and_empty_workers():
    """a validation step updates nothing; a worker with no rows still takes part"""
    from difacto_amd import hotpath as H
    kw = CFGS["fm_v8"]
    jobs = [H.kTraining, H.kTraining, H.kValidation, H.kTraining, H.kTraining]
    ctxs, one, seen = _run(3, kw, steps=5, jobs=jobs, empty={(1, 0), (3, 2), (4, 1)})
    assert _check_model(ctxs, one, seen, 3) > 0
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("name", ["fm_v16", "fm_v5_odd", "logit"])
def test_split_one_owner_equals_fused_step(name):
    """at N = 1 the owner's partial is the whole row: predictions, AUC and the model equal the
    fused single-GPU step (dfx_train_step) exactly, the loss to the order of its double sum"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    kw = CFGS[name]
    cs = H.Context(0, max_keys=1 << 16, **kw)
    cf = H.Context(0, max_keys=1 << 16, **kw)
    sh = [DI.Shard(cs, 1)]
    comm = DI.LoopbackComm(1)
    blocks = []
    for s in range(5):
        blk = D.synthetic(500, 20, 5000, binary=(s % 2 == 0), seed=77 + s, ragged=(s == 3))
        blocks.append(blk)
        ds, df = H.DeviceRowBlock(cs, blk), H.DeviceRowBlock(cf, blk)
        ps = torch.zeros(blk.size, dtype=torch.float32, device=cs.device)
        pf = torch.zeros(blk.size, dtype=torch.float32, device=cf.device)
        DI.split_step(sh, [ds], comm, H.kTraining, push_cnt=s < 2, preds=[ps])
        H.train_step(cf, df, H.kTraining, push_cnt=s < 2, pred=pf)
        assert np.array_equal(ps.cpu().numpy(), pf.cpu().numpy()), (name, s)
        a, b = H.progress(cs), H.progress(cf)
        # the double loss partials are summed over differently sized blocks
        assert a["loss"] == pytest.approx(b["loss"], rel=1e-12) and a["auc"] == b["auc"], (name, s)
    cs.sync()
    cf.sync()
    assert H.Store(cs).stats() == H.Store(cf).stats()
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0] for b in blocks]))
    for k in keys[::7]:
        a, b = H.Store(cs).entry(k), H.Store(cf).entry(k)
        assert (a is None) == (b is None)
        if a is None:
            continue
        assert np.array_equal(a[0], b[0]), k
        assert (a[1] is None) == (b[1] is None)
        if a[1] is not None:
            assert np.array_equal(a[1], b[1]), k
    cs.close()
    cf.close()


@pytest.mark.parametrize("N", [1, 3])
@pytest.mark.parametrize("name", ["fm_v16", "fm_v5_odd", "logit"])
def test_split_pipeline_equals_sync_steps(name, N):
    """SplitPipeline (the next step's partition, key exchange and owner Localizer on the
    Localizer lanes beside the current step's forward / backward) gives split_step's results
    bit for bit: predictions, progress and the model, over count-push, training and
    validation steps"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    kw = CFGS[name]
    jobs = [(H.kTraining, True), (H.kTraining, True), (H.kTraining, False),
            (H.kValidation, False), (H.kTraining, False), (H.kTraining, False),
            (H.kTraining, False)]
    runs = []
    for piped in (False, True):
        ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(N)]
        shards = [DI.Shard(c, N) for c in ctxs]
        comm = DI.LoopbackComm(N)
        pipe = DI.SplitPipeline(shards, comm) if piped else None
        live, preds_all = [], []
        for s, (job, cnt) in enumerate(jobs):
            step = [D.synthetic(300, 12, 5000, binary=(r % 2 == 0), seed=500 + 31 * s + r,
                                ragged=(s == 4)) for r in range(N)]
            dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
            preds = [torch.zeros(300, dtype=torch.float32, device=ctxs[r].device)
                     for r in range(N)]
            if piped:
                pipe.submit(dbs, job, push_cnt=cnt, preds=preds)
                live.append(dbs)
            else:
                DI.split_step(shards, dbs, comm, job, push_cnt=cnt, preds=preds)
            preds_all.append(preds)
        if piped:
            pipe.flush()
        for c in ctxs:
            c.sync()
        out = {"preds": [[p.cpu().numpy() for p in ps] for ps in preds_all],
               "prog": [H.progress(c) for c in ctxs],
               "stats": [H.Store(c).stats() for c in ctxs]}
        runs.append((ctxs, out))
    (ca, a), (cb, b) = runs
    for s in range(len(jobs)):
        for r in range(N):
            assert np.array_equal(a["preds"][s][r], b["preds"][s][r]), (name, N, s, r)
    assert a["stats"] == b["stats"]
    for pa, pb in zip(a["prog"], b["prog"]):
        assert pa["nrows"] == pb["nrows"] and pa["auc"] == pb["auc"]
        assert pa["loss"] == pytest.approx(pb["loss"], rel=1e-12)
    for c in ca + cb:
        c.close()


@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("N", [1, 3])
@pytest.mark.parametrize("name", ["fm_v16", "fm_v5_odd", "logit"])
def test_split_store_cpp_equals_python_schedule(name, N, pipelined):
    """the C++ driver (libdfx_dist.so, host/split_host.cc, loopback transport) gives
    split_step's results bit for bit: predictions, progress and the model, over count-push,
    training and validation steps, mixed binary / valued workers and an empty worker"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    kw = CFGS[name]
    jobs = [(H.kTraining, True), (H.kTraining, True), (H.kTraining, False),
            (H.kValidation, False), (H.kTraining, False), (H.kTraining, False),
            (H.kTraining, False)]
    runs, blocks = [], []
    for cpp in (False, True):
        ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(N)]
        shards = [DI.Shard(c, N) for c in ctxs]
        comm = DI.LoopbackComm(N)
        store = DI.SplitStore(shards, pipelined=pipelined) if cpp else None
        preds_all = []
        for s, (job, cnt) in enumerate(jobs):
            step = [D.synthetic(0 if (s == 5 and r == 1) else 300, 12, 5000,
                                binary=(r % 2 == 0), seed=700 + 31 * s + r, ragged=(s == 4))
                    for r in range(N)]
            if not cpp:
                blocks += step
            dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
            preds = [torch.zeros(300, dtype=torch.float32, device=ctxs[r].device)
                     for r in range(N)]
            if cpp:
                store.submit(dbs, job, push_cnt=cnt, preds=preds)
            else:
                DI.split_step(shards, dbs, comm, job, push_cnt=cnt, preds=preds)
            preds_all.append(preds)
        if cpp:
            store.flush()
        for c in ctxs:
            c.sync()
        out = {"preds": [[p.cpu().numpy() for p in ps] for ps in preds_all],
               "prog": [H.progress(c) for c in ctxs],
               "stats": [H.Store(c).stats() for c in ctxs]}
        if cpp:
            store.close()
        runs.append((ctxs, out))
    (ca, a), (cb, b) = runs
    for s in range(len(jobs)):
        for r in range(N):
            assert np.array_equal(a["preds"][s][r], b["preds"][s][r]), (name, N, s, r)
    assert a["stats"] == b["stats"]
    for pa, pb in zip(a["prog"], b["prog"]):
        assert pa["nrows"] == pb["nrows"] and pa["auc"] == pb["auc"]
        assert pa["loss"] == pytest.approx(pb["loss"], rel=1e-12)
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0] for b in blocks if b.size]))
    for k in keys[::max(1, len(keys) // 150)]:
        for r in range(N):
            ea, eb = H.Store(ca[r]).entry(k), H.Store(cb[r]).entry(k)
            assert (ea is None) == (eb is None)
            if ea is not None:
                assert np.array_equal(ea[0], eb[0])
                assert (ea[1] is None) == (eb[1] is None)
                if ea[1] is not None:
                    assert np.array_equal(ea[1], eb[1])
    for c in ca + cb:
        c.close()


@pytest.mark.parametrize("N", [1, 3])
@pytest.mark.parametrize("name", ["fm_v16", "fm_v5_odd", "fm_v8", "logit"])
def test_split_store_stale_matches_oracle(name, N):
    """the 1-step-stale schedule of the C++ driver (SplitStore(stale=True): step t+1's owner
    forward before step t's backward, the exchanges beside the other step's compute) against
    oracle/dist_oracle.SplitStaleOracle: predictions one step stale, each update's gradient from
    its stale forward with the V term read at update time; count-push, training and validation
    steps, mixed binary / valued workers, an empty worker.  Bars as the synchronous split's:
    predictions, loss and model values within 1e-5; keys, rand_r state and new_w exact."""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    kw = CFGS[name]
    jobs = [(H.kTraining, True), (H.kTraining, True), (H.kTraining, False),
            (H.kValidation, False), (H.kTraining, False), (H.kTraining, False),
            (H.kTraining, False)]
    ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    store = DI.SplitStore(shards, stale=True)
    so = DO.SplitStaleOracle(N, **kw)
    got, want, seen, live = [], [], [], []
    for s, (job, cnt) in enumerate(jobs):
        step = [D.synthetic(0 if (s == 5 and r == 1) else 300, 12, 5000,
                            binary=(r % 2 == 0), seed=500 + 31 * s + r, ragged=(s == 4))
                for r in range(N)]
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        preds = [torch.zeros(300, dtype=torch.float32, device=ctxs[r].device) for r in range(N)]
        store.submit(dbs, job, push_cnt=cnt, preds=preds)
        live.append(dbs)
        got.append(preds)
        want.append(so.submit(step, push_cnt=cnt, train=job == H.kTraining))
        seen.append(D.concat(step))
    store.flush()
    so.flush()
    for c in ctxs:
        c.sync()
    loss = [0.0] * N
    for s in range(len(jobs)):
        for r in range(N):
            B = len(want[s][r][2])
            assert close(got[s][r][:B].cpu().numpy(), want[s][r][2]), (name, N, s, r)
            loss[r] += want[s][r][0]
    for r in range(N):
        assert H.progress(ctxs[r])["loss"] == pytest.approx(loss[r], rel=1e-5)
    n_v = _check_model(ctxs, so.one, seen, N)
    if kw.get("V_dim", 0) > 0:
        assert n_v > 0
    store.close()
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("pipelined", [False, True])
def test_split_store_marks(pipelined):
    """the C++ driver's phase events: every marked step times every main-stream phase"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    kw = CFGS["fm_v16"]
    ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(2)]
    store = DI.SplitStore([DI.Shard(c, 2) for c in ctxs], pipelined=pipelined)
    store.set_marks(range(DI.SplitStore.MARKS))
    for s in range(4):
        step = [D.synthetic(2000, 20, 50000, seed=40 + 2 * s + r) for r in range(2)]
        store.submit([H.DeviceRowBlock(ctxs[r], step[r]) for r in range(2)], H.kTraining,
                     push_cnt=s == 0)
    store.flush()
    m = store.take_marks()
    assert all(n == 4 for _, n in m.values()), m
    assert m["owner_forward"][0] > 0 and m["owner_backward"][0] > 0, m
    assert all(n == 0 for _, n in store.take_marks().values())
    store.close()
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("name", ["fm_v16", "fm_v5_odd"])
def test_split_store_slices_equal(name):
    """the C++ driver's sliced step (SetSlices: slice h's partial exchange beside slice h+1's
    owner forward, its row gather beside the next combine, on streams of their own) gives the
    unsliced step's results bit for bit, for slice counts that do and do not divide the padded
    rows, over count-push / training / validation steps and ragged, uneven workers"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N = 3
    kw = CFGS[name]
    jobs = [(H.kTraining, True), (H.kTraining, False), (H.kValidation, False),
            (H.kTraining, False), (H.kTraining, False)]
    outs = []
    for K in (1, 2, 5):
        ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(N)]
        shards = [DI.Shard(c, N) for c in ctxs]
        store = DI.SplitStore(shards, pipelined=True)
        store.set_slices(K)
        preds_all = []
        for s, (job, cnt) in enumerate(jobs):
            rows = [1300, 700 if s != 3 else 0, 1299]
            step = [D.synthetic(rows[r], 12, 20000, binary=(r % 2 == 0), seed=900 + 31 * s + r,
                                ragged=(s == 1)) for r in range(N)]
            dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
            preds = [torch.zeros(1300, dtype=torch.float32, device=ctxs[r].device)
                     for r in range(N)]
            store.submit(dbs, job, push_cnt=cnt, preds=preds)
            preds_all.append(preds)
        store.flush()
        for c in ctxs:
            c.sync()
        outs.append({"preds": [[p.cpu().numpy() for p in ps] for ps in preds_all],
                     "prog": [H.progress(c) for c in ctxs],
                     "stats": [H.Store(c).stats() for c in ctxs]})
        store.close()
        for c in ctxs:
            c.close()
    a = outs[0]
    for b in outs[1:]:
        for s in range(len(jobs)):
            for r in range(N):
                assert np.array_equal(a["preds"][s][r], b["preds"][s][r]), (name, s, r)
        assert a["stats"] == b["stats"]
        for pa, pb in zip(a["prog"], b["prog"]):
            assert pa["nrows"] == pb["nrows"] and pa["auc"] == pb["auc"]
            assert pa["loss"] == pb["loss"]
