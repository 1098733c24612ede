"""The key-range-sharded store's device phases (dfx_dist_*, through the C-ABI) against the
sharded oracle (oracle/dist_oracle.py: N restated SGDUpdater servers).  N shards live on the
one GPU of the test box and exchange through LoopbackComm (device copies); the
torch.distributed exchange itself is covered by tests/test_dist.py (gloo, world_size 2).
Bars as in test_gpu_parity.py: predictions / state within 1e-5 relative, loss within 1e-4;
InitV seeds, V-row counts and new_w exact."""
import numpy as np
import pytest
import torch

from difacto_amd import data as D
from oracle import dist_oracle as DO
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    floor = 1e-6 * max(1.0, float(np.max(np.abs(b))) if b.size else 1.0)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(a), np.abs(b)) + floor)


CFGS = {
    "fm_v4": (3, dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.5, l2=0.01, seed=7)),
    "fm_v16": (2, dict(V_dim=16, V_threshold=0, lr=0.1, V_lr=0.01, l1=0.0, seed=3)),
    "fm_v5_odd": (4, dict(V_dim=5, V_threshold=2, lr=0.05, l1=0.1, seed=11)),
    "logit": (2, dict(V_dim=0, lr=0.2, l1=0.05)),
    "fm_v8_n6": (6, dict(V_dim=8, V_threshold=1, lr=0.1, V_lr=0.02, l1=0.2, seed=5)),
    # C4-shaped: V_dim 64 over 8 shards (keys drawn from 2^30 in _batches when V_dim == 64)
    "fm_v64_n8": (8, dict(V_dim=64, V_threshold=0, lr=0.05, V_lr=0.01, l1=0.0, seed=9)),
}


def _batches(nranks, steps, rows=300, nnz=8, key_space=3000, seed=0):
    if nranks == 8:  # the C4-shaped case: a 2^30 key space, few repeats
        key_space = 1 << 30
    return [[D.synthetic(rows, nnz, key_space, binary=(r % 2 == 0), seed=seed + 131 * s + r,
                         ragged=(s == 2)) for r in range(nranks)] for s in range(steps)]


def _oracle(N, kw, agg, stale=False):
    if stale:
        return DO.StaleOracle(N, agg=agg, **kw)
    return DO.AggOracle(N, **kw) if agg == "sum" else DO.ShardedOracle(N, **kw)


def _check_servers(name, ctxs, so, keys, N, agg):
    """every server's counters and a sample of its entries against the oracle: per server
    (push_agg=ranks: N SGDUpdaters) or against the one updater the servers together restate
    (push_agg=sum: shared rand_r stream, keys split by owner)"""
    from difacto_amd import hotpath as H
    n_v = 0
    stats = [H.Store(c).stats() for c in ctxs]
    if agg == "sum":
        one = so.up[0]
        assert sum(st["n_keys"] for st in stats) == one.size(), name
        assert sum(st["new_w"] for st in stats) == one.new_w, name
        for g in range(N):
            assert stats[g]["seed"] == one.seed, (name, g)
    for g in range(N):
        up = so.up[0] if agg == "sum" else so.up[g]
        if agg != "sum":
            assert stats[g]["seed"] == up.seed, (name, g)
            assert stats[g]["n_keys"] == up.size(), (name, g)
            assert stats[g]["new_w"] == up.new_w, (name, g)
        own = keys[DO.owner_of(keys, N) == g]
        for k in own[:: max(1, len(own) // 150)]:
            e = up.entry(k)
            got = H.Store(ctxs[g]).entry(k)
            assert (got is None) == (e is None)
            if e is None:
                continue
            assert close(got[0], e[0]), (name, g, k)
            assert (got[1] is None) == (e[1] is None), (name, g, k)
            if e[1] is not None:
                n_v += 1
                assert close(got[1], e[1]), (name, g, k)
    return n_v


@pytest.mark.parametrize("agg", ["sum", "ranks"])
@pytest.mark.parametrize("name", list(CFGS))
def test_sharded_loopback_matches_sharded_oracle(name, agg):
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = CFGS[name]
    ctxs = [H.Context(0, max_keys=1 << 15, push_agg=agg, **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    so = _oracle(N, kw, agg)
    batches = _batches(N, 5)
    for s, step in enumerate(batches):
        push = s < 3
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        preds = [torch.zeros(step[r].size, dtype=torch.float32, device=ctxs[r].device)
                 for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=push, preds=preds)
        out = so.step(step, push_cnt=push)
        for r in range(N):
            p = preds[r].cpu().numpy()
            assert close(p, out[r][2]), (name, s, r)
            pr = H.progress(ctxs[r])
            assert pr["nrows"] == step[r].size
            assert pr["loss"] == pytest.approx(out[r][0], rel=1e-4)
            want_auc = (O.auc_stable_ties(step[r].labels, out[r][2])
                        if O.has_ties(out[r][2]) else out[r][1])
            assert pr["auc"] == pytest.approx(want_auc, rel=1e-4, abs=1e-6)
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0]
                                     for step in batches for b in step]))
    n_v = _check_servers(name, ctxs, so, keys, N, agg)
    if kw.get("V_dim", 0) > 0:
        assert n_v > 0
    for c in ctxs:
        c.sync()
        c.close()


PIPE_JOBS = [(3, True), (3, True), (3, False), (4, False), (3, False), (3, False)]


@pytest.mark.parametrize("agg", ["sum", "ranks"])
@pytest.mark.parametrize("name", ["fm_v4", "fm_v16", "logit", "fm_v8_n6", "fm_v64_n8"])
def test_sharded_pipeline_matches_stale_oracle(name, agg):
    """the pipelined schedule (two step slots in flight, Localizer lane ahead, push of step t
    after the pull of step t+1) against oracle/dist_oracle.StaleOracle"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = CFGS[name]
    ctxs = [H.Context(0, max_keys=1 << 15, push_agg=agg, **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    pipe = DI.ShardedPipeline(shards, DI.LoopbackComm(N))
    so = _oracle(N, kw, agg, stale=True)
    batches = _batches(N, len(PIPE_JOBS))
    live, got, want = [], [], []  # batches stay alive until the pipeline is flushed
    for s, (step, (job, cnt)) in enumerate(zip(batches, PIPE_JOBS)):
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        preds = [torch.zeros(step[r].size, dtype=torch.float32, device=ctxs[r].device)
                 for r in range(N)]
        pipe.submit(dbs, job, push_cnt=cnt, preds=preds)
        live.append(dbs)
        got.append(preds)
        want.append(so.submit(step, push_cnt=cnt, train=job == 3))
    pipe.flush()
    so.flush()
    for s in range(len(PIPE_JOBS)):
        for r in range(N):
            assert close(got[s][r].cpu().numpy(), want[s][r][2]), (name, s, r)
    for r in range(N):
        pr = H.progress(ctxs[r])
        assert pr["nrows"] == sum(step[r].size for step in batches)
        assert pr["loss"] == pytest.approx(sum(w[r][0] for w in want), rel=1e-4)
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0]
                                     for step in batches for b in step]))
    for c in ctxs:
        c.sync()
    n_v = _check_servers(name, ctxs, so, keys, N, agg)
    if kw.get("V_dim", 0) > 0:
        assert n_v > 0
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("N", [2, 3, 8])
def test_sharded_sum_equals_one_step_on_concatenated_batches(N):
    """SURVEY.md §8(e)'s parity claim, pinned to the single-GPU reference semantics: with
    push_agg=sum, one N-GPU step equals one reference local step (the oracle's SGDUpdater +
    FMLoss, sgd_learner.cc:201-317) on the concatenation of the N batches in rank order.  Loss
    is additive over rows; the model keys, V rows, rand_r state and new_w are exact; values
    differ only by the order the gradient sums run in (per worker, then across workers), so
    they are compared at 1e-4 — and at north_star's 1e-5 for the keys no step ever saw in two
    workers' batches, whose sums no per-worker pre-summing reorders."""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    kw = dict(V_dim=8, V_threshold=2, lr=0.1, V_lr=0.05, l1=0.2, seed=13)
    ctxs = [H.Context(0, max_keys=1 << 16, push_agg="sum", **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    one = O.Updater(**kw)
    multi = set()  # keys some step saw in two or more workers' batches
    for s in range(6):
        step = [D.synthetic(400, 12, 6000, binary=(r % 2 == 0), seed=900 + 37 * s + r)
                for r in range(N)]
        push = s < 2
        seen = np.concatenate([np.unique(O.localize(b.offs, b.ids)[0]) for b in step])
        kk, nk = np.unique(seen, return_counts=True)
        multi.update(int(k) for k in kk[nk > 1])
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=push)
        cat = D.concat(step)
        loss, _ = one.train_step(cat.offs, cat.ids, cat.vals, cat.labels, push_cnt=push)
        got = sum(H.progress(c)["loss"] for c in ctxs)
        assert got == pytest.approx(loss, rel=1e-5), (N, s)
    stats = [H.Store(c).stats() for c in ctxs]
    assert sum(st["n_keys"] for st in stats) == one.size()
    assert sum(st["new_w"] for st in stats) == one.new_w
    assert all(st["seed"] == one.seed for st in stats)
    cat_keys = np.unique(O.localize(cat.offs, cat.ids)[0])
    n_v = n_single = 0
    mg, me = [], []  # the reordered keys' values, as one vector (north_star's 1e-5 as a norm)
    for k in cat_keys:
        g = int(DO.owner_of(np.array([k], np.uint64), N)[0])
        e = one.entry(k)
        got = H.Store(ctxs[g]).entry(k)
        assert (got is None) == (e is None)
        if e is None:
            continue
        rt = 1e-4 if int(k) in multi else 1e-5
        n_single += int(k) not in multi
        assert close(got[0], e[0], rtol=rt), k
        assert (got[1] is None) == (e[1] is None), k
        if int(k) in multi:
            mg.append(np.ravel(got[0]).astype(np.float64))
            me.append(np.ravel(e[0]).astype(np.float64))
        if e[1] is not None:
            n_v += 1
            assert close(got[1], e[1], rtol=rt), k
            if int(k) in multi:
                mg.append(np.ravel(got[1]).astype(np.float64))
                me.append(np.ravel(e[1]).astype(np.float64))
    if mg:
        a, b = np.concatenate(mg), np.concatenate(me)
        assert np.linalg.norm(a - b) <= 1e-5 * np.linalg.norm(b), np.linalg.norm(a - b)
    # (at N = 2 about a tenth of the last step's keys never met in two batches)
    assert n_v > 0 and (n_single > 0 or N > 2), (n_v, n_single, len(cat_keys))
    for c in ctxs:
        c.close()


def test_sharded_save_load_parts(tmp_path):
    """each server saves its part as <prefix>_part-<rank> (sgd_learner.h:65-69) in the
    reference's SGDUpdater::Save format: the oracle server loads it back to its own state, and
    fresh shards loading the parts continue training exactly like the original ones"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = CFGS["fm_v4"]
    ctxs = [H.Context(0, max_keys=1 << 15, push_agg="ranks", **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    so = DO.ShardedOracle(N, **kw)
    batches = _batches(N, 4)
    for s, step in enumerate(batches[:3]):
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=s < 2)
        so.step(step, push_cnt=s < 2)
    prefix = tmp_path / "model"
    for r in range(N):
        shards[r].save(prefix, r, save_aux=True)
        assert (tmp_path / ("model_part-%d" % r)).exists()
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0]
                                     for step in batches for b in step]))
    for g in range(N):
        up = O.Updater(**kw)
        up.load(DI.model_name(prefix, g))
        n_saved = 0
        for k in keys[DO.owner_of(keys, N) == g]:
            a, b = up.entry(k), so.up[g].entry(k)
            if a is None:  # Save skips empty entries (w == 0, no V; sgd_updater.h:35-48)
                assert b is None or (b[0][0] == 0 and b[1] is None)
                continue
            n_saved += 1
            assert close(a[0][:3], b[0][:3]) and (a[1] is None) == (b[1] is None)
            if a[1] is not None:
                assert close(a[1], b[1])
        assert n_saved == up.size() > 0
    # fresh shards from the parts: one more step agrees with the original shards
    ctx2 = [H.Context(0, max_keys=1 << 15, push_agg="ranks", **kw) for _ in range(N)]
    sh2 = [DI.Shard(c, N) for c in ctx2]
    for r in range(N):
        sh2[r].load(prefix, r)
    step = batches[3]
    preds = []
    for cs, shs in ((ctxs, shards), (ctx2, sh2)):
        dbs = [H.DeviceRowBlock(cs[r], step[r]) for r in range(N)]
        pr = [torch.zeros(step[r].size, dtype=torch.float32, device=cs[r].device)
              for r in range(N)]
        DI.sharded_step(shs, dbs, comm, H.kValidation, preds=pr)
        preds.append([p.cpu().numpy() for p in pr])
    for r in range(N):
        assert np.array_equal(preds[0][r], preds[1][r])
    for c in ctxs + ctx2:
        c.sync()
        c.close()


@pytest.mark.parametrize("m", [1, 2, 5])
def test_sharded_load_into_other_rank_count(tmp_path, m):
    """a model saved by 3 servers loads into m servers: every server reads every part and keeps
    the keys it owns (dfx_store_load_part); each key lands on its new owner with the state
    the old one saved"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = CFGS["fm_v4"]
    ctxs = [H.Context(0, max_keys=1 << 15, **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    batches = _batches(N, 3)
    for s, step in enumerate(batches):
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=s < 2)
    prefix = tmp_path / "model"
    for r in range(N):
        shards[r].save(prefix, r, save_aux=True)
    new = [H.Context(0, max_keys=1 << 15, **kw) for _ in range(m)]
    for g in range(m):
        DI.Shard(new[g], m).load(prefix, g, saved_ranks=N)
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0]
                                     for step in batches for b in step]))
    total = 0
    for k in keys:
        old = H.Store(ctxs[DO.owner_of(np.array([k]), N)[0]]).entry(k)
        g = DO.owner_of(np.array([k]), m)[0]
        got = H.Store(new[g]).entry(k)
        for h in range(m):
            if h != g:
                assert H.Store(new[h]).entry(k) is None
        if old is None or (old[0][0] == 0 and old[1] is None):
            continue  # Save skips empty entries
        total += 1
        assert got is not None, k
        assert np.array_equal(got[0][:3], old[0][:3])
        assert (got[1] is None) == (old[1] is None)
        if got[1] is not None:
            assert np.array_equal(got[1], old[1])
    assert total > 0
    assert sum(H.Store(c).stats()["n_keys"] for c in new) == total
    for c in ctxs + new:
        c.sync()
        c.close()


def test_sharded_validation_does_not_update():
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = CFGS["fm_v4"]
    ctxs = [H.Context(0, max_keys=1 << 15, **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    step = _batches(N, 1)[0]
    dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
    DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=True)
    before = [H.Store(c).stats() for c in ctxs]
    DI.sharded_step(shards, dbs, comm, H.kValidation)
    after = [H.Store(c).stats() for c in ctxs]
    assert before == after
    for c in ctxs:
        c.sync()
        c.close()


def test_sharded_empty_shard_and_batch():
    """a rank with an empty batch, and ranks that own none of the step's keys"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = 4, dict(V_dim=4, V_threshold=0, lr=0.1, l1=0.0)
    ctxs = [H.Context(0, max_keys=1 << 12, push_agg="ranks", **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    so = DO.ShardedOracle(N, **kw)
    empty = D.RowBlock(np.zeros(1, np.uint64), np.zeros(0, np.uint64), None,
                       np.zeros(0, np.float32))
    # two keys only: most owners receive nothing
    tiny = D.RowBlock(np.array([0, 2, 3], np.uint64), np.array([5, 9, 5], np.uint64), None,
                      np.array([1, -1], np.float32))
    steps = [[tiny, empty, tiny, empty], [empty, empty, empty, tiny]]
    for s, step in enumerate(steps):
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=True)
        so.step(step, push_cnt=True)
    for g in range(N):
        st = H.Store(ctxs[g]).stats()
        assert st["seed"] == so.up[g].seed
        assert st["n_keys"] == so.up[g].size()
    for c in ctxs:
        c.sync()
        c.close()


def _mp_worker(rank, world, port, q, pipelined=False):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from difacto_amd import dist as DI
        from difacto_amd import hotpath as H
        _, kw = CFGS["fm_v4"]
        ctx = H.Context(0, max_keys=1 << 15, push_agg="ranks", **kw)
        shard = DI.Shard(ctx, world)
        comm = DI.TorchComm(device="cpu", stage_cpu=True)
        pipe = DI.ShardedPipeline([shard], comm) if pipelined else None
        preds, live = [], []
        for s, step in enumerate(_batches(world, 4)):
            db = H.DeviceRowBlock(ctx, step[rank])
            live.append(db)
            pred = torch.zeros(step[rank].size, dtype=torch.float32, device=ctx.device)
            if pipe:
                pipe.submit([db], H.kTraining, push_cnt=s < 2, preds=[pred])
            else:
                DI.sharded_step([shard], [db], comm, H.kTraining, push_cnt=s < 2, preds=[pred])
            preds.append(pred)
        if pipe:
            pipe.flush()
        ctx.sync()
        preds = [p.cpu().numpy() for p in preds]
        q.put((rank, preds, H.Store(ctx).stats()))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, True])
def test_sharded_two_processes_one_gpu(pipelined):
    """world_size 2 through torch.distributed with each process's shard on the GPU (the
    exchange staged through host memory over gloo, since RCCL needs a GPU per rank), in the
    synchronous and the pipelined schedule"""
    import socket
    import torch.multiprocessing as mp
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_mp_worker, args=(r, world, port, q, pipelined))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, preds, st = q.get(timeout=100)
            res[r] = (preds, st)
    finally:
        for p in procs:
            p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    _, kw = CFGS["fm_v4"]
    if pipelined:
        so = DO.StaleOracle(world, **kw)
        outs = [so.submit(step, push_cnt=s < 2) for s, step in enumerate(_batches(world, 4))]
        so.flush()
    else:
        so = DO.ShardedOracle(world, **kw)
        outs = [so.step(step, push_cnt=s < 2) for s, step in enumerate(_batches(world, 4))]
    for r in range(world):
        preds, st = res[r]
        for s in range(4):
            assert close(preds[s], outs[s][r][2]), (r, s)
        assert st["seed"] == so.up[r].seed
        assert st["n_keys"] == so.up[r].size()
        assert st["new_w"] == so.up[r].new_w


@pytest.mark.parametrize("collective,sync", [("split", False), ("split", True), ("a2a", False),
                                             ("a2a", True)])
def test_bench_two_ranks_gloo(collective, sync):
    """bench.py's multi-GPU path end to end under torchrun with 2 ranks (the driver's SCALE
    command, with the exchange staged through host memory over gloo since both ranks share
    the test box's GPU): one JSON line from rank 0, whole-job throughput over both ranks"""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # (--standalone: the launcher binds its rendezvous port itself — a port picked here and
    # closed again can be taken before the launcher binds it: EADDRINUSE)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--standalone", "--local-addr", "127.0.0.1", "bench.py", "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--batch", "20000", "--key-bits", "20",
           "--backend", "gloo", "--no-cpu-baseline", "--collective", collective] + (
               ["--sync"] if sync else [])
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["value"] > 0
    assert out["config"]["global_batch"] == 40000
    assert 0.3 < out["train_loss_per_row"] < 0.8 and 0.3 < out["train_auc"] < 0.7
    wl = out["config"]["workload"]
    if collective == "split":
        assert "owner-computes" in wl and ("Localizer lane" in wl) == (not sync)
    else:
        assert "all-to-all-v" in wl and ("bulk-synchronous" in wl) == sync
    main = collective + ("_sync" if sync else "_pipelined")
    assert set(out["collectives"]) == {main, "split_sync", "a2a_sync", "rsag_sync"}


@pytest.mark.timeout(240)
def test_sharded_eight_ranges_at_scale():
    """8 key-range servers, each with its table sized for its own range (1/8 of 2^24 keys),
    fed Criteo-shaped batches of 20,000 rows: every server's keys share their top 3 bits, so
    the ordered hash must place keys by their position inside the range (Table::range_mul) —
    with the plain top-bits hash one server's keys crowd into 1/8 of its table and each probe
    walks ~10^6 slots (this test then runs into its timeout).  Results against the sharded
    oracle: loss per shard within 1e-4, the model's key and V-row counts and seeds exact."""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, rows, kb = 8, 20_000, 24
    kw = dict(V_dim=16, V_threshold=0, lr=0.1, V_lr=0.01, l1=0.0, seed=3)
    ctxs = [H.Context(0, max_keys=(1 << kb) // N, max_vrows=(1 << kb) // N + 65536,
                      push_agg="ranks", **kw)
            for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    so = DO.ShardedOracle(N, **kw)
    for s in range(3):
        step = [D.synthetic(rows, 39, 1 << kb, seed=900 + 17 * s + r) for r in range(N)]
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        DI.sharded_step(shards, dbs, comm, H.kTraining, push_cnt=(s == 0))
        out = so.step(step, push_cnt=(s == 0))
        for r in range(N):
            pr = H.progress(ctxs[r])
            assert pr["loss"] == pytest.approx(out[r][0], rel=1e-4), (s, r)
    for g in range(N):
        st = H.Store(ctxs[g]).stats()
        assert st["n_keys"] == so.up[g].size() and st["seed"] == so.up[g].seed, g
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("name", ["fm_v4", "fm_v16", "logit", "fm_v64_n8"])
def test_rsag_step_matches_agg_oracle(name):
    """the north_star's literal schedule (dist.rsag_step: all-gather of keys -> union,
    union-indexed all-gather of records, reduce-scatter of union-indexed gradients and counts)
    against AggOracle — the same semantics as the all-to-all-v step with push_agg=sum"""
    from difacto_amd import dist as DI
    from difacto_amd import hotpath as H
    N, kw = CFGS[name]
    ctxs = [H.Context(0, max_keys=1 << 15, push_agg="sum", **kw) for _ in range(N)]
    shards = [DI.Shard(c, N) for c in ctxs]
    comm = DI.LoopbackComm(N)
    so = DO.AggOracle(N, **kw)
    batches = _batches(N, 5)
    for s, step in enumerate(batches):
        push = s < 3
        job = H.kValidation if s == 3 else H.kTraining
        dbs = [H.DeviceRowBlock(ctxs[r], step[r]) for r in range(N)]
        preds = [torch.zeros(step[r].size, dtype=torch.float32, device=ctxs[r].device)
                 for r in range(N)]
        DI.rsag_step(shards, dbs, comm, job, push_cnt=push, preds=preds)
        out = so.step(step, push_cnt=push, train=job == H.kTraining)
        for r in range(N):
            assert close(preds[r].cpu().numpy(), out[r][2]), (name, s, r)
            assert H.progress(ctxs[r])["loss"] == pytest.approx(out[r][0], rel=1e-4)
    keys = np.unique(np.concatenate([O.localize(b.offs, b.ids)[0]
                                     for step in batches for b in step]))
    n_v = _check_servers(name, ctxs, so, keys, N, "sum")
    if kw.get("V_dim", 0) > 0:
        assert n_v > 0
    for c in ctxs:
        c.sync()
        c.close()


def test_bench_spawns_its_ranks():
    """`bench.py --gpus 2` without a launcher starts its two ranks itself (one process per GPU;
    gloo here, as both share the test box's GPU) and reports them: n_gpus 2, whole-job
    throughput over both; a launcher whose WORLD_SIZE disagrees with --gpus is refused"""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--batch", "20000", "--key-bits", "20", "--backend", "gloo", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 40000 and out["value"] > 0
    bad = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1"], cwd=root,
                         capture_output=True, text=True, timeout=120,
                         env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr


@pytest.mark.parametrize("collective", ["split", "a2a"])
def test_bench_rccl_collectives_at_world_one(collective):
    """bench.py's sharded path with every exchange forced through RCCL at world size 1 (the
    count all-to-all, the key / record / partial all-to-all-v, the all-gathers) gives the same
    training as the same run whose exchanges are the inputs themselves: the multi-GPU code
    paths of dist.TorchComm — and, for the split, of the C++ driver's RCCL transport
    (libdfx_dist.so) — exercised on the test box's one GPU.  The split's two drivers (C++ and
    Python) train identically."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    drivers = ("cpp", "py") if collective == "split" else ("py",)
    for driver in drivers:
        for force in (False, True):
            # (--standalone: the launcher binds its rendezvous port itself; a port picked here
            # and closed again was once taken first: EADDRINUSE)
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   "--nproc-per-node", "1", "--standalone", "--local-addr", "127.0.0.1",
                   "bench.py", "--sharded", "--steps", "4", "--warmup", "1",
                   "--batch", "20000", "--key-bits", "20", "--no-cpu-baseline", "--collective",
                   collective, "--driver", driver] + (["--force-collectives"] if force else [])
            r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
            lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
            assert len(lines) == 1, r.stdout
            outs.append(json.loads(lines[0]))
    a = outs[0]
    for b in outs[1:]:
        assert a["train_loss_per_row"] == b["train_loss_per_row"]
        assert a["train_auc"] == b["train_auc"]
        assert a["model_keys"] == b["model_keys"] and a["model_vrows"] == b["model_vrows"]
    assert set(outs[0]["collectives"]) == set(outs[1]["collectives"])
