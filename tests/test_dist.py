"""The sharded store's orchestration (difacto_amd/dist.py) on CPU: the owner rule, the
in-process exchange, and world_size 2 over torch.distributed / gloo, each checked against
the sharded oracle (N restated SGDUpdater servers, oracle/dist_oracle.py)."""
import os
import socket

import numpy as np
import pytest
import torch

from difacto_amd import data as D
from difacto_amd import dist as DI
from oracle import dist_oracle as DO
from tests.cpu_shard import CpuShard

KW = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.5, l2=0.01, seed=7)


def _batches(nranks, steps, rows=120, nnz=6, key_space=1500, seed=0):
    out = []
    for s in range(steps):
        out.append([D.synthetic(rows, nnz, key_space, binary=(r % 2 == 0), seed=seed + 97 * s + r,
                                ragged=(s == 1)) for r in range(nranks)])
    return out


def test_owner_rule():
    rng = np.random.default_rng(1)
    keys = np.concatenate([rng.integers(0, 2**63, 500, dtype=np.uint64) * np.uint64(2)
                           + rng.integers(0, 2, 500, dtype=np.uint64),
                           np.array([0, 1, 2**63, 2**64 - 1, 2**64 - 2], np.uint64)])
    for n in (1, 2, 3, 5, 8, 64):
        want = np.array([(int(k) * n) >> 64 for k in keys], np.int64)
        assert np.array_equal(DI.owner_of(keys, n), want)
        assert np.array_equal(DO.owner_of(keys, n), want)
        srt = np.sort(keys)
        assert np.all(np.diff(DO.owner_of(srt, n)) >= 0)  # contiguous ranges of sorted keys


def _state(shard, keys):
    out = {}
    for k in keys:
        e = shard.up.entry(k)
        if e is not None:
            out[int(k)] = (e[0].copy(), None if e[1] is None else e[1].copy())
    return out


def _all_keys(batches):
    from oracle import oracle as O
    return np.unique(np.concatenate([O.localize(b.offs, b.ids)[0]
                                     for step in batches for b in step]))


def _check_against_oracle(shards, so, batches):
    rkeys = _all_keys(batches)
    n_v = 0
    for g in range(so.N):
        own = rkeys[DO.owner_of(rkeys, so.N) == g]
        st = _state(shards[g], own)
        for k in own:
            e = so.up[g].entry(k)
            assert (e is None) == (int(k) not in st)
            if e is None:
                continue
            s, V = st[int(k)]
            assert np.array_equal(s, e[0]), (g, k)
            assert (V is None) == (e[1] is None)
            if V is not None:
                n_v += 1
                assert np.array_equal(V, e[1])
        assert shards[g].up.seed == so.up[g].seed
        assert shards[g].up.new_w == so.up[g].new_w
    return n_v


def _run_oracle(batches, push_epochs, nranks):
    so = DO.ShardedOracle(nranks, **KW)
    losses = []
    for s, step in enumerate(batches):
        out = so.step(step, push_cnt=s < push_epochs)
        losses.append([o[0] for o in out])
    return so, losses


def test_loopback_cpu_matches_sharded_oracle():
    N = 3
    batches = _batches(N, 4)
    shards = [CpuShard(N, **KW) for _ in range(N)]
    comm = DI.LoopbackComm(N)
    for s, step in enumerate(batches):
        DI.sharded_step(shards, step, comm, DI.kTraining, push_cnt=s < 2)
    so, losses = _run_oracle(batches, 2, N)
    for r in range(N):
        assert shards[r].losses == [l[r] for l in losses]
    assert _check_against_oracle(shards, so, batches) > 0  # InitV happened


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = CpuShard(world, **KW)
        comm = DI.TorchComm(device="cpu")
        batches = _batches(world, 4)
        for s, step in enumerate(batches):
            pred = torch.empty(step[rank].size, dtype=torch.float32)
            DI.sharded_step([shard], [step[rank]], comm, DI.kTraining, push_cnt=s < 2,
                            preds=[pred])
        tot = comm.allreduce_sum([[float(sum(shard.losses))]])[0][0]
        # ship the final server state for the keys this rank owns
        keys = _all_keys(batches)
        own = keys[DO.owner_of(keys, world) == rank]
        st = {int(k): v for k, v in _state(shard, own).items()}
        q.put((rank, shard.losses, tot, st, shard.up.seed, shard.up.new_w))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_world2_matches_sharded_oracle(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, losses, tot, st, seed, new_w = q.get(timeout=240)
            res[r] = (losses, tot, st, seed, new_w)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    batches = _batches(world, 4)
    so, losses = _run_oracle(batches, 2, world)
    total = sum(sum(l) for l in losses)
    for r in range(world):
        rl, tot, st, seed, new_w = res[r]
        assert rl == [l[r] for l in losses]
        assert tot == pytest.approx(total, rel=1e-12)
        assert seed == so.up[r].seed and new_w == so.up[r].new_w
        n_v = 0
        for k, (s, V) in st.items():
            e = so.up[r].entry(k)
            assert e is not None and np.array_equal(s, e[0])
            assert (V is None) == (e[1] is None)
            if V is not None:
                n_v += 1
                assert np.array_equal(V, e[1])
        assert n_v > 0  # the run exercised InitV on this server


def test_sharded_oracle_one_server_is_the_local_step():
    """N == 1: the sharded composition equals the oracle's own IterateData step
    (orc_train_step), which the reference's known answers pin."""
    from oracle import oracle as O
    batches = _batches(1, 4)
    so, losses = _run_oracle(batches, 2, 1)
    up = O.Updater(**KW)
    for s, (blk,) in enumerate(batches):
        loss, _ = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels, blk.weights,
                                push_cnt=s < 2)
        assert loss == losses[s][0]
    for k in _all_keys(batches):
        a, b = up.entry(k), so.up[0].entry(k)
        assert np.array_equal(a[0], b[0])
        assert (a[1] is None) == (b[1] is None)
        if a[1] is not None:
            assert np.array_equal(a[1], b[1])
    assert up.seed == so.up[0].seed


# ---- the pipelined (1-step-stale) schedule ---------------------------------------------------
# job per step: (job type, push_cnt); a validation step in the middle checks that it neither
# pushes nor loses the pending push
_PIPE_JOBS = [(DI.kTraining, True), (DI.kTraining, True), (DI.kTraining, False),
              (DI.kValidation, False), (DI.kTraining, False)]


def _run_stale_oracle(batches, nranks):
    so = DO.StaleOracle(nranks, **KW)
    losses = []
    for step, (job, cnt) in zip(batches, _PIPE_JOBS):
        out = so.submit(step, push_cnt=cnt, train=job == DI.kTraining)
        losses.append([o[0] for o in out])
    so.flush()
    return so, losses


def test_stale_oracle_differs_from_synchronous():
    """the pipelined schedule is a different (stale-by-one) schedule, not a relabelling"""
    batches = _batches(2, 4)
    a, la = _run_oracle(batches, 2, 2)
    b = DO.StaleOracle(2, **KW)
    lb = [[o[0] for o in b.submit(step, push_cnt=s < 2)] for s, step in enumerate(batches)]
    b.flush()
    assert la[0] == lb[0]  # the first pull sees the same (empty) model
    assert la[1] != lb[1]


def test_loopback_cpu_pipeline_matches_stale_oracle():
    N = 3
    batches = _batches(N, len(_PIPE_JOBS))
    shards = [CpuShard(N, **KW) for _ in range(N)]
    pipe = DI.ShardedPipeline(shards, DI.LoopbackComm(N))
    for step, (job, cnt) in zip(batches, _PIPE_JOBS):
        pipe.submit(step, job, push_cnt=cnt)
    pipe.flush()
    so, losses = _run_stale_oracle(batches, N)
    for r in range(N):
        assert shards[r].losses == [l[r] for l in losses]
    assert _check_against_oracle(shards, so.so, batches) > 0


def _gloo_pipe_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = CpuShard(world, **KW)
        pipe = DI.ShardedPipeline([shard], DI.TorchComm(device="cpu"))
        batches = _batches(world, len(_PIPE_JOBS))
        for step, (job, cnt) in zip(batches, _PIPE_JOBS):
            pipe.submit([step[rank]], job, push_cnt=cnt)
        pipe.flush()
        keys = _all_keys(batches)
        own = keys[DO.owner_of(keys, world) == rank]
        st = {int(k): v for k, v in _state(shard, own).items()}
        q.put((rank, shard.losses, st, shard.up.seed, shard.up.new_w))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_pipeline_matches_stale_oracle():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_pipe_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, losses, st, seed, new_w = q.get(timeout=240)
            res[r] = (losses, st, seed, new_w)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    so, losses = _run_stale_oracle(_batches(world, len(_PIPE_JOBS)), world)
    for r in range(world):
        rl, st, seed, new_w = res[r]
        assert rl == [l[r] for l in losses]
        assert seed == so.up[r].seed and new_w == so.up[r].new_w
        n_v = 0
        for k, (s, V) in st.items():
            e = so.up[r].entry(k)
            assert e is not None and np.array_equal(s, e[0])
            assert (V is None) == (e[1] is None)
            if V is not None:
                n_v += 1
                assert np.array_equal(V, e[1])
        assert n_v > 0


def _coll_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = DI.TorchComm(device="cpu", stage_cpu=True)
        M, row = 3, 2
        x = torch.arange(rank * 10, rank * 10 + 2 * row, dtype=torch.float32)  # 2 rows
        ag = comm.allgather_rows([x], M, row)[0]
        buf = torch.full((world * M * row,), float(rank + 1))
        rs = comm.reduce_scatter_sum([buf], M, row)[0]
        ai = comm.allgather_i64([torch.tensor([rank + 5], dtype=torch.int64)])[0]
        q.put((rank, ag.tolist(), rs.tolist(), ai.tolist()))
    finally:
        dist.destroy_process_group()


def test_torchcomm_union_collectives_gloo():
    """the rsag schedule's collectives over torch.distributed (world_size 2, gloo): padded
    all-gather of rows, reduce-scatter of union-indexed rows (all-reduce + own chunk on gloo),
    and the all-gather of the owners' InitV counts"""
    import torch.multiprocessing as mp
    world = 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_coll_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ag, rs, ai = q.get(timeout=100)
            res[r] = (ag, rs, ai)
    finally:
        for p in procs:
            p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    want_ag = [0, 1, 2, 3, 0, 0, 10, 11, 12, 13, 0, 0]
    for r in range(world):
        ag, rs, ai = res[r]
        assert ag == want_ag
        assert rs == [3.0] * 6  # 1 + 2 summed, this rank's chunk of M * row
        assert ai == [5, 6]
