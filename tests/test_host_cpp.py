"""The C++ host adapters (difacto_amd/host: GpuLocalizer, GpuFMLoss, GpuSGDUpdater, StoreGPU,
GpuSGDLearner over the C-ABI) and their test driver tests/host/host_tests.cc, which restates
the reference's own gtests (localizer_test.cc, fm_loss_test.cc, sgd_learner_test.cc)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "host_tests")
READER_BIN = os.path.join(ROOT, "build", "reader_tests")
TRAIN_BIN = os.path.join(ROOT, "build", "dfx_train")
DATA = os.path.join(ROOT, "tests", "golden", "rcv1_100.libsvm")


def test_host_adapters_build_and_link():
    """g++ builds the adapters against the C-ABI header alone and the binary resolves
    libdifacto_amd.so (no HIP headers, no torch in the host layer)."""
    subprocess.check_call(["make", "-s", "build/host_tests"], cwd=ROOT)
    out = subprocess.check_output(["ldd", BIN], text=True)
    assert "libdifacto_amd.so" in out and "not found" not in out
    syms = subprocess.check_output(["nm", "-D", "--undefined-only", BIN], text=True)
    for s in ("dfx_train_step", "dfx_localize", "dfx_fm_predict", "dfx_fm_calcgrad",
              "dfx_store_pull", "dfx_store_push", "dfx_store_save", "dfx_store_load"):
        assert s in syms, s


@pytest.mark.gpu
def test_host_adapters_reference_gtests():
    assert os.path.exists(BIN), "build/host_tests missing: run make"
    r = subprocess.run([BIN, DATA], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL PASSED" in r.stdout


def test_readers_reference_batch_reader_known_answers(tmp_path):
    """difacto_amd/host/reader.cc on the CPU: the reference's BatchReader.Read / RandRead /
    PartRead known answers (tests/cpp/batch_reader_test.cc) plus chunking, part, shuffle,
    down-sampling and criteo-layout properties (tests/host/reader_tests.cc)."""
    subprocess.check_call(["make", "-s", "build/reader_tests"], cwd=ROOT)
    r = subprocess.run([READER_BIN, DATA, str(tmp_path)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr


def test_train_driver_builds():
    subprocess.check_call(["make", "-s", "build/dfx_train"], cwd=ROOT)
    syms = subprocess.check_output(["nm", "-D", "--undefined-only", TRAIN_BIN], text=True)
    for s in ("dfx_feeder_create", "dfx_feeder_slot", "dfx_feeder_submit", "dfx_train_step"):
        assert s in syms, s
    r = subprocess.run([TRAIN_BIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


# SGDLearner.Basic (tests/cpp/sgd_learner_test.cc:9-30): the summed loss per epoch
_BASIC_OBJV = [69.314718, 69.314718, 67.151912, 61.414778, 56.244989, 53.218700, 51.248737,
               49.846688, 48.650164, 47.698351, 46.924038, 46.388223, 45.970721, 45.499307,
               45.102245, 44.798413, 44.565211, 44.386417, 44.240657, 44.109764]


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", ["0", "10"])
def test_train_driver_sgd_learner_basic(shuffle):
    """dfx_train (BatchReader -> dfx_feeder -> dfx_train_step) reproduces the reference's
    SGDLearner.Basic trace: same kwargs as sgd_learner_test.cc:32-39; stop_rel_objv=0 so all
    20 epochs run (epochs 0 and 1 have equal loss, which would stop the reference's loop)."""
    assert os.path.exists(TRAIN_BIN), "build/dfx_train missing: run make"
    r = subprocess.run([TRAIN_BIN, "data_in=" + DATA, "V_dim=0", "l2=1", "l1=1", "lr=1",
                        "num_jobs_per_epoch=1", "batch_size=100", "max_num_epochs=20",
                        "shuffle=" + shuffle, "stop_rel_objv=0", "max_keys=16384"],
                       capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    losses = [float(l.split("loss = ")[1].split(",")[0]) for l in r.stdout.splitlines()
              if "Training:" in l]
    assert len(losses) == 20
    for ep, (got, want) in enumerate(zip(losses, _BASIC_OBJV)):
        assert abs(got * 100 - want) < 5e-5, (ep, got * 100, want)


def _train_losses(args):
    r = subprocess.run([TRAIN_BIN, "data_in=" + DATA] + args, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = [(float(l.split("loss = ")[1].split(",")[0]), float(l.split("AUC = ")[1].split()[0]))
           for l in r.stdout.splitlines() if "Training:" in l]
    assert out, r.stdout
    return out


@pytest.mark.gpu
def test_train_driver_feeder_matches_interface_path():
    """Many small batches through the feeder's two pinned slots (fused=1) against the same
    batches through the Localizer/Loss/Store interfaces (fused=0): FM with V_dim 4, 3 jobs per
    epoch, batch 7, shuffled and down-sampled, 4 epochs.  Same kernels, so the traces agree to
    float rounding of the differently ordered reductions."""
    common = ["V_dim=4", "V_threshold=2", "lr=0.1", "V_lr=0.05", "l1=0.1",
              "num_jobs_per_epoch=3", "batch_size=7", "shuffle=3", "neg_sampling=0.7",
              "max_num_epochs=4", "stop_rel_objv=0", "max_keys=65536"]
    a = _train_losses(common + ["fused=1"])
    b = _train_losses(common + ["fused=0"])
    assert len(a) == len(b) == 4
    for (la, aa), (lb, ab) in zip(a, b):
        assert abs(la - lb) <= 1e-4 * abs(lb), (la, lb)
        assert abs(aa - ab) <= 1e-3, (aa, ab)


@pytest.mark.gpu
def test_train_driver_model_parts_and_prediction(tmp_path):
    """dfx_train model_out -> <prefix>_part-0 in SGDUpdater::Save's format (the oracle loads
    it), then task=2 with model_in predicts data_val into <pred_out>_part-0 (SavePred): the
    written probabilities equal the oracle's predictions from the loaded model"""
    import numpy as np
    from oracle import oracle as O
    from difacto_amd import data as D
    kw = ["V_dim=4", "V_threshold=1", "lr=0.1", "V_lr=0.05", "l1=0.1"]
    model = str(tmp_path / "model")
    preds = str(tmp_path / "pred")
    r = subprocess.run([TRAIN_BIN, "data_in=" + DATA, "num_jobs_per_epoch=1", "shuffle=0",
                        "batch_size=30", "max_num_epochs=3", "stop_rel_objv=0",
                        "model_out=" + model, "max_keys=65536"] + kw,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(model + "_part-0")
    r = subprocess.run([TRAIN_BIN, "task=2", "data_val=" + DATA, "model_in=" + model,
                        "pred_out=" + preds, "num_jobs_per_epoch=1", "max_keys=65536"] + kw,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Prediction:" in r.stdout
    lines = [l.split("\t") for l in open(preds + "_part-0").read().splitlines()]
    blk = D.read_libsvm(DATA)
    assert len(lines) == blk.size
    got = np.array([float(p) for _, p in lines])
    assert np.array_equal(np.array([float(y) for y, _ in lines]), blk.labels)
    up = O.Updater(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1)
    up.load(model + "_part-0")
    _, _, pred = up.train_step(blk.offs, blk.ids, blk.vals, blk.labels, train=False,
                               want_pred=True)
    want = 1.0 / (1.0 + np.exp(-pred.astype(np.float64)))
    assert np.allclose(got, want, rtol=2e-5, atol=1e-6)


CONV_BIN = os.path.join(ROOT, "build", "dfx_convert")


def _convert(*args):
    subprocess.check_call(["make", "-s", "build/dfx_convert"], cwd=ROOT)
    r = subprocess.run([CONV_BIN] + list(args), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_converter_libsvm_rec_round_trip(tmp_path):
    """dfx_convert (src/reader/converter.h): libsvm -> rec (CompressedRowBlock RecordIO) ->
    libsvm gives back the same rows (values to the %g precision of the libsvm writer), also
    split into parts"""
    import numpy as np
    from difacto_amd import data as D
    rec, txt = str(tmp_path / "rcv1.rec"), str(tmp_path / "rcv1.txt")
    _convert("data_in=" + DATA, "data_format=libsvm", "data_out=" + rec,
             "data_out_format=rec", "chunk_size=0.01")
    _convert("data_in=" + rec, "data_format=rec", "data_out=" + txt, "data_out_format=libsvm")
    a, b = D.read_libsvm(DATA), D.read_libsvm(txt)
    assert np.array_equal(a.offs, b.offs) and np.array_equal(a.ids, b.ids)
    assert np.array_equal(a.labels, b.labels)
    assert np.allclose(a.vals, b.vals, rtol=1e-5, atol=0)
    parts = str(tmp_path / "p.rec")
    _convert("data_in=" + DATA, "data_format=libsvm", "data_out=" + parts,
             "data_out_format=rec", "chunk_size=0.01", "part_size=0")
    assert os.path.exists(parts + "-part_0")


@pytest.mark.gpu
def test_train_driver_reads_rec(tmp_path):
    """SGDLearner.Basic through dfx_train on the rec conversion of the data"""
    rec = str(tmp_path / "rcv1.rec")
    _convert("data_in=" + DATA, "data_format=libsvm", "data_out=" + rec,
             "data_out_format=rec", "chunk_size=0.02")
    r = subprocess.run([TRAIN_BIN, "data_in=" + rec, "data_format=rec", "V_dim=0", "l2=1",
                        "l1=1", "lr=1", "num_jobs_per_epoch=1", "batch_size=100",
                        "max_num_epochs=20", "shuffle=0", "stop_rel_objv=0", "max_keys=16384"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    losses = [float(l.split("loss = ")[1].split(",")[0]) for l in r.stdout.splitlines()
              if "Training:" in l]
    assert len(losses) == 20
    for ep, (got, want) in enumerate(zip(losses, _BASIC_OBJV)):
        assert abs(got * 100 - want) < 5e-5, (ep, got * 100, want)


def _part_rows(path, part, nparts):
    """row indices of part k of n of a text file: byte range [size*k/n, size*(k+1)/n), both
    ends moved to the next line start (reader.cc TextReader, InputSplit semantics)"""
    data = open(path, "rb").read()
    size = len(data)

    def line_start(at):
        if at == 0 or at >= size:
            return min(at, size)
        nl = data.find(b"\n", at - 1)
        return size if nl < 0 else nl + 1

    b, e = line_start(size * part // nparts), line_start(size * (part + 1) // nparts)
    starts = [0] + [i + 1 for i, c in enumerate(data) if c == 10][:-1]
    return [r for r, s in enumerate(starts) if b <= s < e]


def _slice(blk, rows):
    from difacto_amd import data as D
    import numpy as np
    if not rows:
        return D.RowBlock(np.zeros(1, np.uint64), np.zeros(0, np.uint64), None,
                          np.zeros(0, np.float32))
    offs = blk.offs.astype(np.int64)
    lo, hi = rows[0], rows[-1] + 1
    o = offs[lo:hi + 1] - offs[lo]
    vals = blk.vals[offs[lo]:offs[hi]]
    if np.all(vals == 1):
        vals = None  # batch_reader.cc:71-73
    return D.RowBlock(o.astype(np.uint64), blk.ids[offs[lo]:offs[hi]], vals,
                      blk.labels[lo:hi])


@pytest.mark.gpu
@pytest.mark.parametrize("agg,max_keys", [("sum", 65536), ("ranks", 65536), ("sum", 256),
                                          ("ranks", 256)])
@pytest.mark.parametrize("pipelined", [1, 0])
def test_train_driver_sharded_loopback_matches_oracle(tmp_path, pipelined, agg, max_keys):
    """dfx_train shards=3: the C++ sharded store (dist_host.cc, loopback exchange) against the
    sharded oracle of the same schedule, on the batches the driver forms (shard r reads part
    r of 3, batches of 10 rows, shards step together with empty batches once done): per-epoch
    loss, and every server's saved part against the oracle's server state.
    max_keys=256: each server's table starts below its ~900 keys and grows at the owner
    steps' begins (the reference's model is an unbounded map, sgd_updater.h:178); in the
    pipelined schedule the other step, which holds table positions until its push, gets them
    moved by the rebuild"""
    import numpy as np
    from oracle import dist_oracle as DO
    from oracle import oracle as O
    from difacto_amd import data as D
    N, bs, epochs = 3, 10, 3
    kw = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1, seed=7)
    model = str(tmp_path / "m")
    args = [TRAIN_BIN, "data_in=" + DATA, "shards=%d" % N, "pipelined=%d" % pipelined,
            "num_jobs_per_epoch=1", "shuffle=0", "batch_size=%d" % bs,
            "max_num_epochs=%d" % epochs, "stop_rel_objv=0", "model_out=" + model, "has_aux=1",
            "max_keys=%d" % max_keys, "push_agg=" + agg] + ["%s=%s" % kv for kv in kw.items()]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = [float(l.split("loss = ")[1].split(",")[0]) for l in r.stdout.splitlines()
           if "Training:" in l]
    assert len(got) == epochs, r.stdout
    blk = D.read_libsvm(DATA)
    parts = [_part_rows(DATA, p, N) for p in range(N)]
    nsteps = max((len(p) + bs - 1) // bs for p in parts)
    if pipelined:
        so = DO.StaleOracle(N, agg=agg, **kw)
    else:
        so = DO.AggOracle(N, **kw) if agg == "sum" else DO.ShardedOracle(N, **kw)
    for ep in range(epochs):
        loss = 0.0
        for t in range(nsteps):
            step = [_slice(blk, parts[p][t * bs:(t + 1) * bs]) for p in range(N)]
            out = (so.submit(step, push_cnt=ep == 0) if pipelined
                   else so.step(step, push_cnt=ep == 0))
            loss += sum(o[0] for o in out)
        if pipelined:
            so.flush()
        assert abs(got[ep] - loss / blk.size) <= 1e-5 * abs(loss / blk.size), (ep, got[ep])
    ups = so.up
    for g in range(N):
        up = O.Updater(**kw)
        up.load(model + "_part-%d" % g)
        keys = np.unique(blk.ids)
        n = 0
        for k in O.localize(blk.offs, blk.ids)[0]:
            a, b = up.entry(k), ups[0 if agg == "sum" else g].entry(k)
            if a is None:
                continue
            n += 1
            assert b is not None
            assert np.allclose(a[0][:3], b[0][:3], rtol=1e-5, atol=1e-6), (g, k)
            assert (a[1] is None) == (b[1] is None)
            if a[1] is not None:
                assert np.allclose(a[1], b[1], rtol=1e-5, atol=1e-6)
        assert n == up.size() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined,max_keys", [(1, 65536), (0, 65536), (1, 256)])
def test_train_driver_split_loopback_matches_oracle(tmp_path, pipelined, max_keys):
    """dfx_train shards=3 exchange=split: the sharded epochs through GpuSplitLearner (the
    owner-computes split) on the batches the driver forms, against the synchronous sum oracle
    (one reference step per batch index on the concatenated batches; the pipelined schedule
    only overlaps model-free work): per-epoch loss and every server's saved part; max_keys=256
    grows the servers' tables mid-run"""
    import numpy as np
    from oracle import dist_oracle as DO
    from oracle import oracle as O
    from difacto_amd import data as D
    N, bs, epochs = 3, 10, 3
    kw = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1, seed=7)
    model = str(tmp_path / "m")
    args = [TRAIN_BIN, "data_in=" + DATA, "shards=%d" % N, "pipelined=%d" % pipelined,
            "exchange=split", "num_jobs_per_epoch=1", "shuffle=0", "batch_size=%d" % bs,
            "max_num_epochs=%d" % epochs, "stop_rel_objv=0", "model_out=" + model, "has_aux=1",
            "max_keys=%d" % max_keys] + ["%s=%s" % kv for kv in kw.items()]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = [float(l.split("loss = ")[1].split(",")[0]) for l in r.stdout.splitlines()
           if "Training:" in l]
    assert len(got) == epochs, r.stdout
    blk = D.read_libsvm(DATA)
    parts = [_part_rows(DATA, p, N) for p in range(N)]
    nsteps = max((len(p) + bs - 1) // bs for p in parts)
    so = DO.AggOracle(N, **kw)
    for ep in range(epochs):
        loss = 0.0
        for t in range(nsteps):
            out = so.step([_slice(blk, parts[p][t * bs:(t + 1) * bs]) for p in range(N)],
                          push_cnt=ep == 0)
            loss += sum(o[0] for o in out)
        assert abs(got[ep] - loss / blk.size) <= 1e-5 * abs(loss / blk.size), (ep, got[ep])
    for g in range(N):
        up = O.Updater(**kw)
        up.load(model + "_part-%d" % g)
        n = 0
        for k in O.localize(blk.offs, blk.ids)[0]:
            a, b = up.entry(k), so.up[0].entry(k)
            if a is None:
                continue
            n += 1
            assert b is not None
            assert np.allclose(a[0][:3], b[0][:3], rtol=1e-5, atol=1e-6), (g, k)
            assert (a[1] is None) == (b[1] is None)
            if a[1] is not None:
                assert np.allclose(a[1], b[1], rtol=1e-5, atol=1e-6)
        assert n == up.size() > 0


@pytest.mark.gpu
def test_train_driver_sharded_rccl_world1(tmp_path):
    """shards=-1: one shard per process over RCCL (communicators from a node-local id file);
    at world size 1 it trains like the single-context store: the same batches (one part),
    the same stale-by-one pipelined schedule as a 1-shard StaleOracle"""
    from oracle import dist_oracle as DO
    from difacto_amd import data as D
    kw = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1, seed=7)
    env = dict(os.environ, DFX_COMM_ID_FILE=str(tmp_path / "id"))
    r = subprocess.run([TRAIN_BIN, "data_in=" + DATA, "shards=-1", "num_jobs_per_epoch=1",
                        "shuffle=0", "batch_size=25", "max_num_epochs=2", "stop_rel_objv=0",
                        "max_keys=65536", "push_agg=sum"] + ["%s=%s" % kv for kv in kw.items()],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    got = [float(l.split("loss = ")[1].split(",")[0]) for l in r.stdout.splitlines()
           if "Training:" in l]
    blk = D.read_libsvm(DATA)
    so = DO.StaleOracle(1, agg="sum", **kw)
    for ep in range(2):
        loss = 0.0
        for t in range(4):
            loss += so.submit([_slice(blk, list(range(25 * t, 25 * t + 25)))],
                              push_cnt=ep == 0)[0][0]
        so.flush()
        assert abs(got[ep] - loss / 100) <= 1e-5 * abs(loss / 100), (ep, got[ep])
    assert not os.path.exists(str(tmp_path / "id"))


@pytest.mark.gpu
@pytest.mark.parametrize("shards,agg,max_keys", [(3, "sum", 65536), (3, "ranks", 65536),
                                                 (-1, "sum", 65536), (3, "sum", 256),
                                                 (-1, "sum", 256)])
def test_dist_store_iterate_data_matches_oracle(tmp_path, shards, agg, max_keys):
    """GpuDistStore behind the reference's Store interface (dist_store.h): IterateData's
    executor (Compact -> Push(kFeaCount) + Wait -> Pull -> Predict / Evaluate / AUC -> CalcGrad
    -> Push(kGradient), through GpuSGDLearner's interface path) with N=3 loopback workers on
    their own threads, or one RCCL worker (world 1), against the synchronous sharded oracle of
    the same aggregation: per-epoch loss and AUC, and every server's saved part.  max_keys=256:
    the servers' tables start far below the model and grow mid-run (sgd_updater.h:178)"""
    import numpy as np
    from oracle import dist_oracle as DO
    from oracle import oracle as O
    from difacto_amd import data as D
    N = shards if shards > 0 else 1
    bs, epochs = 10, 3
    kw = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1, seed=7)
    model = str(tmp_path / "m")
    env = dict(os.environ, DFX_COMM_ID_FILE=str(tmp_path / "id"))
    r = subprocess.run([BIN, "dist", DATA, "shards=%d" % shards, "epochs=%d" % epochs,
                        "batch_size=%d" % bs, "model_out=" + model, "max_keys=%d" % max_keys,
                        "push_agg=" + agg] + ["%s=%s" % kv for kv in kw.items()],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL PASSED" in r.stdout, r.stdout
    got = [l.split() for l in r.stdout.splitlines() if l.startswith("epoch ")]
    assert len(got) == epochs, r.stdout
    blk = D.read_libsvm(DATA)
    n = blk.size
    parts = [list(range(p * n // N, (p + 1) * n // N)) for p in range(N)]
    nsteps = max((len(p) + bs - 1) // bs for p in parts)
    so = DO.AggOracle(N, **kw) if agg == "sum" else DO.ShardedOracle(N, **kw)
    for ep in range(epochs):
        loss = auc = 0.0
        for t in range(nsteps):
            out = so.step([_slice(blk, parts[p][t * bs:(t + 1) * bs]) for p in range(N)],
                          push_cnt=ep == 0)
            loss += sum(o[0] for o in out)
            auc += sum(o[1] for o in out)
        g_loss, g_auc, g_rows = float(got[ep][3]), float(got[ep][5]), float(got[ep][7])
        assert g_rows == n
        assert abs(g_loss - loss) <= 1e-5 * abs(loss), (ep, g_loss, loss)
        assert abs(g_auc - auc) <= 1e-4 * n, (ep, g_auc, auc)
    for g in range(N):
        up = O.Updater(**kw)
        up.load(model + "_part-%d" % g)
        cnt = 0
        for k in O.localize(blk.offs, blk.ids)[0]:
            a, b = up.entry(k), so.up[0 if agg == "sum" else g].entry(k)
            if a is None:
                continue
            cnt += 1
            assert b is not None
            assert np.allclose(a[0][:3], b[0][:3], rtol=1e-5, atol=1e-6), (g, k)
            assert (a[1] is None) == (b[1] is None)
            if a[1] is not None:
                assert np.allclose(a[1], b[1], rtol=1e-5, atol=1e-6)
        assert cnt == up.size() > 0
    assert not os.path.exists(str(tmp_path / "id"))


@pytest.mark.gpu
@pytest.mark.parametrize("shards,max_keys,extra", [(3, 65536, []), (-1, 65536, []),
                                                   (3, 256, []), (-1, 256, []),
                                                   (3, 65536, ["slices=2"]),
                                                   (3, 256, ["pipelined=0"])])
def test_split_learner_iterate_data_matches_oracle(tmp_path, shards, max_keys, extra):
    """GpuSplitLearner (split_learner.h): IterateData's executor fed raw minibatches, the
    owner-computes split behind it (libdfx_dist.so) — N=3 loopback workers on their own
    threads, or one RCCL worker (world 1) — against the synchronous sum oracle (one reference
    step on the concatenated batches): per-epoch loss and AUC, and every server's saved part.
    max_keys=256: each server's table starts below its share of the model and grows mid-run
    (sgd_updater.h:178); slices=2: the sliced exchange schedule; pipelined=0: synchronous"""
    import numpy as np
    from oracle import dist_oracle as DO
    from oracle import oracle as O
    from difacto_amd import data as D
    N = shards if shards > 0 else 1
    bs, epochs = 10, 3
    kw = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1, seed=7)
    model = str(tmp_path / "m")
    env = dict(os.environ, DFX_COMM_ID_FILE=str(tmp_path / "id"))
    r = subprocess.run([BIN, "split", DATA, "shards=%d" % shards, "epochs=%d" % epochs,
                        "batch_size=%d" % bs, "model_out=" + model, "max_keys=%d" % max_keys]
                       + extra + ["%s=%s" % kv for kv in kw.items()],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL PASSED" in r.stdout, r.stdout
    got = [l.split() for l in r.stdout.splitlines() if l.startswith("epoch ")]
    assert len(got) == epochs, r.stdout
    blk = D.read_libsvm(DATA)
    n = blk.size
    parts = [list(range(p * n // N, (p + 1) * n // N)) for p in range(N)]
    nsteps = max((len(p) + bs - 1) // bs for p in parts)
    so = DO.AggOracle(N, **kw)
    for ep in range(epochs):
        loss = auc = 0.0
        for t in range(nsteps):
            out = so.step([_slice(blk, parts[p][t * bs:(t + 1) * bs]) for p in range(N)],
                          push_cnt=ep == 0)
            loss += sum(o[0] for o in out)
            auc += sum(o[1] for o in out)
        g_loss, g_auc, g_rows = float(got[ep][3]), float(got[ep][5]), float(got[ep][7])
        assert g_rows == n
        assert abs(g_loss - loss) <= 1e-5 * abs(loss), (ep, g_loss, loss)
        assert abs(g_auc - auc) <= 1e-4 * n, (ep, g_auc, auc)
    for g in range(N):
        up = O.Updater(**kw)
        up.load(model + "_part-%d" % g)
        cnt = 0
        for k in O.localize(blk.offs, blk.ids)[0]:
            a, b = up.entry(k), so.up[0].entry(k)
            if a is None:
                continue
            cnt += 1
            assert b is not None
            assert np.allclose(a[0][:3], b[0][:3], rtol=1e-5, atol=1e-6), (g, k)
            assert (a[1] is None) == (b[1] is None)
            if a[1] is not None:
                assert np.allclose(a[1], b[1], rtol=1e-5, atol=1e-6)
        assert cnt == up.size() > 0
    assert not os.path.exists(str(tmp_path / "id"))


def _dist_oracle_epochs(blk, N, bs, epochs, agg, kw):
    """per-epoch (loss, auc) of the lockstep sharded oracle: worker p trains rows
    [p n / N, (p + 1) n / N) in batches of bs, the workers stepping together"""
    from oracle import dist_oracle as DO
    n = blk.size
    parts = [list(range(p * n // N, (p + 1) * n // N)) for p in range(N)]
    nsteps = max((len(p) + bs - 1) // bs for p in parts)
    so = DO.AggOracle(N, **kw) if agg == "sum" else DO.ShardedOracle(N, **kw)
    out = []
    for ep in range(epochs):
        loss = auc = 0.0
        for t in range(nsteps):
            res = so.step([_slice(blk, parts[p][t * bs:(t + 1) * bs]) for p in range(N)],
                          push_cnt=ep == 0)
            loss += sum(o[0] for o in res)
            auc += sum(o[1] for o in res)
        out.append((loss, auc))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("shards,sync,uneven", [(1, "lockstep", 0), (3, "lockstep", 0),
                                                (-1, "lockstep", 0), (3, "async", 1)])
def test_dist_store_async_iterate_data(tmp_path, shards, sync, uneven):
    """SGDLearner::IterateData with its own threads (host_tests.cc IterateDataAsync: a reader
    thread that localizes and pushes counts ahead, an executor whose pull callback computes and
    pushes the gradient, two batches in flight) over GpuDistStore workers:
    requests queue per worker and one progress thread per process serves them.
    * lockstep, even parts: the result equals the lockstep oracle (one step per batch index);
    * async, uneven parts (worker r holds r + 1 sixths of the rows): no worker waits for the
      others, every row is trained once per epoch, and the loss stays near the lockstep run's
      (which requests share an update depends on timing, as on ps-lite's server)."""
    from difacto_amd import data as D
    N = shards if shards > 0 else 1
    bs, epochs = 10, 3
    kw = dict(V_dim=4, V_threshold=1, lr=0.1, V_lr=0.05, l1=0.1, seed=7)
    env = dict(os.environ, DFX_COMM_ID_FILE=str(tmp_path / "id"))
    r = subprocess.run([BIN, "dist_async", DATA, "shards=%d" % shards, "epochs=%d" % epochs,
                        "batch_size=%d" % bs, "uneven=%d" % uneven, "max_keys=65536",
                        "store_sync=" + sync, "push_agg=sum"]
                       + ["%s=%s" % kv for kv in kw.items()],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL PASSED" in r.stdout, r.stdout
    got = [l.split() for l in r.stdout.splitlines() if l.startswith("epoch ")]
    assert len(got) == epochs, r.stdout
    blk = D.read_libsvm(DATA)
    want = _dist_oracle_epochs(blk, N, bs, epochs, "sum", kw)
    for ep in range(epochs):
        g_loss, g_auc, g_rows = float(got[ep][3]), float(got[ep][5]), float(got[ep][7])
        assert g_rows == blk.size
        loss, auc = want[ep]
        if uneven:
            assert abs(g_loss - loss) <= 0.05 * abs(loss), (ep, g_loss, loss)
        else:
            assert abs(g_loss - loss) <= 1e-5 * abs(loss), (ep, g_loss, loss)
            assert abs(g_auc - auc) <= 1e-4 * blk.size, (ep, g_auc, auc)
