#!/usr/bin/env python3
"""bench.py — train examples/sec of DiFacto's FM (V_dim=16) hot path on MI355X.

Workload (BASELINE.json configs[2]): Criteo-shaped synthetic data,
39 binary nnz per row, feature ids ~ U[0, 2^24), labels +1 w.p. 0.25; FM V_dim=16 with the
throughput settings l1=0, V_threshold=0 (every key carries V once touched), lr=.1,
V_lr=.01; B=100,000 rows per GPU per step.

A "step" is one minibatch through the whole per-batch hot path of SGDLearner::IterateData
(sgd_learner.cc:201-317): Localizer (sort/unique/remap) -> pull -> FM forward -> Evaluate
-> AUC -> FM backward -> FTRL/AdaGrad push (+ InitV), as ONE dfx_train_step on device-resident
input.  Before timing, one untimed "epoch 0" pass over the key space pushes feature counts
(kFeaCount) so the model is in its steady state (every key has V); then W warmup steps and K
timed steps run on fresh batches (epoch >= 1, no count push), as in the reference.

Prints one JSON line (driver contract) with a roofline object for the dominant kernel and a
cpu_baseline (the oracle restatement timed on this host on a bounded sample).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without a launcher bench.py starts them")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="BASELINE.json workload: c3 (the metric's, default), c2 (LR V_dim=0, "
                         "40 valued nnz, 2^20 keys, FTRL L1), c5 (Zipf(1.1) keys, V_dim=128, "
                         "lazy V), c4shard (one GPU's share of C4: 2^27 keys, V_dim=64)")
    # 100 timed steps: the first step's Localizer (not yet overlapped) and the pipeline's
    # drain are amortised (+2 % over 20 steps, same box); still well under a second of GPU
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="rows per GPU per step")
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--key-bits", type=int, default=None)
    ap.add_argument("--vdim", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sharded", action="store_true",
                    help="use the key-range-sharded store even at N=1 (default for N>1)")
    ap.add_argument("--sync", action="store_true",
                    help="sharded store: bulk-synchronous steps instead of the pipelined "
                         "(1-step-stale) schedule")
    ap.add_argument("--push-agg", default="sum", choices=("sum", "ranks"),
                    help="sharded store: sum = one Update per key per step on the workers' "
                         "summed gradients (SURVEY §8(e): a step is one reference step over "
                         "the concatenated batches); ranks = one Update per pushing worker "
                         "(KVStoreDist HandlePush)")
    ap.add_argument("--collective", default="split", choices=("split", "a2a"),
                    help="sharded store schedule: split = owner-computes FM (owners run the "
                         "forward partials and the backward on their keys; per-row partials "
                         "all-to-all + [XV*p | p] all-gather, bulk synchronous); a2a = model "
                         "records / gradients all-to-all-v (pipelined unless --sync).  The "
                         "other schedules, and the north_star's literal union all-gather / "
                         "reduce-scatter (rsag), are measured beside it on short runs")
    ap.add_argument("--slices", type=int, default=0,
                    help="split C++ driver: rows of a step in this many slices, each slice's "
                         "exchanges beside the next slice's compute (0: the driver's default, "
                         "one slice)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="sharded store: run every exchange as an RCCL collective even at N=1 "
                         "(tests the multi-GPU code paths on one GPU)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="sharded store transport; gloo (staged through host memory) runs "
                         "several ranks on one GPU, for tests")
    ap.add_argument("--main-prio", default=None, choices=("normal", "high"),
                    help="priority of the compute stream (default: high for the sharded "
                         "store, normal for the fused step).  Streams of one HIP priority "
                         "share that priority's hardware queues, whose packets run in order: "
                         "a high-priority compute stream keeps the step's kernels off the "
                         "queues of RCCL's (normal-priority) streams")
    ap.add_argument("--stale", action="store_true",
                    help="sharded split, C++ driver: the 1-step-stale schedule (step t+1's owner "
                         "forward before step t's backward, each step's partial exchange and "
                         "row gather beside the other step's compute; oracle: "
                         "dist_oracle.SplitStaleOracle)")
    ap.add_argument("--driver", default="cpp", choices=("cpp", "py"),
                    help="the split step's driver over RCCL: C++ (libdfx_dist.so, its own "
                         "communicators) or Python (dist.SplitPipeline over torch.distributed)")
    ap.add_argument("--comm-prio", default="high", choices=("normal", "high"),
                    help="priority of RCCL's streams (TorchComm comm_priority)")
    ap.add_argument("--ctx", default="",
                    help="extra context kwargs k=v,... (A/B of execution choices, e.g. "
                         "sort_pack=0)")
    ap.add_argument("--cpu-rows", type=int, default=200_000)
    ap.add_argument("--cpu-batch", type=int, default=10_000)
    args = ap.parse_args()
    cf = CONFIGS[args.config]
    for k in ("batch", "nnz", "key_bits", "vdim"):
        if getattr(args, k) is None:
            setattr(args, k, cf[k])
    return args


# BASELINE.json configs (SURVEY.md §8(d) shapes).  keys: rows per step, nnz per row, key space
# bits, V_dim, valued data, Zipf exponent (None: uniform ids), the updater's .conf keys
CONFIGS = {
    "c3": dict(batch=100_000, nnz=39, key_bits=24, vdim=16, valued=False, zipf=None,
               upd=dict(V_threshold=0, l1=0, lr=.1, V_lr=.01),
               name="C3 Criteo-shaped FM V_dim=%(vdim)d, %(nnz)d binary nnz/row, 2^%(key_bits)d "
                    "keys, l1=0 V_threshold=0"),
    "c2": dict(batch=100_000, nnz=40, key_bits=20, vdim=0, valued=True, zipf=None,
               upd=dict(l1=1, l2=0, lr=.1),
               name="C2 LR-only (V_dim=0) FTRL L1 (l1=1), %(nnz)d valued nnz/row, 2^%(key_bits)d "
                    "keys"),
    "c5": dict(batch=100_000, nnz=39, key_bits=24, vdim=128, valued=False, zipf=1.1,
               upd=dict(lr=.05, V_lr=.01),
               name="C5 Zipf(1.1) keys over [1, 2^%(key_bits)d], FM V_dim=%(vdim)d, %(nnz)d binary "
                    "nnz/row, defaults (V_threshold=10, l1=1, l1_shrk): lazy V for hot keys"),
    "c4shard": dict(batch=100_000, nnz=39, key_bits=27, vdim=64, valued=False, zipf=None,
                    upd=dict(V_threshold=0, l1=0, lr=.1, V_lr=.01),
                    name="C4 one GPU's share: 2^%(key_bits)d keys (2^30 over 8 GPUs), FM "
                         "V_dim=%(vdim)d, %(nnz)d binary nnz/row, l1=0 V_threshold=0, fused step"),
}


class DevBatch:
    """A synthetic RowBlock generated directly in HBM (torch is only the allocator/RNG).
    Uniform ids ~ U[0, 2^key_bits) on the device; Zipf(s) ids over [1, 2^key_bits] drawn on the
    host (difacto_amd.data.zipf_keys) and copied once, before timing.  valued: x ~ U(0, 1]."""

    def __init__(self, torch, dev, B, k, key_bits, seed, valued=False, zipf=None):
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        self.size = B
        self.nnz = B * k
        if zipf is None:
            self.ids = torch.randint(0, 1 << key_bits, (self.nnz,), device=dev, generator=g,
                                     dtype=torch.int64)
        else:
            from difacto_amd import data as D
            ids = D.zipf_keys(np.random.default_rng(seed), self.nnz, zipf, 1 << key_bits)
            self.ids = torch.from_numpy(ids.view(np.int64)).to(dev)
        self.offs = torch.arange(0, self.nnz + 1, k, device=dev, dtype=torch.int64)
        r = torch.rand(B, device=dev, generator=g)
        self.labels = torch.where(r < 0.25, 1.0, -1.0).to(torch.float32)
        self.vals = (1.0 - torch.rand(self.nnz, device=dev, generator=g)) if valued else None
        self.weights = None

    def as_batch(self):
        from difacto_amd import _lib
        import ctypes
        return _lib.Batch(self.size, self.nnz, ctypes.c_void_p(self.offs.data_ptr()),
                          ctypes.c_void_p(self.ids.data_ptr()),
                          ctypes.c_void_p(self.vals.data_ptr()) if self.vals is not None else None,
                          ctypes.c_void_p(self.labels.data_ptr()), None)


def algorithmic_bytes(B, nnz, U, d, valued=False, U_V=None, occ_V=None):
    """Essential HBM bytes per launch, every datum counted once per step: a
    key's entry and V row once however many of the batch's nnz read it (hot Zipf keys are read
    from cache, not HBM), a row's [XV*p | p] once however many occurrences read it.  U_V: keys
    with live V (dfx_prof_counts; default: every key); valued: + the value per nnz.  occ_V is
    accepted for the callers' sake and no longer priced (per-occurrence gathers of one key's V
    are reuse, not traffic)"""
    if U_V is None:
        U_V = U
    x = 4 if valued else 0
    row = 4 * (d + 1) if d > 0 else 4  # a row's [XV*p | p] (p alone at V_dim 0)
    # forward: per row its offset, label, pred and the [XV*p | p] row it writes; per nnz its
    # id (+ value); per unique key its entry {key, w, vrow} and, when live, its V row
    fwd = B * (8 + 4 + 4 + row) + nnz * (8 + x) + U * 16 + U_V * 4 * d
    # backward: per unique key its segment start, key, slot, entry read + written; V and Vaux
    # read + written when live; per occurrence its row index (+ value); per row its [XV*p | p]
    bwd = U * (8 + 4 + 8 + 32 + 4) + U_V * 16 * d + nnz * (4 + x) + B * row
    return {"forward": fwd, "backward_update": bwd}


def algorithmic_bytes_sharded(B, nnz, U, d):
    """Essential HBM bytes of the worker's dfx_dist_fwd_bwd (forward + backward over pulled
    records of S = d + 4 floats, binary data, all V live), each datum once per step: forward
    per row offs / label / pred / [XV*p | p], per nnz its col, per unique key its record;
    backward per key its segment start and the whole gradient record written, per occurrence
    its row index, per row its [XV*p | p]."""
    S = d + 4
    row = 4 * (d + 1)
    fwd = B * (8 + 4 + 4 + row) + nnz * 4 + U * 4 * S
    bwd = U * (4 + 4 * S) + nnz * 4 + B * row
    return fwd + bwd


PMC_ROUND = "r6"

# Random 128-byte lines per second on MI355X in the step's own access patterns, measured alone
# with cold caches (tools/membench/spanbench, profiles/r5/spanbench_cold.txt): the forward's
# read of 3.9 M random fat slots (84.3 us), the backward's read-modify-write of 3.48 M sorted
# keys' slot + Vaux row (329.3 us: 2 lines per key; in one 256-B span the same 331 us, so two
# lines per key is this layout's floor)
CHUNK_READS_PER_S = 46.2e9
CHUNK_RMW_PER_S = 21.1e9
STREAM_BYTES_PER_S = 5.0e12  # the Localizer lane's streaming passes
LOC_BYTES_PER_NNZ = 70.0     # the bucket Localizer's traffic per nnz (profiles/r4 PMC: ~273 MB)


def chunk_model(nnz, U, ms_per_step):
    """The step's floor in random 128-B chunks: the forward reads one fat slot
    per nnz, the backward read-modify-writes two chunks per unique key (its slot and its Vaux
    row), the Localizer streams; the measured step against that floor"""
    floor_ms = (nnz / CHUNK_READS_PER_S + 2 * U / CHUNK_RMW_PER_S
                + nnz * LOC_BYTES_PER_NNZ / STREAM_BYTES_PER_S) * 1e3
    return {"floor_ms": round(floor_ms, 4), "frac": round(floor_ms / ms_per_step, 3),
            "source": "tools/membench/spanbench cold-cache line rates; DESIGN.md (d)"}  # the profiles/<round>/ the traffic figures come from (tools/profile.sh)


def pmc_traffic(prefixes, fname="pmc_hbm.json"):
    """HBM bytes per step of a phase's kernels (every kernel whose name starts with one of
    prefixes, e.g. the backward phase's k_fm_bwd* and k_chunk_hotsum) from the committed
    rocprofv3 PMC passes (profiles/<PMC_ROUND>/<fname>: FETCH_SIZE + WRITE_SIZE per dispatch,
    separate --pmc runs of this bench, tools/profile.sh).  None when absent."""
    path = os.path.join(ROOT, "profiles", PMC_ROUND, fname)
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    if isinstance(prefixes, str):
        prefixes = (prefixes,)
    hit = [v for name, v in ks.items() if name.startswith(prefixes)]
    if not hit:
        return None
    return int(sum(v["fetch_size_kb_per_dispatch"] + v["write_size_kb_per_dispatch"]
                   for v in hit) * 1024)


def pmc_requests(kernel_prefix, fname="pmc_requests.json"):
    """the L2's memory-side read / write requests per launch of a kernel (a separate --pmc pass,
    profiles/<PMC_ROUND>/pmc_requests.json), or None"""
    path = os.path.join(ROOT, "profiles", PMC_ROUND, fname)
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    for name, v in ks.items():
        if name.startswith(kernel_prefix):
            return v
    return None


def sharded_traffic():
    """the a2a sharded worker's forward + backward (record mode) HBM bytes per step (round 1's
    passes: the a2a schedule is unchanged since)"""
    path = os.path.join(ROOT, "profiles", "r1", "pmc_hbm_sharded.json")
    try:
        ks = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    tot = 0
    for pre in ("k_fm_fwd<4, 4, 2, false, true>", "k_fm_bwd<4, 4, false, true>"):
        v = next((v for n, v in ks.items() if n.startswith(pre)), None)
        if v is None:
            return None
        tot += int((v["fetch_size_kb_per_dispatch"] + v["write_size_kb_per_dispatch"]) * 1024)
    return tot


def forward_roofline(fwd_bytes, fwd_ms, config):
    """The forward's fraction of the byte peak (its phase time from the diagnostic pass, which
    runs beside the Localizer lane as the timed steps do) and its HBM traffic.  FETCH_SIZE counts
    a 128-byte memory request at 64 B on gfx950 (MI355X_MICROARCH.md §HBM); the fat forward reads
    its slots as 128-B requests, so the corrected read traffic is the L2's memory-side read
    requests x 128 B (an upper bound: some requests are 64 B)"""
    achieved = fwd_bytes / (max(fwd_ms, 1e-9) * 1e-3) / 1e9
    out = {"bound": "hbm", "kernel": "forward", "achieved": round(achieved, 1),
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_launch": int(fwd_bytes), "launch_ms": round(fwd_ms, 4),
           "traffic": None}
    if config != "c3":
        return out
    raw = pmc_traffic("k_fm_fwd")
    req = pmc_requests("k_fm_fwd")
    if raw is not None:
        out["traffic_fetch_write_raw"] = raw
    if req is not None:
        out["traffic"] = int(req["rdreq_per_launch"] * 128 + req["wrreq_per_launch"] * 64)
        out["traffic_source"] = ("profiles/%s/pmc_requests.json: TCC_EA0_RDREQ x 128 B + "
                                 "TCC_EA0_WRREQ x 64 B per launch (the guide's 128-B request "
                                 "correction)" % PMC_ROUND)
    return out


def cpu_baseline(args):
    """The reference's CPU hot path restated WITH its threading (oracle/cpu_ref.cc: OpenMP
    row / column splits of SpMV / SpMM, ParallelSort, the two-thread IterateData pipeline, the
    single-threaded unordered_map SGDUpdater of StoreLocal) on a bounded sample of the same
    workload: one untimed count-push epoch, then one timed steady-state epoch per thread count
    over the same rows — 1 thread, the reference's default blk_nthreads_ = 2, and every host
    core this job may use (OMP_NUM_THREADS, else the CPU count)."""
    from difacto_amd import data as D
    from oracle import cpu_ref as C
    cores = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    nb = max(1, args.cpu_rows // args.cpu_batch)
    blocks = [D.synthetic(args.cpu_batch, args.nnz, 1 << args.key_bits, seed=1000 + i)
              for i in range(nb)]
    ref = C.CpuRef(cores, V_dim=args.vdim, V_threshold=0, l1=0, lr=.1, V_lr=.01)
    for b in blocks:
        ref.step(b, push_cnt=True)
    by_threads, phases = {}, {}
    for nt in sorted({1, 2, cores}):
        ref.nt = nt
        C.phases()
        dt, _, _, n = ref.iterate(blocks)
        by_threads[str(nt)] = round(n / dt, 1)
        phases[str(nt)] = {k: round(v / n * 1e6, 3) for k, v in C.phases().items()}
    ref.close()
    # the best thread count is the baseline (on a shared host, all cores is not always the
    # fastest: the single-threaded updater competes with the OpenMP threads)
    best = max(by_threads, key=lambda k: by_threads[k])
    cal = None  # the port against the survey's reference number, in the survey's own container
    try:
        cj = json.load(open(os.path.join(ROOT, "profiles", "r6", "cpu_calibration.json")))
        al = cj["all_V (bench settings)"]["by_threads"]
        cal = {"in_container_vs_survey_2thr_sequential": al["2"]["sequential"]["vs_survey"],
               "in_container_vs_survey_1thr_sequential": al["1"]["sequential"]["vs_survey"],
               "in_container_vs_survey_2thr_pipelined": al["2"]["pipelined"]["vs_survey"],
               "source": "profiles/r6/cpu_calibration.json (tools/cpu_calibrate.py: B=10^4, "
                         "k=39, d=16, 2^24 keys, the bench's updater settings, in the build "
                         "container the survey measured 35.8 k ex/s in)"}
    except (OSError, ValueError, KeyError):
        pass
    return {"value": by_threads[best], "unit": "train examples/sec", "cores": int(best),
            "calibration": cal,
            "cores_available": cores, "kind": "port",
            "by_threads": by_threads,
            "us_per_row_by_phase": phases,
            "vs_survey_2thr": round(by_threads["2"] / 35800.0, 3),
            "sample": "%d rows (%d batches of %d), Criteo-shaped C3, one steady-state epoch per "
                      "thread count after a count-push epoch; oracle/cpu_ref.cc: the reference's "
                      "threading (OpenMP SpMV/SpMM row/column splits, ParallelSort, reader + "
                      "executor threads, single-threaded unordered_map updater)"
                      % (nb * args.cpu_batch, nb, args.cpu_batch)}


def step_window(torch, dev, world, batches, run):
    """The timed window's shape (untimed replay of the same K steps, same barrier + sync
    bracket): one event on the main stream after each step's enqueue, so the K intervals are
    the main stream's time per step — the first holds the Localizer of its batch that no
    earlier step overlapped (the pipeline's fill); the wall time past the last event is the
    drain of the side lanes (the last AUC).  Only the first/last/median are reported."""
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(batches) + 1)]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i, bt in enumerate(batches):
        run(bt)
        evs[i + 1].record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(len(batches))]
    mid = sorted(ms[1:-1] or ms)
    med = mid[len(mid) // 2]
    span = evs[0].elapsed_time(evs[-1])
    return {"steps": len(ms), "first_ms": round(ms[0], 4), "second_ms": round(ms[1], 4)
            if len(ms) > 1 else None, "median_ms": round(med, 4), "last_ms": round(ms[-1], 4),
            "main_span_ms": round(span, 4), "wall_ms": round(wall, 4),
            "fill_ms": round(sum(ms[:2]) - 2 * med, 4) if len(ms) > 1 else None,
            "launch_and_drain_ms": round(wall - span, 4),
            "ms": [round(x, 3) for x in ms]}


def spawn_ranks(args):
    """`--gpus N` without a launcher: run this script as N ranks, one process per GPU, with the
    environment torch.distributed.run gives them (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), and
    exit with the worst rank's status.  Called before anything touches the GPU; rank 0 prints
    the JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    return next((rc for rc in rcs if rc != 0), 0)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s (launch with --nproc-per-node %d, or "
                 "without a launcher)" % (args.gpus, os.environ.get("WORLD_SIZE"), args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":
        local = local % max(1, torch.cuda.device_count())  # ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sharded = world > 1 or args.sharded
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from difacto_amd import hotpath as H
    import ctypes

    prio = args.main_prio or ("high" if sharded else "normal")
    if prio == "high":
        # everything below (the library context takes torch's current stream) on it
        cs = torch.cuda.Stream(device=dev, priority=-1)
        torch.cuda.set_stream(cs)
    if sharded:
        run_sharded(args, torch, dist, dev, rank, world, local)
        dist.destroy_process_group()
        return

    B, k, kb, d = args.batch, args.nnz, args.key_bits, args.vdim
    cf = CONFIGS[args.config]
    keyspace = 1 << kb
    extra = dict(kv.split("=", 1) for kv in args.ctx.split(",") if kv)
    upd = dict(cf["upd"], **{kk: v for kk, v in extra.items() if kk in cf["upd"]})
    extra = {kk: v for kk, v in extra.items() if kk not in upd}
    ctx = H.Context(local, V_dim=d, max_keys=keyspace, max_vrows=keyspace if d > 0 else 0,
                    **upd, **extra)
    ctx.reserve(B, B * k)
    lib = H._lib.lib()

    def step(batch, push_cnt):
        b = batch.as_batch()
        H.check(lib.dfx_train_step(ctx.h, ctypes.byref(b), H.kTraining, int(push_cnt),
                                   ctypes.c_uint64(H.MAX_INDEX), None))

    # Batches come from a loader stream (as a reader's host->device copies would): the
    # library's Localizer lane waits only for that stream, so it overlaps the previous batch's
    # forward / backward on the context stream.  Batches stay referenced until a sync point.
    loader = torch.cuda.Stream(device=dev)
    if not os.environ.get("DFX_SERIAL"):
        ctx.set_input_stream(loader)

    zipf_pool = {}

    def make(seed):
        if cf["zipf"] is not None:
            # host-drawn Zipf ids: a pool of 8 batches, reused (drawing takes ~0.3 s each)
            seed = seed % 8
            if seed not in zipf_pool:
                with torch.cuda.stream(loader):
                    zipf_pool[seed] = DevBatch(torch, dev, B, k, kb, seed, cf["valued"],
                                               cf["zipf"])
            return zipf_pool[seed]
        with torch.cuda.stream(loader):
            return DevBatch(torch, dev, B, k, kb, seed, cf["valued"])

    # untimed epoch 0: touch the key space with count pushes (all keys end up with V)
    n_warm_epoch = max(1, math.ceil(4.6 * keyspace / (B * k)))
    live = []
    warm = [make(1_000_000 * (rank + 1) + i) for i in range(n_warm_epoch)]
    torch.cuda.synchronize()
    tw = time.perf_counter()  # (the cold model's epoch: every key new, reported, not timed)
    for bt in warm:
        live.append(bt)
        step(live[-1], True)
    torch.cuda.synchronize()
    t_warm = time.perf_counter() - tw
    live.clear()
    warm.clear()
    H.progress(ctx)
    for i in range(args.warmup):
        live.append(make(2_000_000 * (rank + 1) + i))
        step(live[-1], False)
    batches = [make(3_000_000 * (rank + 1) + i) for i in range(args.steps)]
    torch.cuda.synchronize()
    live.clear()
    H.prof_read(ctx)
    H.progress(ctx)
    # The timed steps record only the two events around the backward (the roofline's launch
    # time): every timing event adds latency to the step (all eight phase marks and the lane
    # marks cost ~4 %).  The per-phase and lane breakdown comes from an untimed diagnostic
    # pass afterwards.  DFX_NOPROF: no events at all (A/B of their cost; no roofline).
    H.prof_enable(ctx, 0 if os.environ.get("DFX_NOPROF") else args.steps,
                  phases=("backward_update",))

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    H.prof_host(ctx)
    t0 = time.perf_counter()
    for bt in batches:
        step(bt, False)
    t_enq = time.perf_counter() - t0
    host_wait = H.prof_host(ctx)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    phases, nrec, mean_u = H.prof_read(ctx)
    bwd_ms = phases["backward_update"]
    prog = H.progress(ctx)
    window = step_window(torch, dev, world, batches, lambda bt: step(bt, False))
    # the per-step counters restart here: the live-V counts below are the diagnostic pass's
    # alone, and so must be the step count they are divided by (the window's steps counted
    # none of them: a mean over both halved them, and with them the roofline's bytes)
    H.prof_counts(ctx)
    # diagnostic pass (untimed): every phase and the lanes, over the same batches again
    H.prof_enable(ctx, len(batches))
    for bt in batches:
        step(bt, False)
    torch.cuda.synchronize()
    counts = H.prof_counts(ctx)  # live-V keys / occurrences, counted in the diagnostic pass
    phases, nrec_diag, _ = H.prof_read(ctx)
    phases = {p: v * nrec / max(nrec_diag, 1) for p, v in phases.items()}  # per timed step
    phases["backward_update"] = bwd_ms
    lanes = H.prof_lanes(ctx)
    # the host's own cost of a step call, measured on an idle device (a sync before each call:
    # no capacity-guard wait, no full hardware queue to block a launch) — in the timed loop the
    # call time also holds the blocks of a host running ahead of the device
    H.prof_enable(ctx, 0)
    host_idle = []
    for bt in batches[:20]:
        torch.cuda.synchronize()
        t = time.perf_counter()
        step(bt, False)
        host_idle.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    host_idle.sort()
    H.progress(ctx)
    ctx.sync()
    st = H.Store(ctx).stats()

    value = world * B * args.steps / elapsed
    per_launch_ms = {p: phases[p] / max(nrec, 1) for p in phases}
    ab = algorithmic_bytes(B, B * k, mean_u, d, cf["valued"], counts["U_V"], counts["occ_V"])
    dom = max(ab, key=lambda p: per_launch_ms[p])
    achieved = ab[dom] / (max(per_launch_ms[dom], 1e-9) * 1e-3) / 1e9
    pmc_file = "pmc_hbm.json" if args.config == "c3" else "pmc_hbm_%s.json" % args.config
    out = {
        "metric": "train examples/sec (FM V_dim=16) at 1/8 GPU + achieved HBM GB/s",
        "value": round(value, 1),
        "unit": "train examples/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated, resident in HBM before timing)",
        "config": {"workload": (cf["name"] % dict(vdim=d, nnz=k, key_bits=kb))
                               + ", fused dfx_train_step",
                   "config": args.config,
                   "rows_per_gpu_step": B, "global_batch": B * world,
                   "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic(("k_fm_bwd", "k_chunk_hot")
                                            if dom == "backward_update" else "k_fm_fwd",
                                            pmc_file),
                     "traffic_source": "profiles/%s/" % PMC_ROUND + pmc_file +
                                       " (rocprofv3 FETCH_SIZE + "
                                       "WRITE_SIZE per launch, summed over the phase's "
                                       "kernels; request counts per key / nnz "
                                       "in profiles/%s/pmc_requests.json); counters "
                                       "calibrated for these access shapes in "
                                       "profiles/r1/pmc_calibration.json (64-B requests "
                                       "counted exactly, factor 1.00)" % PMC_ROUND,
                     "algorithmic_bytes_per_launch": int(ab[dom]),
                     "launch_ms": round(per_launch_ms[dom], 4)},
        "roofline_forward": forward_roofline(ab["forward"], per_launch_ms["forward"],
                                             args.config),
        "phases_ms_per_step": {p: round(v, 4) for p, v in per_launch_ms.items()},
        "cold_epoch_ms_per_step": round(t_warm / n_warm_epoch * 1e3, 4),
        "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
        # the host's own work per step: the calls' time less their waits on the capacity guard
        # (which lets the host run a few steps ahead of the device, then blocks it)
        "host_busy_ms_per_step": round((t_enq - host_wait["wait_s"]) / args.steps * 1e3, 4),
        "host_waits": host_wait["waits"],
        "host_call_ms_idle_device": round(host_idle[len(host_idle) // 2] * 1e3, 4),
        "lanes_ms": {k_: round(v, 4) for k_, v in lanes.items()},
        "step_window": window,
        "mean_unique_keys": round(mean_u, 1),
        "mean_live_v_keys": counts["U_V"] and round(counts["U_V"], 1),
        "mean_live_v_occurrences": counts["occ_V"] and round(counts["occ_V"], 1),
        "chunk_model": (chunk_model(B * k, mean_u, elapsed / args.steps * 1e3)
                        if args.config == "c3" else None),
        "train_loss_per_row": round(prog["loss"] / max(prog["nrows"], 1), 6),
        "train_auc": round(prog["auc"] / max(prog["nrows"], 1), 6),
        "model_keys": st["n_keys"], "model_vrows": st["n_vrows"],
    }
    if dom == "backward_update" and args.config == "c3":
        # the ceiling of this kernel is the random-line rate, not the byte peak: a key's 144 B
        # of hot state (entry 16, V 64, Vaux 64) is 2 random 128-B line read-modify-writes,
        # and two lines in one 256-B span cost the same as two unrelated ones
        # (tools/membench/spanbench, profiles/r5/spanbench_cold.txt)
        lines = 2 * mean_u / (max(per_launch_ms[dom], 1e-9) * 1e-3)
        out["roofline"]["line_roofline"] = {
            "bound": "random 128-B line read-modify-writes", "achieved": round(lines / 1e9, 2),
            "peak": round(CHUNK_RMW_PER_S / 1e9, 2), "unit": "G lines/s",
            "frac": round(lines / CHUNK_RMW_PER_S, 4),
            "source": "tools/membench/spanbench (cold caches): 3.48 M sorted keys x 2 lines in "
                      "329 us alone; a 256-B-span layout 331 us"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c3":
        out["cpu_baseline"] = cpu_baseline(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def run_sharded(args, torch, dist, dev, rank, world, local):
    """N > 1: data parallel over N GPUs with the model sharded by key range
    (difacto_amd/dist.py; keys / records exchanged with RCCL all-to-all-v over xGMI).
    Weak scaling: B rows per GPU per step."""
    cf = CONFIGS[args.config]
    from difacto_amd import hotpath as H
    from difacto_amd import dist as DI

    B, k, kb, d = args.batch, args.nnz, args.key_bits, args.vdim
    keyspace = 1 << kb
    per = keyspace // world + keyspace // (8 * world) + 4096
    # max_keys sizes the table (cap = pow2 >= 2 * max_keys; a soft bound): the owner's share
    # of the key space, so its table runs at the single-GPU bench's load factor (~0.5);
    # max_vrows (a hard bound) has headroom for an uneven share
    extra = dict(kv.split("=", 1) for kv in args.ctx.split(",") if kv)
    ctx = H.Context(local, V_dim=d, V_threshold=0, l1=0, lr=.1, V_lr=.01,
                    max_keys=max(keyspace // world, 1), max_vrows=per, push_agg=args.push_agg,
                    **extra)
    shard = DI.Shard(ctx, world)
    comm = DI.TorchComm(device=dev, stage_cpu=args.backend == "gloo",
                        force_collectives=args.force_collectives, comm_priority=args.comm_prio)
    # batches come from a loader stream (as a reader's host->device copies would): the
    # worker's first phase (split partition / Localizer) waits only for that stream, not for
    # the compute stream's previous step
    loader = torch.cuda.Stream(device=dev)
    ctx.set_input_stream(loader)

    zipf_pool = {}

    def make(seed):
        if cf["zipf"] is not None:
            # host-drawn Zipf ids: a pool of 8 batches, reused (drawing takes ~0.3 s each)
            seed = seed % 8
            if seed not in zipf_pool:
                with torch.cuda.stream(loader):
                    zipf_pool[seed] = DevBatch(torch, dev, B, k, kb, seed, cf["valued"],
                                               cf["zipf"])
            return zipf_pool[seed]
        with torch.cuda.stream(loader):
            return DevBatch(torch, dev, B, k, kb, seed, cf["valued"])

    host_t = None
    if os.environ.get("DFX_HOSTTIME"):  # host seconds per call of each shard / comm method
        import collections
        host_t = collections.defaultdict(float)

        def timed(obj, name):
            f = getattr(obj, name)

            def w(*a, **kw):
                t = time.perf_counter()
                r = f(*a, **kw)
                host_t[name] += time.perf_counter() - t
                return r
            setattr(obj, name, w)
        for nm in ("localize", "localize_wait", "fwd_bwd", "owner_begin", "owner_pull",
                   "owner_push", "split_partition", "split_partition_wait", "split_owner_begin",
                   "split_owner_forward", "split_combine", "split_owner_backward",
                   "split_initv_local", "split_initv_draw"):
            timed(shard, nm)
        lw = shard.localize_wait

        def lw_probe(*a, **kw):  # was the main stream already drained when the Localizer joined?
            e = torch.cuda.Event()
            e.record()
            r = lw(*a, **kw)
            host_t["main_idle_at_join"] += 1e-3 * float(e.query())
            return r
        shard.localize_wait = lw_probe
        for nm in ("exchange_counts", "exchange_counts2", "alltoallv_async",
                   "alltoallv_keys_async", "allgather_rows", "allgather_i64"):
            timed(comm, nm)
    split = args.collective == "split"
    # the split's C++ driver (libdfx_dist.so) over its own RCCL communicators: the schedule of
    # split_step / SplitPipeline without the interpreter between the launches
    cpp = split and args.driver == "cpp" and args.backend == "nccl"
    store = None
    if cpp:
        ids = torch.zeros(DI.SplitStore.rccl_ids_size(), dtype=torch.uint8)
        if rank == 0:
            ids = torch.frombuffer(bytearray(DI.SplitStore.rccl_ids()), dtype=torch.uint8)
        dist.broadcast(ids, src=0, group=comm.cgroup)
        store = DI.SplitStore([shard], pipelined=not args.sync, stale=args.stale and not args.sync,
                              rccl=(rank, world, ids.numpy().tobytes(), args.force_collectives))
        if args.slices:
            store.set_slices(args.slices)
        pipe = None
    elif args.sync:
        pipe = None
    elif split:
        pipe = DI.SplitPipeline([shard], comm)
    else:
        pipe = DI.ShardedPipeline([shard], comm)
    live = []  # a batch stays alive until the submit after the one that took it
    sync_fn = DI.split_step if split else DI.sharded_step

    def step(batch, push_cnt, mark=None):
        if store is not None:
            store.submit([batch], H.kTraining, push_cnt=push_cnt)
        elif pipe is None:
            sync_fn([shard], [batch], comm, H.kTraining, push_cnt=push_cnt, mark=mark)
        else:
            pipe.submit([batch], H.kTraining, push_cnt=push_cnt, mark=mark)
            live.append(batch)
            del live[:-3]

    n_warm_epoch = max(1, math.ceil(4.6 * keyspace / (world * B * k)))
    for i in range(n_warm_epoch):
        step(make(1_000_000 * (rank + 1) + i), True)
    for i in range(args.warmup):
        step(make(2_000_000 * (rank + 1) + i), False)
    if pipe is not None:
        pipe.flush()
    if store is not None:
        store.flush()
    batches = [make(3_000_000 * (rank + 1) + i) for i in range(args.steps)]
    torch.cuda.synchronize()
    H.progress(ctx)
    # per-phase events on the stream everything is ordered on (torch's current stream: the
    # library's kernels and the wait on each RCCL collective).  In the pipelined schedule
    # the phases of neighbouring steps overlap; the marks are in issue order.
    nph = len(DI.SPLIT_PHASES if split else DI.PHASES)
    # Timing events add latency to the step, so the timed steps record only the two marks
    # around the roofline's kernels (split: the owner's backward + its InitV; a2a: the worker's
    # forward+backward); the per-phase breakdown comes from an untimed diagnostic pass over the
    # same batches afterwards.
    FB = ((6, 7) if pipe is None and store is None else (3, 4)) if split else (4, 5)

    def run_steps(js):
        if store is not None:  # the driver's own events at its main-stream boundaries
            store.set_marks([j + 1 for j in js if j < DI.SplitStore.MARKS - 1])
            for bt in batches:
                step(bt, False)
            store.flush()
            store.set_marks([])
            return None
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(nph + 1)]
               for _ in range(args.steps)]

        def marker(e):
            return lambda j: e[j + 1].record() if j in js else None
        for i, bt in enumerate(batches):
            if pipe is None:
                step(bt, False, mark=marker(evs[i]))
            else:  # a submit runs the previous batch's step
                step(bt, False, mark=marker(evs[i - 1]) if i else None)
        if pipe is not None:
            pipe.flush(mark=marker(evs[-1]))
        return evs

    if host_t is not None:
        host_t.clear()
    prof = None
    if os.environ.get("DFX_PYPROF") and rank == 0:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    dist.barrier()
    torch.cuda.synchronize()
    if isinstance(pipe, DI.SplitPipeline):
        pipe.throttle_s = 0.0
    if store is not None:
        store.throttle_seconds()
    t0 = time.perf_counter()
    evs = run_steps(FB)
    t_enq = time.perf_counter() - t0
    # the host's own work per step: enqueue time less its waits on the run-ahead bound
    t_busy = t_enq - (pipe.throttle_s if isinstance(pipe, DI.SplitPipeline) else
                      store.throttle_seconds() if store is not None else 0.0)
    if host_t is not None:
        print("host ms/step", {k_: round(v / args.steps * 1e3, 4) for k_, v in host_t.items()},
              file=sys.stderr, flush=True)
        host_t.clear()
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.environ["DFX_PYPROF"])
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=comm.cgroup)
    elapsed = float(t.item())
    # the worker's forward+backward launch pair (pipelined: including the wait for the record
    # exchange, so `achieved` is a lower bound)
    if store is not None:
        v, n = store.take_marks()["owner_backward"]
        fb_ms = v / max(n, 1)
    else:
        fb_ms = sum(evs[i][FB[0] + 1].elapsed_time(evs[i][FB[1] + 1])
                    for i in range(args.steps)) / args.steps
    prog = H.progress(ctx)

    # diagnostic pass (untimed): every phase
    evs = run_steps(range(-1, nph))
    torch.cuda.synchronize()
    if store is not None:
        ph = {p: v / max(n, 1) for p, (v, n) in store.take_marks().items()}
    else:
        if split:
            names = DI.SPLIT_PHASES if pipe is None else DI.SPLIT_PIPE_PHASES
        else:
            names = DI.PHASES if pipe is None else DI.PIPE_PHASES
        ph = {p: sum(evs[i][j].elapsed_time(evs[i][j + 1]) for i in range(args.steps))
              / args.steps for j, p in enumerate(names)}
    H.progress(ctx)
    # the other collective schedules on the same batches, bulk synchronous (short runs): the
    # all-to-all-v step, and the north_star's literal union all-gather / reduce-scatter
    # (dist.rsag_step) — the measured baseline of the exchange design
    colls = {}
    if pipe is not None:
        pipe.flush()
    if split:  # the owner's share of the last step, for the roofline's bytes
        o_rows, o_nnz, o_uniq = shard.split_owner_stats(0)
    nb = min(args.steps, 20)
    main_name = (("split_sync" if args.sync else "split_pipelined") if split else
                 ("a2a_sync" if args.sync else "a2a_pipelined"))
    if store is not None:
        main_name += "_cpp"
    if store is not None and args.stale and not args.sync:
        main_name = "split_stale_cpp"
    py_pipe = [None]

    def py_split_pipelined(shards, dblks, comm_, job):
        if py_pipe[0] is None:
            py_pipe[0] = DI.SplitPipeline(shards, comm_)
        py_pipe[0].submit(dblks, job)

    def cpp_other_slices(shards, dblks, comm_, job):
        store.submit(dblks, job)

    sched = [("split_sync", DI.split_step), ("a2a_sync", DI.sharded_step),
             ("rsag_sync", DI.rsag_step)]
    if store is not None and not args.sync:  # the same schedule driven from Python
        sched.insert(0, ("split_pipelined_py", py_split_pipelined))
        # the C++ driver with the other slicing (rows in 2 slices, each slice's exchanges
        # beside the next slice's compute; or unsliced if the main run was sliced)
        other_k = 1 if args.slices > 1 else 2
        if not args.stale:  # (the stale schedule runs unsliced)
            sched.insert(1, ("split_pipelined_cpp_slices%d" % other_k, cpp_other_slices))
    for cname, fn in sched:
        if cname == main_name or (cname != "a2a_sync" and args.push_agg != "sum"):
            continue
        if fn is cpp_other_slices:
            store.set_slices(other_k)
        for bt in batches[:2]:
            fn([shard], [bt], comm, H.kTraining)
        if py_pipe[0] is not None:
            py_pipe[0].flush()
        if fn is cpp_other_slices:
            store.flush()
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for bt in batches[:nb]:
            fn([shard], [bt], comm, H.kTraining)
        if py_pipe[0] is not None:
            py_pipe[0].flush()
            py_pipe[0] = None
        if fn is cpp_other_slices:
            store.flush()
            store.set_slices(args.slices)
        torch.cuda.synchronize()
        dist.barrier()
        dt = time.perf_counter() - t1
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=comm.cgroup)
        dt = float(t.item())
        colls[cname] = {"ms_per_step": round(dt / nb * 1e3, 4),
                        "value": round(world * B * nb / dt, 1), "steps": nb}
    used_cpp = store is not None
    if store is not None and not args.sync and args.push_agg == "sum":
        # the C++ driver's other pipelined schedule on the same batches, so that one N-GPU run
        # reports both: the pipelined default (bulk-synchronous results) beside the 1-step-stale
        # one (each step's exchanges beside the other step's compute; DESIGN.md (e) predicts
        # ~0.8 of the fused step per GPU at N = 8 against ~0.7) — or the default when --stale
        # ran the main line.  A store of its own (its own RCCL communicators) on the same shard.
        other_stale = not args.stale
        store.flush()
        store.close()
        store = None
        ids2 = torch.zeros(DI.SplitStore.rccl_ids_size(), dtype=torch.uint8)
        if rank == 0:
            ids2 = torch.frombuffer(bytearray(DI.SplitStore.rccl_ids()), dtype=torch.uint8)
        dist.broadcast(ids2, src=0, group=comm.cgroup)
        st2 = DI.SplitStore([shard], pipelined=True, stale=other_stale,
                            rccl=(rank, world, ids2.numpy().tobytes(), args.force_collectives))
        for bt in batches[:2]:
            st2.submit([bt], H.kTraining)
        st2.flush()
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for bt in batches[:nb]:
            st2.submit([bt], H.kTraining)
        st2.flush()
        torch.cuda.synchronize()
        dist.barrier()
        dt = time.perf_counter() - t1
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=comm.cgroup)
        dt = float(t.item())
        colls["split_stale_cpp" if other_stale else "split_pipelined_cpp"] = {
            "ms_per_step": round(dt / nb * 1e3, 4), "value": round(world * B * nb / dt, 1),
            "steps": nb}
        st2.close()
    H.progress(ctx)
    ctx.sync()
    st = H.Store(ctx).stats()
    tot = comm.allreduce_sum([[prog["loss"], prog["auc"], prog["nrows"], float(st["n_keys"]),
                               float(st["n_vrows"]), float(max(shard._U))]])[0]
    if split:
        # roofline of the owner's fused backward + update on this rank (the fused step's
        # backward formula over the owner's rows, keys and unique keys)
        ab = algorithmic_bytes(o_rows, o_nnz, o_uniq, d)["backward_update"]
        rkernel = "owner_backward (split: fused backward + FTRL/AdaGrad + InitV, rank 0)"
        traffic, tsrc = (pmc_traffic(("k_fm_bwd", "k_chunk_hot"), "pmc_hbm_split.json"),
                         "profiles/%s/pmc_hbm_split.json (rocprofv3 FETCH_SIZE + WRITE_SIZE "
                         "per launch of the owner's backward, bench.py --sharded)" % PMC_ROUND)
    else:
        # roofline of the worker's forward+backward launch pair on this rank
        ab = algorithmic_bytes_sharded(B, B * k, max(shard._U), d)
        rkernel = "fwd_bwd (dist forward+AUC+backward, rank 0)"
        traffic, tsrc = sharded_traffic(), ("profiles/r1/pmc_hbm_sharded.json (rocprofv3 "
                                            "FETCH_SIZE + WRITE_SIZE per launch of the "
                                            "worker's forward and backward, N = 1 sharded "
                                            "bench)")
    achieved = ab / (fb_ms * 1e-3) / 1e9
    value = world * B * args.steps / elapsed
    out = {
        "metric": "train examples/sec (FM V_dim=16) at 1/8 GPU + achieved HBM GB/s",
        "value": round(value, 1),
        "unit": "train examples/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (device-generated, resident in HBM before timing)",
        "config": {"workload": "C3 Criteo-shaped FM V_dim=%d, %d binary nnz/row, 2^%d keys, "
                               "l1=0 V_threshold=0, key-range-sharded store over %d GPUs, %s, "
                               "push_agg=%s"
                               % (d, k, kb, world,
                                  "owner-computes split (RCCL all-to-all of per-row partials "
                                  "+ all-gather of [XV*p | p] rows), %s"
                                  % ("bulk-synchronous" if args.sync else
                                     "1-step-stale (step t+1's owner forward before step t's "
                                     "backward, the exchanges beside the other step's compute)"
                                     if args.stale and used_cpp else
                                     "bulk-synchronous results, next step's partition / key "
                                     "exchange / owner Localizer on the Localizer lane")
                                  if split else
                                  "RCCL all-to-all-v of records / gradients, %s schedule"
                                  % ("bulk-synchronous" if args.sync
                                     else "pipelined 1-step-stale"),
                                  args.push_agg),
                   "rows_per_gpu_step": B, "global_batch": B * world,
                   "parallelism": "dp%d + model sharded by key range" % world,
                   "driver": "cpp (libdfx_dist.so)" if used_cpp else "python"},
        "roofline": {"bound": "hbm", "kernel": rkernel,
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": tsrc,
                     "algorithmic_bytes_per_launch": int(ab),
                     "launch_ms": round(fb_ms, 4)},
        "phases_ms_per_step_rank0": {p: round(v, 4) for p, v in ph.items()},
        "collectives": dict({main_name:
                             {"ms_per_step": round(elapsed / args.steps * 1e3, 4),
                              "value": round(value, 1), "steps": args.steps}}, **colls),
        "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
        "host_busy_ms_per_step": round(t_busy / args.steps * 1e3, 4),
        "train_loss_per_row": round(tot[0] / max(tot[2], 1), 6),
        "train_auc": round(tot[1] / max(tot[2], 1), 6),
        "model_keys": int(tot[3]), "model_vrows": int(tot[4]),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if store is not None:
        store.close()
    ctx.close()


if __name__ == "__main__":
    main()
