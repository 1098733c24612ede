// The fused minibatch: the body of SGDLearner::IterateData's executor
// (src/sgd/sgd_learner.cc:201-317) with StoreLocal's inline Pull/Push, run entirely on the
// device with no host round trip:
//
//   localize (sort/unique/remap)          Localizer::Compact        localizer.cc:11-107
//   [Update(kFeaCount) + InitV]           epoch 0, V_dim > 0        sgd_learner.cc:272,304-307
//   resolve + pull {w, V offset}          SGDUpdater::Get           sgd_updater.cc:34-58
//   forward (pred, p, XV*p, loss)         FMLoss::Predict/Evaluate  fm_loss.h:67-119
//   AUC                                   BinClassMetric::AUC       bin_class_metric.h:35-57
//   backward fused with FTRL/AdaGrad      CalcGrad + Update         fm_loss.h:148-203,
//                                                                   sgd_updater.cc:76-142
//   InitV for keys whose w left zero      sgd_updater.cc:118-121,144-152
//
// Every grid is sized from host-known B and nnz; U lives on the device, so a step needs no
// host round trip.  It is not captured into a hipGraph: the host enqueues a step in ~0.16 ms
// against a ~0.8 ms GPU step, and a replayed graph would serialise the
// Localizer lane of step t + 1 behind step t.

#include "fm_args.h"

namespace dfx {
void sum_parts(Context* c, const double* part, int64_t n, double* out, bool accumulate);
}

namespace dfx {

// Row stride of the fused step's XV_*p rows: a multiple of 32 floats (128 B) carrying p after
// XV_*p, so the backward's per-occurrence p and XV_*p sit in one 128-byte line (+3 % of the
// step at d = 16, same-box A/B against rows of d floats with p apart).  At d a multiple of 32 p
// would fill a 128-byte line of its own: the rows are d floats and the backward reads p from
// the per-row array (fm.hip row_p), which stays in the L2
int xvp_stride(const Context* c) {
  const int d = c->P.V_dim;
  return (d > 0 && d % 32 != 0) ? (d + 1 + 31) / 32 * 32 : d;
}

// main lane: per-row arrays of the forward / backward and the InitV scan
int ws_reserve(Context* c, int64_t rows, int64_t nnz) {
  Workspace& ws = c->ws;
  const int d = c->P.V_dim;
  if (rows < 1) rows = 1;
  if (nnz < 1) nnz = 1;
  DFX_TRY(ws.flags.ensure((nnz + 1) * 4));
  DFX_TRY(ws.tiles.ensure(sizeof(uint32_t) * ((nnz + 2047) / 2048 + 1)));
  DFX_TRY(ws.p.ensure(rows * 4));
  DFX_TRY(ws.pred.ensure(rows * 4));
  if (d > 0) DFX_TRY(ws.XVp.ensure((size_t)rows * xvp_stride(c) * 4));
  DFX_TRY(ws.dscratch.ensure((rows / 4 + 64) * 8));
  DFX_TRY(ws.wv.ensure(nnz * 8));
  DFX_TRY(ws.Vb.ensure((size_t)max_chunks(nnz) * (d + 2) * 8));  // chunk partials (f64)
  ws.rows = rows;
  ws.nnz = nnz;
  return DFX_OK;
}

// a Localizer lane: its sort buffers and per-nnz / per-key outputs
int loc_reserve(Workspace& w, int64_t nnz, hipStream_t st) {
  if (nnz < 1) nnz = 1;
  DFX_TRY(w.keys0.ensure(nnz * 8));
  DFX_TRY(w.keys1.ensure(nnz * 8));
  DFX_TRY(w.vals0.ensure(nnz * 8));
  DFX_TRY(w.vals1.ensure(nnz * 8));
  DFX_TRY(w.os_reserve((nnz + 2047) / 2048, st));
  DFX_TRY(w.tiles.ensure(sizeof(uint32_t) * ((nnz + 2047) / 2048 + 1)));
  DFX_TRY(w.segstart.ensure((nnz + 1) * 4));
  DFX_TRY(w.col.ensure(nnz * 4));
  DFX_TRY(w.uniq.ensure(nnz * 8));
  DFX_TRY(w.flags.ensure((nnz + 1) * 4));                   // chunk plan: choff
  DFX_TRY(w.rowtmp.ensure(max_chunks(nnz) * 4));      // chunk plan: chunk_seg
  DFX_TRY(w.slot.ensure((nnz + 1) * 4));
  DFX_TRY(w.occ_row.ensure(nnz * 4));
  DFX_TRY(w.occ_x.ensure(nnz * 4));
  w.nnz = nnz;
  return DFX_OK;
}

// the AUC lane (metric.hip auc_finish): the snapshot (keys ak0, labels av0) and the merge
// ping-pong buffers (u64 keys, u32 labels)
int auc_reserve(Workspace& w, int64_t rows, hipStream_t st) {
  if (rows < 1) rows = 1;
  if (w.rows >= rows && w.ak0.p) return DFX_OK;
  DFX_TRY(w.ak0.ensure(rows * 4));
  DFX_TRY(w.av0.ensure(rows * 4));
  DFX_TRY(w.keys0.ensure(rows * 8));
  DFX_TRY(w.keys1.ensure(rows * 8));
  DFX_TRY(w.vals0.ensure(rows * 4));
  DFX_TRY(w.vals1.ensure(rows * 4));
  DFX_TRY(w.os_reserve((rows + 2047) / 2048, st));  // the radix sort's look-back words
  w.rows = rows;
  return DFX_OK;
}

// the fused step's AUC snapshot double-buffered: a forward waits (through the Localizer lane's
// join) only for the AUC of two steps back.  At B <= kAucBlockMax the one-block AUC (~94 us
// beside the backward) outlasts the rest of a small step (B = 10^4: 58.6 / 61.6 -> 68.0 / 68.8
// M ex/s, round 4); since round 6 at every size (two boxes, ABBA, driver command: C2 200.6 ->
// 206.1 and 202.0 -> 207.4, C3 132.0 -> 130.7 (one outlier) and 140.2 -> 142.0, C5 a tie;
// round 4 had measured B = 10^5 a tie with the wait on the main stream)
static bool auc_db_on(const Context*, int64_t) { return true; }

int step_reserve(Context* c, int64_t rows, int64_t nnz) {
  DFX_TRY(pipeline_init(c));
  DFX_TRY(ws_reserve(c, rows, nnz));
  DFX_TRY(loc_reserve(c->bws[0], nnz, c->loc_stream));
  DFX_TRY(loc_reserve(c->bws[1], nnz, c->loc_stream));
  if (auc_db_on(c, rows)) DFX_TRY(auc_reserve(c->aws_alt, rows, c->aux_stream));
  return auc_reserve(c->aws, rows, c->aux_stream);
}

// SGDUpdater::Get (sgd_updater.cc:34-58) over the batch's sorted unique keys, as the
// reference's Pull does: find-or-insert each key (model_[key]), record its slot for the
// backward and its {w, vrow} for the forward (pulled[rank]; the forward reaches it through
// col).  In a count-push step the slots come first and the pull follows the push's InitV.
// Keys arrive in sorted order; kProbeUnr home slots are read at once (latency-bound loop).
constexpr int kProbeNT = 256, kProbeUnr = 4;
__global__ __launch_bounds__(kProbeNT) void k_probe_keys(const uint64_t* __restrict__ uniq,
                                                         const DevState* nds, Table T,
                                                         int2* __restrict__ pulled,
                                                         uint32_t* __restrict__ segslot,
                                                         DevState* ds) {
  __shared__ int red[kProbeNT / kWave];
  const int64_t n = (int64_t)nds->u_count;
  const int64_t ub = (int64_t)blockIdx.x * kProbeNT * kProbeUnr + threadIdx.x;
  uint64_t key[kProbeUnr], h[kProbeUnr];
  unsigned long long kk[kProbeUnr];
  int2 wr[kProbeUnr];
  int ins = 0;
#pragma unroll
  for (int v = 0; v < kProbeUnr; ++v) {
    const int64_t u = ub + (int64_t)v * kProbeNT;
    key[v] = u < n ? uniq[u] : 0ull;
    h[v] = tbl_hash(key[v], T);
  }
#pragma unroll
  for (int v = 0; v < kProbeUnr; ++v) {
    const int64_t u = ub + (int64_t)v * kProbeNT;
    if (u < n) {
      kk[v] = ent_at(T, h[v])->key;
      wr[v] = *reinterpret_cast<const int2*>(ent_at(T, h[v]));
    }
  }
#pragma unroll
  for (int v = 0; v < kProbeUnr; ++v) {
    const int64_t u = ub + (int64_t)v * kProbeNT;
    if (u >= n) continue;
    int64_t s = (int64_t)h[v];
    if (kk[v] != key[v]) {
      bool inserted;
      s = tbl_insert(T, key[v], &inserted);
      ins += inserted ? 1 : 0;
      if (s < 0) {  // the key reads as absent and is never updated (kNoSlot)
        atomicOr(&ds->err, insert_error(s));
        wr[v] = make_int2(0, -1);
      } else {
        wr[v] = *reinterpret_cast<const int2*>(ent_at(T, s));
      }
    }
    segslot[u] = s < 0 ? kNoSlot : (uint32_t)s;
    if (pulled) pulled[u] = wr[v];
  }
  for (int off = 32; off > 0; off >>= 1) ins += __shfl_xor(ins, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = ins;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < kProbeNT / kWave; ++i) t += red[i];
    if (t) atomicAdd(&ds->n_keys, (unsigned long long)t);
  }
}

// find-or-insert of a lane's sorted unique keys (u_count of the lane's state) into segslot
int probe_keys_run(Context* c, const Lane& L, int64_t bound, const uint64_t* uniq,
                   uint32_t* segslot) {
  if (bound <= 0) return DFX_OK;
  const dim3 ug((unsigned)((bound + kProbeNT * kProbeUnr - 1) / (kProbeNT * kProbeUnr)));
  hipLaunchKernelGGL(k_probe_keys, ug, dim3(kProbeNT), 0, L.stream, uniq, L.ds, c->T, nullptr,
                     segslot, c->ds);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}


__global__ __launch_bounds__(kFinNT) void k_step_finalize(FinArgs f) {
  __shared__ double red[kFinNT / kWave];
  step_finalize_body<kFinNT>(f, red);
}

// the fused backward's striped {new_w, n_keys} folded into the state (k_step_finalize's first
// part) when a step ends on an error after its backward was enqueued: the counts then reach
// dfx_store_stats and the capacity guard at once, not in a later step's finalize
__global__ __launch_bounds__(kWave) void k_fold_stripes(DevState* ds) {
  unsigned long long nw = 0, nk = 0;
  if (threadIdx.x < kBwStripes) {
    unsigned long long* st = ds->bw_stripe[threadIdx.x];
    nw = st[0];
    nk = st[1];
    st[0] = 0ull;
    st[1] = 0ull;
  }
  for (int off = 32; off > 0; off >>= 1) {
    nw += __shfl_xor(nw, off, kWave);
    nk += __shfl_xor(nk, off, kWave);
  }
  if (threadIdx.x == 0) {
    if (nw) atomicAdd((unsigned long long*)&ds->new_w, nw);
    if (nk) atomicAdd(&ds->n_keys, nk);
  }
}

static int fold_stripes_on_error(Context* c, int rc) {
  hipLaunchKernelGGL(k_fold_stripes, dim3(1), dim3(kWave), 0, c->stream, c->ds);
  (void)hipGetLastError();
  return rc;
}

// One minibatch, pipelined over three streams:
//   loc lane   Localizer (transform + find-or-insert, sort, segments) of this batch.  It needs
//              only the batch and the key -> slot map, which the backward never changes
//              (inserts only claim empty slots; the backward writes values), so it runs while
//              the main stream is still on the previous batch's forward / backward.  Its
//              buffers alternate between two sets (parity), each reused only after the main
//              stream finished the batch that used it before.
//   main       [count push] -> forward -> backward + FTRL/AdaGrad -> InitV: reads the model
//              strictly after the previous batch's update, so results equal the sequential
//              schedule exactly (SGDLearner::IterateData with StoreLocal).
//   aux lane   AUC of a snapshot of (pred, label) taken on the main stream, beside the
//              backward; it adds into the progress itself and is joined by the next step's
//              snapshot (and by dfx_progress_read / dfx_sync).
int train_step(Context* c, const dfx_batch* b, int job_type, int push_cnt, uint64_t max_index,
               float* pred_out) {
  const int64_t B = b->size, nnz = b->nnz;
  const int d = c->P.V_dim;
  DFX_TRY(step_reserve(c, B, nnz));
  // this step inserts at most nnz keys and draws at most nnz V rows: grow the store first if
  // they might not fit (at a sync point; in the steady state the check costs no wait)
  DFX_TRY(cap_check(c, nnz));
  Workspace& ws = c->ws;
  const int k = c->parity;
  c->parity ^= 1;
  Workspace& bw = c->bws[k];
  DevState* bds = c->bds[k];
  const Lane LL{c->loc_stream, &bw, bds, &c->ds->err};
  // the AUC snapshot's buffers: one, or two alternating (auc_db)
  // (the form switches with B: a single-buffered step uses buffer 0 and waits for the latest
  // AUC; every step records which AUC last read its buffer)
  const bool db = auc_db_on(c, B);
  const int ap = db ? c->auc_par : 0;
  Workspace& aw = ap ? c->aws_alt : c->aws;
  hipEvent_t ev_auc_mine = db ? c->ev_auc_p[ap] : c->ev_auc;
  if (db) c->auc_par ^= 1;
  const Lane AL{c->aux_stream, &aw, c->ads, &c->ds->err};
  uint32_t* segstart = bw.segstart.as<uint32_t>();
  uint64_t* uniq = bw.uniq.as<uint64_t>();     // per rank: the key
  uint32_t* segslot = bw.slot.as<uint32_t>();  // per rank: its model-table slot
  uint32_t* occ_row = bw.occ_row.as<uint32_t>();
  float* occ_x = b->value ? bw.occ_x.as<float>() : nullptr;
  uint32_t* flags = ws.flags.as<uint32_t>();
  uint32_t* total = &c->ds->totals[0];
  float* pred = pred_out ? pred_out : ws.pred.as<float>();

  // ---- loc lane: the batch is ready on the caller's stream; this parity's buffers are free
  // once the main stream finished the batch that used them before
  DFX_HIP(hipEventRecord(c->ev_in, c->has_in_stream ? c->in_stream : c->stream));
  DFX_HIP(hipStreamWaitEvent(c->loc_stream, c->ev_in, 0));
  DFX_HIP(hipStreamWaitEvent(c->loc_stream, c->slot_free[k] ? c->slot_free[k] : c->ev_free[k], 0));
  // Localizer::Compact: sorted unique keys (segments in key order, the order Update walks
  // keys in — InitV draws — and, per key, the (row, nnz) order of its gradient sums)
  LocOut o;
  o.segstart = segstart;
  o.value = b->value;
  o.occ_row = occ_row;
  o.occ_x = occ_x;
  o.col = nullptr;  // probe mode: the forward finds keys itself
  o.uniq = uniq;
  const uint2* rowof = c->loc_rowof[k];  // (lb_gather=2) kept with the parity's outputs
  o.rowof_out = &rowof;
  lane_mark(c, 0, c->loc_stream);
  uint32_t* choff = bw.flags.as<uint32_t>();
  uint32_t* chunk_seg = bw.rowtmp.as<uint32_t>();
  uint32_t* nchunks = &bds->totals[1];
  if (!((c->diag & 2) && c->loc_done[k])) {  // (diag: measurement only)
    rowof = nullptr;
    c->lb_skip = c->loc_done[k] ? (c->lb_diag & (16 | 32 | 64 | 128 | 256 | 512)) : 0;  // (measurement only)
    DFX_TRY(localize_run(c, LL, B, nnz, b->offset, b->index, max_index, o));
    c->lb_skip = 0;
    c->loc_rowof[k] = rowof;
    // long segments (skewed keys) get reduced in chunks: plan them here, off the main stream
    DFX_TRY(chunk_plan(LL, nnz, segstart, choff, chunk_seg, nchunks));
    c->loc_done[k] = true;
  }
  lane_mark(c, 1, c->loc_stream);
  // the forward writes the AUC lane's snapshot of (pred, label), whose buffers are free once the
  // AUC that last read them is done: the lane joins that AUC before it hands its batch over, so
  // the main stream waits on one event instead of two (a cross-stream wait costs the stream that
  // waits ~4 us, tools/membench/waitbench.hip; the AUC ends long before this lane does)
  DFX_HIP(hipStreamWaitEvent(c->loc_stream, ev_auc_mine, 0));
  DFX_HIP(hipEventRecord(c->ev_loc[k], c->loc_stream));

  // Get over the sorted unique keys (find-or-insert + pull); a count push goes in between
  const bool cnt_first = push_cnt && d > 0;
  // a training step whose forward finds keys itself needs no Get pass: absent keys read as
  // the empty entry and the backward inserts them (its find-or-insert is Get's)
  const bool bwd_inserts = !cnt_first && job_type == DFX_JOB_TRAINING &&
                           B > 0 && nnz > 0;
  // ---- main: wait for this batch's Localizer (the exposed part of it is the "localize" phase).
  // (The probe forward needs only the batch, but a forward that waits for the batch alone and
  // the backward for the Localizer measured worse: same box, driver command, 139.0 / 138.3 /
  // 130.7 -> 133.6 / 125.5 / 126.3 M ex/s — the fill shrinks 0.26 -> 0.05 ms, but the lane then
  // runs beside the backward instead of the forward and ends 0.04-0.16 ms before it is needed)
  prof_mark(c, 0);
  DFX_HIP(hipStreamWaitEvent(c->stream, c->ev_loc[k], 0));
  prof_mark(c, 1);
  const dim3 ug((unsigned)((nnz + kProbeNT * kProbeUnr - 1) / (kProbeNT * kProbeUnr)));
  if (nnz > 0 && !bwd_inserts)
    hipLaunchKernelGGL(k_probe_keys, ug, dim3(kProbeNT), 0, c->stream, uniq, bds, c->T,
                       nullptr, segslot, c->ds);
  prof_mark(c, 2);
  if (cnt_first) {
    DFX_TRY(push_cnt_seg_run(c, nnz, segstart, segslot, flags, total, bds));
  }
  prof_mark(c, 3);

  FwdArgs a{};
  a.B = B; a.offs = b->offset; a.val = b->value;
  a.index = b->index; a.max_index = max_index;  // probe mode: the forward finds its keys
  a.T = c->T; a.l1_shrk = c->P.l1_shrk; a.Vbase = c->T.V; a.zpad = c->zpad;
  a.no_fat_fwd = !c->fat_fwd;
  a.cpl = c->fwd_cpl;
  a.lr_lanes = c->lr_lanes;
  a.nt = c->nt_mask;
  a.d = d; a.label = b->label; a.rw = b->weight; a.pred = pred; a.p_out = ws.p.as<float>();
  a.XVp = ws.XVp.as<float>(); a.xs = xvp_stride(c);
  a.loss_part = ws.dscratch.as<double>() + 8;
  // the forward writes the AUC lane's snapshot of (pred, label) (free: ev_loc joined the AUC
  // that last read it).  (A last-block loss reduction inside the forward cost more than the
  // launch it saves: the device-scope fence of each block writes back its XCD's L2.)
  a.auc_key = aw.ak0.as<uint32_t>();
  a.auc_lab = aw.av0.as<uint32_t>();
  int nblk = 0;
  DFX_TRY(launch_fwd_fused(a, c->stream, &nblk, true));
  prof_mark(c, 4);
  // (the forward's loss partials are summed by k_step_finalize, the step's last kernel)

  // ---- aux lane: AUC of this batch's predictions, beside the backward.  Started from the
  // event of phase mark 5 (the backward's start, after the chunk kernels): one record where a
  // separate ev_fwd and mark cost ~5 us of the main stream each (tools/membench/waitbench.hip)
  auto auc_lane = [&]() -> int {
    const hipEvent_t e = prof_mark_or(c, 5, c->ev_fwd);
    DFX_HIP(hipStreamWaitEvent(c->aux_stream, e, 0));
    lane_mark(c, 2, c->aux_stream);
    if (!(c->diag & 1)) DFX_TRY(auc_finish(AL, B, &c->ds->prog[2], true, c->auc_sort));
    lane_mark(c, 3, c->aux_stream);
    DFX_HIP(hipEventRecord(c->ev_auc, c->aux_stream));  // the lane's latest (syncs join it)
    DFX_HIP(hipEventRecord(c->ev_auc_p[ap], c->aux_stream));  // this buffer's last reader
    ++c->auc_seq_p[ap];
    return DFX_OK;
  };

  const bool bwd_runs = job_type == DFX_JOB_TRAINING && B > 0 && nnz > 0;
  const bool initv = bwd_runs && d > 0;
  // the step's last work: folded into the InitV launch when one runs (its last block), else a
  // kernel of its own
  FinArgs fin;
  fin.ds = c->ds; fin.bds = bds; fin.B = B; fin.initv_total = initv ? total : nullptr;
  fin.d = d; fin.vcap = c->T.vcap; fin.loss_part = a.loss_part; fin.nparts = nblk;
  if (bwd_runs) {
    BwdArgs g{};
    g.segstart = segstart; g.ds = bds; g.nseg_host = -1; g.segcol = nullptr;
    g.occ_row = occ_row; g.occ_x = occ_x; g.occ_rx = rowof; g.zpad = c->zpad;
    g.p = ws.p.as<float>();
    g.XVp = ws.XVp.as<float>(); g.xs = xvp_stride(c); g.d = d; g.slot = segslot;
    g.T = c->T; g.Pm = c->P;  g.cpl = c->bwd_cpl; g.cpl_from = c->bwd_cpl_from; g.nt = c->nt_mask;
    g.flags = flags; g.dsw = c->ds; g.stripes = &c->ds->bw_stripe[0][0];
    g.uniq = uniq; g.insert_keys = bwd_inserts ? 1 : 0;
    g.choff = choff; g.chunk_seg = chunk_seg; g.nchunks = nchunks; g.part = ws.Vb.as<double>();
    // (diagnostic, dfx_prof_enable_marks bit 9) the live-V key / occurrence counts
    const bool count_live = c->prof_n < c->prof_max && (c->prof_mask >> 9 & 1u);
    DFX_TRY(bwd_two_pass_reserve(c, ws, nnz, &g));
    const int64_t nbb = bwd_fused_blocks(d, nnz, g.vlist != nullptr, g.cpl | g.cpl_from << 8);
    if (count_live) {
      DFX_TRY(ws.live.ensure((size_t)nbb * sizeof(uint2)));
      g.live_part = ws.live.as<uint2>();
    }
    DFX_TRY(launch_bwd_chunks(g, max_chunks(nnz), c->stream, true));
    DFX_TRY(auc_lane());
    DFX_TRY(launch_bwd_fused(g, nnz, c->stream, c->bwd_lds));
    if (count_live) DFX_TRY(sum_live(g.live_part, nbb, c->ds, c->stream));
    prof_mark(c, 6);
  } else {
    DFX_TRY(auc_lane());
    prof_mark(c, 6);
  }
  {
    const int rc = cap_record_slot(c, &fin.cap_host);
    if (rc != DFX_OK) return bwd_runs ? fold_stripes_on_error(c, rc) : rc;
  }
  if (initv) {
    const int rc = run_initv(c, -1, nnz, flags, total, segslot, bds, &c->ds->n_init, false, &fin);
    if (rc != DFX_OK) return fold_stripes_on_error(c, rc);
  } else {
    hipLaunchKernelGGL(k_step_finalize, dim3(1), dim3(kFinNT), 0, c->stream, fin);
  }
  // this parity's buffers are free past here: the capacity guard's step event when it records
  // one, else ev_free (one record, not two)
  hipEvent_t fe = nullptr;
  DFX_TRY(cap_record_commit(c, &fe));
  if (!fe) {
    DFX_HIP(hipEventRecord(c->ev_free[k], c->stream));
    fe = c->ev_free[k];
  }
  c->slot_free[k] = fe;
  prof_mark(c, 7);
  if (c->prof_n < c->prof_max) ++c->prof_n;
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

}  // namespace dfx

using namespace dfx;

extern "C" int dfx_train_step(dfx_ctx* ctx, const dfx_batch* batch, int job_type, int push_cnt,
                              uint64_t max_index, float* pred_out) {
  DFX_CHECK_ARG(ctx && batch, "null argument");
  DFX_CHECK_ARG(batch->size >= 0 && batch->nnz >= 0, "train_step: negative sizes");
  DFX_CHECK_ARG(batch->size == 0 || (batch->offset && batch->label), "train_step: null buffer");
  DFX_CHECK_ARG(batch->nnz == 0 || batch->index, "train_step: null index");
  DFX_CHECK_ARG(job_type == DFX_JOB_TRAINING || job_type == DFX_JOB_VALIDATION ||
                    job_type == DFX_JOB_PREDICTION,
                "train_step: bad job type");
  return train_step(&ctx->c, batch, job_type, push_cnt, max_index, pred_out);
}

// ---- phase timing ----------------------------------------------------------------------
extern "C" int dfx_prof_enable(dfx_ctx* ctx, int max_steps) {
  return dfx_prof_enable_marks(ctx, max_steps, ~0u);
}

extern "C" int dfx_prof_enable_marks(dfx_ctx* ctx, int max_steps, unsigned mask) {
  DFX_CHECK_ARG(ctx && max_steps >= 0, "bad argument");
  Context* c = &ctx->c;
  c->prof_mask = mask;
  DFX_HIP(hipStreamSynchronize(c->stream));
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  c->prof_ev.assign((size_t)max_steps * kProfMarks, nullptr);
  for (auto& e : c->prof_ev) DFX_HIP(hipEventCreate(&e));
  for (hipEvent_t e : c->lane_ev) (void)hipEventDestroy(e);
  c->lane_ev.assign((size_t)max_steps * 4, nullptr);
  for (auto& e : c->lane_ev) DFX_HIP(hipEventCreate(&e));
  c->prof_max = max_steps;
  c->prof_n = 0;
  return DFX_OK;
}

// ms[7]: summed milliseconds of localize (wait), probe+pull, feacnt, forward, eval (the AUC
// lane's launch and, in a training step, the chunk kernels), backward+update, initv+finalize
// over the recorded steps; *n_steps their count; *mean_u the mean U per step over all
// dfx_train_step calls since the last read.  Resets the recording.
// after dfx_prof_read: out[4] = mean ms of the Localizer lane per batch, of its start after
// the context stream reached that batch (negative: it ran ahead), of its end after that point
// (positive: the exposed wait), and of the AUC lane
// out[4]: per dfx_train_step since the last call, the mean number of unique keys, of keys with
// live V (their V is read and updated) and of those keys' occurrences; then the number of
// batches the bucket Localizer placed by its hot-key map; resets the counters
extern "C" int dfx_prof_counts(dfx_ctx* ctx, double* out) {
  DFX_CHECK_ARG(ctx && out, "bad argument");
  Context* c = &ctx->c;
  double h[2];
  unsigned long long lv[2];
  DFX_HIP(hipMemcpyAsync(h, &c->ds->sum_u, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipMemcpyAsync(lv, &c->ds->live_keys, sizeof(lv), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  const double n = h[1] > 0 ? h[1] : 1;
  out[0] = h[0] / n;
  out[1] = (double)lv[0] / n;
  out[2] = (double)lv[1] / n;
  DFX_HIP(hipMemsetAsync(&c->ds->sum_u, 0, sizeof(h), c->stream));
  DFX_HIP(hipMemsetAsync(&c->ds->live_keys, 0, sizeof(lv), c->stream));
  // the Localizer lanes' hot-key map use (their own states; the lane is drained first)
  if (c->loc_stream) DFX_HIP(hipStreamSynchronize(c->loc_stream));
  out[3] = 0;
  for (DevState* s : c->bds) {
    if (!s) continue;
    unsigned m = 0;
    DFX_HIP(hipMemcpy(&m, &s->lb_map_steps, sizeof(unsigned), hipMemcpyDeviceToHost));
    DFX_HIP(hipMemset(&s->lb_map_steps, 0, sizeof(unsigned)));
    out[3] += (double)m;
  }
  DFX_HIP(hipStreamSynchronize(c->stream));
  return DFX_OK;
}

// out[2]: host seconds dfx_train_step calls spent waiting (the capacity guard's waits on
// earlier steps' counts, store.hip cap_check) since the last call, and the number of waits;
// resets.  The rest of a call's time is the host's own work of enqueueing the step.
extern "C" int dfx_prof_host(dfx_ctx* ctx, double* out) {
  DFX_CHECK_ARG(ctx && out, "bad argument");
  out[0] = ctx->c.host_wait_s;
  out[1] = (double)ctx->c.host_waits;
  ctx->c.host_wait_s = 0;
  ctx->c.host_waits = 0;
  return DFX_OK;
}

extern "C" int dfx_prof_lanes(dfx_ctx* ctx, double* out) {
  DFX_CHECK_ARG(ctx && out, "bad argument");
  for (int i = 0; i < 4; ++i) out[i] = ctx->c.lane_stats[i];
  return DFX_OK;
}

extern "C" int dfx_prof_read(dfx_ctx* ctx, double* ms, int* n_steps, double* mean_u) {
  DFX_CHECK_ARG(ctx && ms, "bad argument");
  Context* c = &ctx->c;
  DFX_HIP(hipStreamSynchronize(c->stream));
  for (int m = 0; m < kProfMarks - 1; ++m) ms[m] = 0;
  for (int s = 0; s < c->prof_n; ++s) {
    for (int m = 0; m < kProfMarks - 1; ++m) {
      if ((c->prof_mask >> m & 3u) != 3u) continue;  // a mark of this phase not recorded
      float t = 0;
      DFX_HIP(hipEventElapsedTime(&t, c->prof_ev[(size_t)s * kProfMarks + m],
                                  c->prof_ev[(size_t)s * kProfMarks + m + 1]));
      ms[m] += t;
    }
  }
  // lanes: mean Localizer-lane time, its start relative to the main stream's wait for it,
  // the main stream's wait past its end, mean AUC-lane time
  for (double& v : c->lane_stats) v = 0;
  if (c->loc_stream) DFX_HIP(hipStreamSynchronize(c->loc_stream));
  if (c->aux_stream) DFX_HIP(hipStreamSynchronize(c->aux_stream));
  const bool lanes = (c->prof_mask >> kProfMarks & 1u) && (c->prof_mask & 1u);
  for (int s = 0; s < c->prof_n && !c->lane_ev.empty() && lanes; ++s) {
    hipEvent_t* L = &c->lane_ev[(size_t)s * 4];
    hipEvent_t* M = &c->prof_ev[(size_t)s * kProfMarks];
    float t[4] = {0, 0, 0, 0};
    DFX_HIP(hipEventElapsedTime(&t[0], L[0], L[1]));
    DFX_HIP(hipEventElapsedTime(&t[1], M[0], L[0]));
    DFX_HIP(hipEventElapsedTime(&t[2], M[0], L[1]));
    DFX_HIP(hipEventElapsedTime(&t[3], L[2], L[3]));
    for (int i = 0; i < 4; ++i) c->lane_stats[i] += t[i] / c->prof_n;
  }
  if (n_steps) *n_steps = c->prof_n;
  c->prof_n = 0;
  double h[2];
  DFX_HIP(hipMemcpyAsync(h, &c->ds->sum_u, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  if (mean_u) *mean_u = h[1] > 0 ? h[0] / h[1] : 0;
  // the counters are the context stream's (k_step_finalize): zeroed in its order
  DFX_HIP(hipMemsetAsync(&c->ds->sum_u, 0, sizeof(h), c->stream));
  DFX_HIP(hipMemsetAsync(&c->ds->live_keys, 0, 2 * sizeof(unsigned long long), c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  return DFX_OK;
}
