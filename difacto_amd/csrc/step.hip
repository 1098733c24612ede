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
// Every grid is sized from host-known B and nnz; U lives on the device, so the sequence is
// capturable into a hipGraph once dfx_reserve has sized the workspace.

#include "fm_args.h"

namespace dfx {
void sum_parts(Context* c, const double* part, int64_t n, double* out, bool accumulate);
}

namespace dfx {

int ws_reserve(Context* c, int64_t rows, int64_t nnz) {
  Workspace& ws = c->ws;
  const int d = c->P.V_dim;
  if (rows < 1) rows = 1;
  if (nnz < 1) nnz = 1;
  const int64_t ntiles = (nnz + 2047) / 2048;
  DFX_TRY(ws.keys0.ensure(nnz * 8));
  DFX_TRY(ws.keys1.ensure(nnz * 8));
  DFX_TRY(ws.vals0.ensure(nnz * 8));
  DFX_TRY(ws.vals1.ensure(nnz * 8));
  DFX_TRY(ws.wv.ensure(nnz * 8));
  DFX_TRY(ws.os_reserve((nnz + kOsSortTile - 1) / kOsSortTile));
  DFX_TRY(ws.rowid.ensure(nnz * 4));
  DFX_TRY(ws.tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  DFX_TRY(ws.segstart.ensure((nnz + 1) * 4));
  DFX_TRY(ws.col.ensure(nnz * 4));
  DFX_TRY(ws.slot.ensure((nnz + 1) * 4));
  DFX_TRY(ws.flags.ensure((nnz + 1) * 4));
  DFX_TRY(ws.occ_row.ensure(nnz * 4));
  DFX_TRY(ws.occ_x.ensure(nnz * 4));
  DFX_TRY(ws.p.ensure(rows * 4));
  DFX_TRY(ws.pred.ensure(rows * 4));
  if (d > 0) DFX_TRY(ws.XVp.ensure((size_t)rows * d * 4));
  DFX_TRY(ws.dscratch.ensure((rows / 4 + 64) * 8));
  DFX_TRY(ws.ak0.ensure(rows * 4));
  DFX_TRY(ws.ak1.ensure(rows * 4));
  DFX_TRY(ws.av0.ensure(rows * 4));
  DFX_TRY(ws.av1.ensure(rows * 4));
  const int64_t at = (rows + 2047) / 2048;
  DFX_TRY(ws.atiles.ensure(at * 4 + at * 8 + 64));
  ws.rows = rows;
  ws.nnz = nnz;
  return DFX_OK;
}

__global__ void k_step_finalize(DevState* ds, int64_t B, int train) {
  // sgd::Progress: nrows, loss, auc (sgd_learner.cc:213-229)
  ds->prog[0] += (double)B;
  ds->prog[1] += ds->scratch[3];
  ds->prog[2] += ds->auc_n;
  ds->sum_u += (double)ds->u_count;
  ds->n_steps += 1;
  (void)train;
}

int train_step(Context* c, const dfx_batch* b, int job_type, int push_cnt, uint64_t max_index,
               float* pred_out) {
  const int64_t B = b->size, nnz = b->nnz;
  const int d = c->P.V_dim;
  Workspace& ws = c->ws;
  DFX_TRY(ws_reserve(c, B, nnz));
  uint32_t* segstart = ws.segstart.as<uint32_t>();
  uint32_t* nslot = ws.col.as<uint32_t>();   // per nnz: model-table slot of its key
  uint32_t* segslot = ws.slot.as<uint32_t>();  // per unique key (sorted): its slot
  uint32_t* flags = ws.flags.as<uint32_t>();
  uint32_t* total = &c->ds->totals[0];
  float* pred = pred_out ? pred_out : ws.pred.as<float>();
  uint32_t* occ_row = ws.occ_row.as<uint32_t>();
  float* occ_x = b->value ? ws.occ_x.as<float>() : nullptr;

  prof_mark(c, 0);
  // Localizer::Compact + the pull's key resolution: each nnz's key is found-or-inserted in
  // the model table (Get's model_[key], sgd_updater.cc:37); segments come out in sorted key
  // order, which is the order Update walks keys in (InitV draws) and the (row, nnz) order of
  // every key's gradient sum.
  // Without a count push nothing changes the table between this probe and the forward, so
  // the probe hands each nnz's {w, vrow} straight to it; a count push (epoch 0) may InitV
  // first, so the forward then re-reads the entry by slot.
  const bool cnt_first = push_cnt && d > 0;
  LocOut o;
  o.segstart = segstart;
  o.value = b->value;
  o.occ_row = occ_row;
  o.occ_x = occ_x;
  o.segslot = segslot;
  if (cnt_first) {
    o.nslot = nslot;
  } else {
    o.wv = ws.wv.as<int2>();
  }
  DFX_TRY(localize_run(c, B, nnz, b->offset, b->index, max_index, o));
  prof_mark(c, 1);
  if (cnt_first) DFX_TRY(push_cnt_seg_run(c, nnz, segstart, segslot, flags, total));
  prof_mark(c, 2);
  prof_mark(c, 3);  // the pull is the forward's direct read of each key's table entry

  FwdArgs a{};
  a.B = B; a.offs = b->offset; a.col = nslot; a.wv = cnt_first ? nullptr : ws.wv.as<int2>();
  a.val = b->value; a.T = c->T;
  a.l1_shrk = c->P.l1_shrk; a.Vbase = c->T.V; a.zpad = c->zpad;
  a.d = d; a.label = b->label; a.rw = b->weight; a.pred = pred; a.p_out = ws.p.as<float>();
  a.XVp = ws.XVp.as<float>();
  a.loss_part = ws.dscratch.as<double>() + 8;
  int nblk = 0;
  DFX_TRY(launch_fwd_fused(a, c->stream, &nblk));
  prof_mark(c, 4);
  sum_parts(c, a.loss_part, nblk, &c->ds->scratch[3], false);
  DFX_TRY(auc_run(c, B, b->label, pred, &c->ds->auc_n));
  prof_mark(c, 5);

  if (job_type == DFX_JOB_TRAINING && B > 0 && nnz > 0) {
    BwdArgs g{};
    g.segstart = segstart; g.ds = c->ds; g.nseg_host = -1; g.segcol = nullptr;
    g.occ_row = occ_row; g.occ_x = occ_x; g.zpad = c->zpad; g.p = ws.p.as<float>();
    g.XVp = ws.XVp.as<float>(); g.d = d; g.slot = segslot; g.T = c->T; g.Pm = c->P;
    g.flags = flags; g.dsw = c->ds;
    DFX_TRY(launch_bwd_fused(g, nnz, c->stream));
    prof_mark(c, 6);
    DFX_TRY(run_initv(c, -1, nnz, flags, total, segslot));
  } else {
    prof_mark(c, 6);
  }
  hipLaunchKernelGGL(k_step_finalize, dim3(1), dim3(1), 0, c->stream, c->ds, B,
                     job_type == DFX_JOB_TRAINING);
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
  DFX_CHECK_ARG(ctx && max_steps >= 0, "bad argument");
  Context* c = &ctx->c;
  DFX_HIP(hipStreamSynchronize(c->stream));
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  c->prof_ev.assign((size_t)max_steps * kProfMarks, nullptr);
  for (auto& e : c->prof_ev) DFX_HIP(hipEventCreate(&e));
  c->prof_max = max_steps;
  c->prof_n = 0;
  return DFX_OK;
}

// ms[7]: summed milliseconds of localize, feacnt, pull, forward, auc+eval, backward+update,
// initv+finalize over the recorded steps; *n_steps their count; *mean_u the mean U per step
// over all dfx_train_step calls since the last read.  Resets the recording.
extern "C" int dfx_prof_read(dfx_ctx* ctx, double* ms, int* n_steps, double* mean_u) {
  DFX_CHECK_ARG(ctx && ms, "bad argument");
  Context* c = &ctx->c;
  DFX_HIP(hipStreamSynchronize(c->stream));
  for (int m = 0; m < kProfMarks - 1; ++m) ms[m] = 0;
  for (int s = 0; s < c->prof_n; ++s) {
    for (int m = 0; m < kProfMarks - 1; ++m) {
      float t = 0;
      DFX_HIP(hipEventElapsedTime(&t, c->prof_ev[(size_t)s * kProfMarks + m],
                                  c->prof_ev[(size_t)s * kProfMarks + m + 1]));
      ms[m] += t;
    }
  }
  if (n_steps) *n_steps = c->prof_n;
  c->prof_n = 0;
  double h[2];
  DFX_HIP(hipMemcpy(h, &c->ds->sum_u, sizeof(h), hipMemcpyDeviceToHost));
  if (mean_u) *mean_u = h[1] > 0 ? h[0] / h[1] : 0;
  DFX_HIP(hipMemset(&c->ds->sum_u, 0, sizeof(h)));
  return DFX_OK;
}
