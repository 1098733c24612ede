// Context lifecycle, .conf-key parsing, device memory helpers and error plumbing.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <vector>

#include "internal.h"

namespace dfx {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int DevBuf::ensure(size_t n) {
  if (n == 0) n = 16;
  if (n <= bytes) return DFX_OK;
  if (p) {
    DFX_HIP(hipFree(p));
    p = nullptr;
    bytes = 0;
  }
  size_t want = n + n / 4;  // headroom so ragged batches do not reallocate each step
  DFX_HIP(hipMalloc(&p, want));
  bytes = want;
  return DFX_OK;
}

void DevBuf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}

// SGDUpdaterParam / FMLossParam defaults (sgd_param.h:109-122, fm_loss.h:25)
static void default_params(Params* P) {
  P->l1 = 1; P->l2 = 0; P->V_l2 = .01f; P->lr = .01f; P->lr_beta = 1; P->V_lr = .01f;
  P->V_lr_beta = 1; P->V_init_scale = .01f; P->V_dim = 0; P->V_threshold = 10; P->l1_shrk = 1;
}

struct Kw {
  Params P;
  unsigned seed = 0;
  long long max_keys = 1ll << 22;
  long long max_vrows = -1;
  int loss_fm = 1;
  int ordered = 1;
  // execution choices (context kwargs, not behaviour switches of the process environment)
  long bwd_lds = -1;    // bwd_lds=<bytes>: LDS reserved per backward block (-1: default cap)
  int autogrow = 1;     // autogrow=0: never grow the table / V pool on its own
  int dist_sum = 1;     // push_agg=sum|ranks (sharded store, dist.hip)
  int sort_pack = 1;    // sort_pack=0: the Localizer sorts 12-byte (key, row) pairs
  // auc_sort=radix (default): the AUC lane's onesweep radix passes; merge: tile sorts + merge
  // rounds (round 4's bucket AUC, a shorter lane but a slower step, is gone: DESIGN.md (d))
  int auc_sort = 1;
  // slot_layout=auto (default): fat slots (entry + V in one 64/128-byte slot, common.h Table)
  // when V_dim allows them (4 <= d <= 24, d % 4 == 0), else the split layout; split | fat force
  int slot_layout = -1;
  int fat_fwd = 1;  // fat_fwd=0: with fat slots, the split forward walk (A/B of the one-trip read)
  // diag=noauc|noloc|noauc_noloc: MEASUREMENT ONLY (the headroom of the side lanes): no AUC
  // lane, or each Localizer parity run once and its output reused (results are then wrong
  // unless the batches repeat); never set by the product path
  int diag = 0;
  // lr_lanes=1 (default): the LR forward (V_dim 0) on four lanes per row with a chunk's entry
  // loads in flight together (fm.hip fwd_probe_body, d == 0); 0: one thread per row
  int lr_lanes = 1;
  // loc_bucket=1 (default): the Localizer of the fused step and of the split owner (no col) as a
  // bucket sort — histogram, scatter into key-range buckets, one LDS sort per bucket
  // (locbucket.hip); 0: the onesweep radix sort's LSD passes (localize.hip, sort.hip)
  int loc_bucket = 1;
  // lb_diag=<bits>: MEASUREMENT ONLY (tools/locbench): parts of k_lb_wbucket skipped — 1 the LDS
  // sort, 4 the outputs, 8 k_lb_scatter's row search; launches skipped on a workspace that holds
  // an earlier batch of the same shape — 16 k_lb_scatter, 32 k_lb_wbucket, 64 k_lb_out; 128
  // k_lb_scatter's items written by input position to a scratch buffer, 256 to the scratch buffer
  // at tile-local positions (the tile's items grouped by bucket; binary batches); the
  // Localizer's results are then wrong
  int lb_diag = 0;
  // lb_gather: valued batches sort (key | position) items alone, the row and the value gathered
  // by position at the outputs (1; A/B at C2: 126 -> 161 M ex/s) or, in the fused step, read by
  // position in the backward itself (2, the default: no gather launch on the Localizer lane;
  // C2 187.5-194.5 -> 195.1-195.5 M ex/s, four same-box rounds); 0: {value, row} carried
  // beside each item
  int lb_gather = 2;
  int lb_hnt = 0;  // lb_hnt=256|512|1024: its histogram / scatter blocks' threads (0: auto,
                   // 512 for valued batches, 1024 for binary ones)
  // nt=<mask>: streaming (non-temporal) cache policy for 1 the Localizer lane's sort passes and
  // transform, 2 the backward's model-table lines, 4 the forward's, 8 the backward's
  // per-occurrence arrays (common.h ld4 / st4)
  int nt = 0;
  // bwd_two_pass=1: the wide-V_dim (V_dim >= 128) fused backward in two passes (fm.hip
  // k_fm_bwd_w / _v, bit-identical; A/B with the hot keys' chunk sums: C5 65.7 -> 92.3 M ex/s,
  // the default); 0: one kernel
  int bwd_two_pass = 1;
  // bwd_cpl=8: the fused backward at V_dim >= 64 with 8 coordinates per lane (half the lanes
  // per key: G = d / 8), bit-identical (every coordinate's terms and order are a lane's own);
  // 4: one float4 per lane (d / 4 lanes per key, capped at 64)
  int bwd_cpl = 8;
  // fwd_cpl=8: the probe forward at V_dim >= 64 with two float4 of V per lane (bit-identical;
  // same-box A/B: C5 63.5 -> 65.7 M ex/s, forward 0.30 -> 0.23 ms; C4 shard a tie); 4: one
  int fwd_cpl = 8;
  int bwd_cpl_from = 64;  // bwd_cpl_from=<V_dim>: the least V_dim (multiple of 8) bwd_cpl=8 takes
  // loc_xpay=0: valued 16-byte items carry the position and the write pass gathers the value
  // (A/B; 1: the value's bits ride in the payload, read by the transform in input order)
  int loc_xpay = 1;
  int strict = 0;     // strict=1: unknown kwargs are an error
};

static int parse_kwargs(const char* kwargs, Kw* kw) {
  default_params(&kw->P);
  if (!kwargs) return DFX_OK;
  std::string s(kwargs);
  for (char& ch : s)
    if (ch == ',' || ch == ';' || ch == '\n' || ch == '\t') ch = ' ';
  std::istringstream is(s);
  std::string tok, unknown;
  while (is >> tok) {
    auto eq = tok.find('=');
    if (eq == std::string::npos) continue;
    std::string k = tok.substr(0, eq), v = tok.substr(eq + 1);
    const char* cv = v.c_str();
    auto f = [&]() { return strtof(cv, nullptr); };
    if (k == "l1") kw->P.l1 = f();
    else if (k == "l2") kw->P.l2 = f();
    else if (k == "V_l2") kw->P.V_l2 = f();
    else if (k == "lr") kw->P.lr = f();
    else if (k == "lr_beta") kw->P.lr_beta = f();
    else if (k == "V_lr") kw->P.V_lr = f();
    else if (k == "V_lr_beta") kw->P.V_lr_beta = f();
    else if (k == "V_init_scale") kw->P.V_init_scale = f();
    else if (k == "V_dim") kw->P.V_dim = atoi(cv);
    else if (k == "V_threshold") kw->P.V_threshold = atoi(cv);
    else if (k == "l1_shrk") kw->P.l1_shrk = !(v == "0" || v == "false");
    else if (k == "seed") kw->seed = (unsigned)strtoul(cv, nullptr, 10);
    else if (k == "max_keys") kw->max_keys = atoll(cv);
    else if (k == "max_vrows") kw->max_vrows = atoll(cv);
    else if (k == "bwd_lds") kw->bwd_lds = atol(cv);
    else if (k == "autogrow") kw->autogrow = atoi(cv) != 0;
    else if (k == "sort_pack") kw->sort_pack = atoi(cv) != 0;
    else if (k == "fat_fwd") kw->fat_fwd = atoi(cv) != 0;
    else if (k == "diag") {
      if (v == "noauc") kw->diag = 1;
      else if (v == "noloc") kw->diag = 2;
      else if (v == "noauc_noloc") kw->diag = 3;
      else { set_error("unknown diag: " + v + " (noauc|noloc|noauc_noloc)"); return DFX_ERR_ARG; }
    }
    else if (k == "loc_bucket") kw->loc_bucket = atoi(cv) != 0;
    else if (k == "lb_diag") kw->lb_diag = atoi(cv);
    else if (k == "lb_gather") kw->lb_gather = atoi(cv) < 0 ? 0 : (atoi(cv) > 2 ? 2 : atoi(cv));
    else if (k == "lb_hnt") kw->lb_hnt = atoi(cv);
    else if (k == "lr_lanes") kw->lr_lanes = atoi(cv) != 0;
    else if (k == "bwd_two_pass") kw->bwd_two_pass = atoi(cv);
    else if (k == "bwd_cpl_from") kw->bwd_cpl_from = atoi(cv);
    else if (k == "fwd_cpl") {
      kw->fwd_cpl = atoi(cv);
      if (kw->fwd_cpl != 4 && kw->fwd_cpl != 8) {
        set_error("fwd_cpl must be 4 or 8");
        return DFX_ERR_ARG;
      }
    }
    else if (k == "bwd_cpl") {
      kw->bwd_cpl = atoi(cv);
      if (kw->bwd_cpl != 4 && kw->bwd_cpl != 8 && kw->bwd_cpl != 16) {
        set_error("bwd_cpl must be 4, 8 or 16");
        return DFX_ERR_ARG;
      }
    }
    else if (k == "loc_xpay") kw->loc_xpay = atoi(cv) != 0;
    else if (k == "nt") {
      kw->nt = atoi(cv);
      if (kw->nt < 0 || kw->nt > 15) {
        set_error("nt must be a mask of 1, 2, 4, 8");
        return DFX_ERR_ARG;
      }
    }
    else if (k == "slot_layout") {
      if (v == "auto") kw->slot_layout = -1;
      else if (v == "split") kw->slot_layout = 0;
      else if (v == "fat") kw->slot_layout = 1;
      else { set_error("unknown slot_layout: " + v + " (auto|split|fat)"); return DFX_ERR_ARG; }
    }
    else if (k == "auc_sort") {
      if (v == "radix") kw->auc_sort = 1;
      else if (v == "merge") kw->auc_sort = 0;
      else { set_error("unknown auc_sort: " + v + " (radix|merge)"); return DFX_ERR_ARG; }
    }
    else if (k == "push_agg") {
      if (v == "sum") kw->dist_sum = 1;
      else if (v == "ranks") kw->dist_sum = 0;
      else { set_error("unknown push_agg: " + v + " (sum|ranks)"); return DFX_ERR_ARG; }
    }
    else if (k == "hash") {
      if (v == "ordered") kw->ordered = 1;
      else if (v == "mixed") kw->ordered = 0;
      else { set_error("unknown hash: " + v + " (ordered|mixed)"); return DFX_ERR_ARG; }
    }
    else if (k == "loss") {
      if (v == "fm") kw->loss_fm = 1;
      else if (v == "logit") kw->loss_fm = 0;
      else { set_error("unknown loss: " + v + " (fm|logit)"); return DFX_ERR_ARG; }
    }
    else if (k == "strict") kw->strict = atoi(cv) != 0;
    else {
      // unknown keys are ignored (dmlc::Parameter::InitAllowUnknown: the C++ adapters pass the
      // learner's kwargs through) unless strict=1 (the Python mirror sets it): a misspelt or
      // retired kwarg must not silently run the default there
      unknown += (unknown.empty() ? "" : ", ") + k;
    }
  }
  if (kw->strict && !unknown.empty()) {
    set_error("unknown context kwargs: " + unknown);
    return DFX_ERR_ARG;
  }
  if (kw->P.V_dim < 0 || kw->P.V_dim > 1024) {
    set_error("V_dim must be in [0, 1024]");
    return DFX_ERR_ARG;
  }
  if (!kw->loss_fm) kw->P.V_dim = 0;  // LogitLoss ignores V (logit_loss.h)
  if (kw->slot_layout == 1 && fat_es(kw->P.V_dim) == 0) {
    set_error("slot_layout=fat needs 4 <= V_dim <= 24 with V_dim % 4 == 0");
    return DFX_ERR_ARG;
  }
  return DFX_OK;
}

// store allocation: table capacity = next pow2 >= 2*n_keys (load factor <= 0.5)
int table_alloc(Context* c, int64_t n_keys, int64_t n_vrows);
void table_release(Context* c);

static void release_ws(Workspace& w) {
  DevBuf* bufs[] = {&w.keys0, &w.keys1, &w.vals0, &w.vals1, &w.rowid, &w.hist, &w.tiles,
                    &w.uniq, &w.cnt, &w.segstart, &w.col, &w.slot, &w.flags, &w.wb, &w.Vb,
                    &w.vpos, &w.p, &w.pred, &w.XVp, &w.rowtmp, &w.dscratch, &w.os, &w.wv,
                    &w.occ_row, &w.occ_x, &w.ak0, &w.ak1, &w.av0, &w.av1,
                    &w.oflags, &w.ofrank, &w.osegstart, &w.osegslot, &w.oseg_of, &w.osorted,
                    &w.ivstat, &w.live, &w.hstat, &w.vlist, &w.lbcnt, &w.lbq, &w.lbsplit, &w.cptiles};
  for (DevBuf* b : bufs) b->release();
  if (w.lb_hint) (void)hipHostFree(w.lb_hint);
  w.lb_hint = nullptr;
}

// streams, events and lane states of the fused step's pipeline, created on first use
int pipeline_init(Context* c) {
  if (c->loc_stream) return DFX_OK;
  // the side lanes run latency-bound chains of small launches beside a full-occupancy
  // backward: the AUC lane gets priority so its workgroups are not queued behind its tail;
  // the Localizer lane, which has a step of slack, runs at the context stream's priority (the
  // sharded bench runs its compute on a high-priority stream: a Localizer lane below it
  // starved, 108 -> 70 M ex/s).  The other assignments were measured in rounds 2-4 (DESIGN.md
  // (d)) and pruned as kwargs in round 6
  int lo = 0, hi = 0;
  DFX_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  (void)lo;
  int main_prio = 0;
  if (hipStreamGetPriority(c->stream, &main_prio) != hipSuccess) main_prio = 0;
  DFX_HIP(hipStreamCreateWithPriority(&c->loc_stream, hipStreamNonBlocking, main_prio));
  DFX_HIP(hipStreamCreateWithPriority(&c->aux_stream, hipStreamNonBlocking, hi));
  c->own_loc_stream = c->loc_stream;
  DFX_HIP(hipStreamCreateWithPriority(&c->part_stream, hipStreamNonBlocking, hi));
  c->own_part_stream = c->part_stream;
  for (hipEvent_t* e : {&c->ev_in, &c->ev_fwd, &c->ev_auc, &c->ev_auc_p[0], &c->ev_auc_p[1]})
    DFX_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  for (int s = 0; s < kSlots; ++s)
    for (hipEvent_t* e : {&c->ev_loc[s], &c->ev_free[s], &c->ev_part[s]})
      DFX_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  std::vector<DevState**> states{&c->ads};
  for (int s = 0; s < kSlots; ++s) {
    states.push_back(&c->bds[s]);
    states.push_back(&c->ods[s]);
  }
  for (DevState** d : states) {
    DFX_HIP(hipMalloc(d, sizeof(DevState)));
    DFX_HIP(hipMemsetAsync(*d, 0, sizeof(DevState), c->stream));
  }
  // complete the zeroing before any lane (a non-blocking stream) can run
  DFX_HIP(hipStreamSynchronize(c->stream));
  for (auto& h : c->dist_host)
    DFX_HIP(hipHostMalloc(reinterpret_cast<void**>(&h), (kMaxDistRanks + 2) * 8,
                          hipHostMallocDefault));
  return DFX_OK;
}

}  // namespace dfx

using namespace dfx;

extern "C" {

const char* dfx_last_error(void) { return g_last_error.c_str(); }

int dfx_ctx_create(int device, const char* kwargs, dfx_ctx** out) {
  DFX_CHECK_ARG(out, "dfx_ctx_create: null out");
  Kw kw;
  DFX_TRY(parse_kwargs(kwargs, &kw));
  int ndev = 0;
  DFX_HIP(hipGetDeviceCount(&ndev));
  if (device < 0) device = 0;
  DFX_CHECK_ARG(device < ndev, "dfx_ctx_create: no such device");
  DFX_HIP(hipSetDevice(device));
  dfx_ctx* ctx = new dfx_ctx();
  Context* c = &ctx->c;
  c->device = device;
  c->P = kw.P;
  c->loss_fm = kw.loss_fm;
  c->bwd_lds = kw.bwd_lds;
  c->autogrow = kw.autogrow;
  c->dist_sum = kw.dist_sum;
  c->sort_pack = kw.sort_pack;
  c->auc_sort = kw.auc_sort;
  c->slot_es = kw.slot_layout == 0 ? 0 : fat_es(c->P.V_dim);
  c->fat_fwd = kw.fat_fwd;
  c->nt_mask = kw.nt;
  c->bwd_two_pass = kw.bwd_two_pass;
  c->bwd_cpl = kw.bwd_cpl;
  c->bwd_cpl_from = kw.bwd_cpl_from;
  c->fwd_cpl = kw.fwd_cpl;
  c->loc_x_payload = kw.loc_xpay;
  c->lr_lanes = kw.lr_lanes;
  c->diag = kw.diag;
  c->loc_bucket = kw.loc_bucket;
  c->lb_diag = kw.lb_diag;
  c->lb_hnt = kw.lb_hnt;
  c->lb_gather = kw.lb_gather;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    set_error("hipStreamCreate failed");
    return DFX_ERR_HIP;
  }
  c->stream = c->own_stream;
  if (hipMalloc(&c->ds, sizeof(DevState)) != hipSuccess) {
    (void)hipStreamDestroy(c->own_stream);
    delete ctx;
    set_error("hipMalloc(DevState) failed");
    return DFX_ERR_HIP;
  }
  if (hipMalloc(&c->zpad, kZpadFloats * sizeof(float)) != hipSuccess ||
      hipMemsetAsync(c->zpad, 0, kZpadFloats * sizeof(float), c->stream) != hipSuccess) {
    set_error("hipMalloc(zpad) failed");
    dfx_ctx_destroy(ctx);
    return DFX_ERR_HIP;
  }
  DevState init;
  memset(&init, 0, sizeof(init));
  init.seed = kw.seed;
  (void)hipMemcpy(c->ds, &init, sizeof(init), hipMemcpyHostToDevice);
  int64_t vrows = kw.max_vrows >= 0 ? kw.max_vrows : (c->P.V_dim > 0 ? kw.max_keys : 0);
  c->T.ordered = kw.ordered;
  c->T.range_mul = 1;
  c->T.probe_flag = &c->ds->probe_flag;
  int rc = table_alloc(c, kw.max_keys, vrows);
  if (rc != DFX_OK) {
    dfx_ctx_destroy(ctx);
    return rc;
  }
  // the zpad memset and the table's initialisation done before any other stream runs
  if (hipDeviceSynchronize() != hipSuccess) {
    set_error("dfx_ctx_create: device synchronisation failed");
    dfx_ctx_destroy(ctx);
    return DFX_ERR_HIP;
  }
  *out = ctx;
  return DFX_OK;
}

int dfx_ctx_destroy(dfx_ctx* ctx) {
  if (!ctx) return DFX_OK;
  Context* c = &ctx->c;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  release_ws(c->ws);
  for (int s = 0; s < kSlots; ++s) {
    release_ws(c->bws[s]);
    release_ws(c->ows[s]);
  }
  release_ws(c->aws);
  release_ws(c->aws_alt);
  release_ws(c->uws);
  for (auto h : c->dist_host)
    if (h) (void)hipHostFree(h);
  for (hipEvent_t e : {c->ev_in, c->ev_fwd, c->ev_auc, c->ev_auc_p[0], c->ev_auc_p[1]})
    if (e) (void)hipEventDestroy(e);
  for (int s = 0; s < kSlots; ++s) {
    for (hipEvent_t e : {c->ev_loc[s], c->ev_free[s], c->ev_part[s]})
      if (e) (void)hipEventDestroy(e);
    for (DevState* d : {c->bds[s], c->ods[s]})
      if (d) (void)hipFree(d);
  }
  if (c->ads) (void)hipFree(c->ads);
  if (c->loc_stream) (void)hipStreamSynchronize(c->loc_stream);
  if (c->own_loc_stream) (void)hipStreamDestroy(c->own_loc_stream);
  if (c->part_stream) (void)hipStreamSynchronize(c->part_stream);
  if (c->own_part_stream) (void)hipStreamDestroy(c->own_part_stream);
  if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->lane_ev) (void)hipEventDestroy(e);
  table_release(c);
  cap_release(c);
  if (c->zpad) (void)hipFree(c->zpad);
  if (c->ds) (void)hipFree(c->ds);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete ctx;
  return DFX_OK;
}

int dfx_ctx_set_stream(dfx_ctx* ctx, void* hip_stream) {
  DFX_CHECK_ARG(ctx, "null ctx");
  // NULL is HIP's null (legacy default) stream, which is also torch's default stream
  // (kwarg main_excl keeps its CU-masked main stream)
  ctx->c.stream = static_cast<hipStream_t>(hip_stream);
  return DFX_OK;
}

int dfx_ctx_set_input_stream(dfx_ctx* ctx, void* hip_stream) {
  DFX_CHECK_ARG(ctx, "null ctx");
  ctx->c.in_stream = static_cast<hipStream_t>(hip_stream);
  ctx->c.has_in_stream = hip_stream != nullptr;
  return DFX_OK;
}

int dfx_ctx_lane_stream(dfx_ctx* ctx, int which, void** out) {
  DFX_CHECK_ARG(ctx && out, "null argument");
  DFX_CHECK_ARG(which >= 0 && which <= 3,
                "dfx_ctx_lane_stream: 0 (Localizer), 1 (AUC), 2 (split partition) or 3 (the "
                "context stream)");
  DFX_TRY(pipeline_init(&ctx->c));
  const Context& c = ctx->c;
  *out = which == 0 ? c.loc_stream : which == 1 ? c.aux_stream : which == 2 ? c.part_stream
                                                                            : c.stream;
  return DFX_OK;
}

int dfx_ctx_set_lane_stream(dfx_ctx* ctx, int which, void* hip_stream) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_CHECK_ARG(which == 0 || which == 2,
                "dfx_ctx_set_lane_stream: the Localizer lane (0) or the split partition (2)");
  Context* c = &ctx->c;
  DFX_TRY(pipeline_init(c));
  hipStream_t& cur = which == 0 ? c->loc_stream : c->part_stream;
  hipStream_t own = which == 0 ? c->own_loc_stream : c->own_part_stream;
  DFX_HIP(hipStreamSynchronize(cur));  // work queued on the previous stream is done
  cur = hip_stream ? static_cast<hipStream_t>(hip_stream) : own;
  return DFX_OK;
}

int dfx_ctx_use_own_stream(dfx_ctx* ctx) {
  DFX_CHECK_ARG(ctx, "null ctx");
  ctx->c.stream = ctx->c.own_stream;
  return DFX_OK;
}

int dfx_ctx_vdim(dfx_ctx* ctx) { return ctx ? ctx->c.P.V_dim : -1; }

int dfx_sync(dfx_ctx* ctx) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  // the AUC lane runs behind the context stream: join it first
  if (c->ev_auc) DFX_HIP(hipStreamWaitEvent(c->stream, c->ev_auc, 0));
  int err = 0;
  DFX_HIP(hipMemcpyAsync(&err, &c->ds->err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  if (!err) {
    DFX_TRY(table_unclump(c));
    DFX_TRY(store_maybe_grow(c));  // a sync point: grow once the load passes 0.5
  }
  if (err) {
    (void)hipMemsetAsync(&c->ds->err, 0, sizeof(int), c->stream);
    (void)hipStreamSynchronize(c->stream);
    std::string m = "device error:";
    if (err & kErrTableFull) m += " hash table full (raise max_keys / dfx_store_reserve);";
    if (err & kErrPoolFull) m += " V pool full (raise max_vrows);";
    if (err & kErrLens) m += " CHECK_EQ(lens[i], V_dim+1) failed (sgd_updater.cc:83);";
    if (err & kErrNoV) m += " CHECK(e.V != nullptr) failed (sgd_updater.cc:84);";
    if (err & kErrSort) m += " a look-back (radix sort or InitV ranking) never completed;";
    if (err & kErrBadKey) m += " key 0xffffffffffffffff is reserved (the empty-slot marker);";
    set_error(m);
    return (err & (kErrTableFull | kErrPoolFull)) ? DFX_ERR_CAPACITY : DFX_ERR_CHECK;
  }
  return DFX_OK;
}

int dfx_malloc(dfx_ctx* ctx, void** ptr, size_t bytes) {
  DFX_CHECK_ARG(ctx && ptr, "dfx_malloc: null argument");
  DFX_HIP(hipSetDevice(ctx->c.device));
  DFX_HIP(hipMalloc(ptr, bytes ? bytes : 16));
  return DFX_OK;
}

int dfx_free(dfx_ctx* ctx, void* ptr) {
  (void)ctx;
  if (ptr) DFX_HIP(hipFree(ptr));
  return DFX_OK;
}

int dfx_memcpy(dfx_ctx* ctx, void* dst, const void* src, size_t bytes, int kind) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_CHECK_ARG(kind >= 0 && kind <= 2, "dfx_memcpy: kind must be 0, 1 or 2");
  if (bytes == 0) return DFX_OK;
  DFX_CHECK_ARG(dst && src, "dfx_memcpy: null pointer");
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                              : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
  DFX_HIP(hipMemcpyAsync(dst, src, bytes, k, ctx->c.stream));
  if (kind == 1) DFX_HIP(hipStreamSynchronize(ctx->c.stream));
  return DFX_OK;
}

int dfx_reserve(dfx_ctx* ctx, int64_t max_rows, int64_t max_nnz) {
  DFX_CHECK_ARG(ctx, "null ctx");
  return step_reserve(&ctx->c, max_rows, max_nnz);
}

int dfx_progress_read(dfx_ctx* ctx, dfx_progress* out, int reset) {
  DFX_CHECK_ARG(ctx && out, "null argument");
  Context* c = &ctx->c;
  double prog[5];
  if (c->ev_auc) DFX_HIP(hipStreamWaitEvent(c->stream, c->ev_auc, 0));
  DFX_HIP(hipMemcpyAsync(prog, c->ds->prog, sizeof(prog), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  out->nrows = prog[0];
  out->loss = prog[1];
  out->auc = prog[2];
  out->penalty = prog[3];
  out->nnz_w = prog[4];
  if (reset) {
    DFX_HIP(hipMemsetAsync(c->ds->prog, 0, sizeof(prog), c->stream));
    DFX_HIP(hipStreamSynchronize(c->stream));
  }
  return dfx_sync(ctx);
}

}  // extern "C"
