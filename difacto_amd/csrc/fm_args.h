// Argument blocks of the FM forward/backward kernels (fm.hip), shared with step.hip.
#pragma once
#include "expf.h"
#include "internal.h"

namespace dfx {

// the exp2 table of glibc's expf (expf.h), one copy per translation unit in constant memory
static __constant__ const uint64_t kExp2fTab[32] = DFX_EXP2F_TAB;
__device__ inline float dfx_expf(float x) {
  return expf_glibc(x, [](int i) { return kExp2fTab[i]; });
}

// CalcGrad's p = -y / (1 + expf(y * pred)) [* weight] (fm_loss.h:159-164), expf as glibc's
__device__ inline float logit_p(float label, float pred, const float* rw, int64_t r) {
  float y = label > 0 ? 1.f : -1.f;
  float t = y * pred;
  float e = dfx_expf(t);
  float den = 1.f + e;
  float p = -y / den;
  if (rw) p = p * rw[r];
  return p;
}

struct FwdArgs {
  int64_t B;
  const uint64_t* offs;
  const uint32_t* col;   // remapped column, or (fused) the nnz's model-table slot
  const int2* wv;        // the nnz's {w, vrow} (col unused)
  const int2* wv_rank;   // {w, vrow} per key rank, reached through col (the Pull's output)
  // fused, probe mode: the nnz's raw feature id; the forward finds its key in the table
  // (every key of the batch was inserted by the Get before), so the Localizer writes no col
  const uint64_t* index;
  uint64_t max_index;
  const float* val;
  // fused: the model table itself (SGDUpdater::Get semantics, l1_shrk from P);
  // standalone: interleaved weights addressed by positions
  Table T;
  int l1_shrk;
  const float* W;
  const int32_t* wpos;
  const int32_t* vpos;
  const float* Vbase;
  const float* zpad;     // kZpadFloats device zeros: targets of masked (clamped) gathers
  int d;
  // sharded store: W holds one pulled record of rec_S floats [V(d) | w | live | 0 0] per
  // column (wpos / vpos unused)
  int rec_S;
  const float* label;
  const float* rw;
  const float* pred_in;  // gradient prep: p from this pred
  float* pred;           // predict: in/out (+=); fused: out
  float* p_out;
  float* XVp;            // B rows of xs floats: XV_ * p (xs = 0: d)
  // xs > d: row r also carries p at XVp[r*xs + d], so the backward reads p from the line it
  // reads XV_*p from (one random row instead of two)
  int xs;
  double* loss_part;     // fused: per-block partial sums of Evaluate
  // fused: the AUC lane's snapshot (orderable pred key, label > 0), written by the forward
  uint32_t* auc_key;
  uint32_t* auc_lab;
  // owner-computes split (split.hip): index holds the final keys (no ReverseBytes / max_index),
  // and the forward writes per row its partial [XV(d) | XXVV(d) | sum w x | 0 0 0]
  // (split_part_floats(d) floats) instead of pred / p / XV*p / loss
  int keys_ready;
  int part_n;      // owners of the split step (the partial's layout, split_part_floats)
  int no_fat_fwd;  // fat slots: the split forward walk instead of the one-trip read (A/B)
  int cpl;         // kwarg fwd_cpl: V coordinates per lane of the probe forward (0 / 4, or 8)
  int lr_lanes;    // V_dim 0: four lanes per row (kwarg lr_lanes)
  float* part;
  int nt;  // kwarg nt: kNtFwdTable = the slots with the streaming policy
  // the split's sliced owner forward (slice_len > 0): B = workers * slice_len logical rows,
  // logical row i being the owner's row (i / slice_len) * slice_m + slice_lo + i % slice_len
  int64_t slice_m, slice_lo, slice_len;
};

__device__ inline int64_t fwd_row(const FwdArgs& a, int64_t i) {
  if (a.slice_len <= 0) return i;
  return (i / a.slice_len) * a.slice_m + a.slice_lo + i % a.slice_len;
}

// the owner-computes split's per-row forward partial and its per-row [XV*p | p] record
// the owner's partial per row: one owner (N = 1) [XV(d) | XXVV(d) | sum w x | 0 0 0], so the
// worker finishes the row exactly as the fused forward; N > 1 owners [XV(d) | sum w x |
// sum_l XXVV_l | 0 0] (d + 4 floats: the partial exchange is ~half as large, and the regrouped
// sums are within the tolerance either way)
__host__ __device__ inline int split_part_floats(int d, int n) { return n > 1 ? d + 4 : 2 * d + 4; }
// [XV*p (d) | p | pad] rows of the split's all-gather: wide = whole 128-byte lines (the fused
// step's xvp_row layout: one line per occurrence in the backward), else d + 4 floats
__host__ __device__ inline int split_pxv_floats(int d, int wide = 0) {
  const int w = (d + 1 + 31) / 32 * 32;
  return (wide && d > 0 && w > d + 4) ? w : d + 4;
}

struct BwdArgs {
  int no_fat_spec;           // fat slots: no V / Vaux loads beside the home entry (A/B)
  int nt;                    // kwarg nt: kNtBwdTable / kNtBwdOcc with the streaming policy
  int cpl;                   // kwarg bwd_cpl (fused launches; 0 = 4)
  int cpl_from;              // kwarg bwd_cpl_from: the least V_dim bwd_cpl applies to (0 = 64)
  const uint32_t* segstart;  // nseg+1
  const DevState* ds;        // nseg = ds->u_count when nseg_host < 0
  int64_t nseg_host;
  const uint32_t* segcol;    // column of each segment (NULL: segment index == column)
  const uint32_t* occ_row;   // row of every occurrence, in sorted (key, pos) order
  const float* occ_x;        // its value (NULL: binary data)
  const uint2* occ_rx;       // (lb_gather=2) occ_row holds input positions: {row, value} here
  const float* zpad;
  const float* p;
  const float* XVp;
  int xs;                    // XVp row stride (0: d); xs > d: p at XVp[row*xs + d]
  int d;
  // standalone CalcGrad: positions into grad
  const int32_t* wpos;
  const int32_t* vpos;
  const float* W;
  float* grad;
  // sharded store: W / grad hold one record of rec_S floats per column, pulled
  // [V(d) | w | live | 0 0] and gradient [gV(d) | gw | live | 0 0]; every gradient record is
  // written whole (no pre-zeroing)
  int rec_S;
  // fused update
  uint32_t* slot;            // model-table slot of each segment's key (written when inserting)
  // training step without a separate Get pass: the backward finds-or-inserts each key itself
  // (the forward read absent keys as the empty entry); uniq: the sorted unique keys
  const uint64_t* uniq;
  int insert_keys;
  Table T;
  Params Pm;
  uint32_t* flags;  // InitV request per key
  DevState* dsw;
  // (diagnostic) per block {keys with live V, their occurrences}: plain stores, summed by
  // k_sum_live only when dfx_prof_counts is being fed (same-address atomics from every block
  // serialise at one L2 channel: they tripled the backward)
  uint2* live_part;
  // long segments (chunk_plan): first chunk of each segment, segment of each chunk, the
  // chunk count (device) and the chunks' partials [g_w, XXp, sum (XV p) x (d)] in double
  const uint32_t* choff;
  const uint32_t* chunk_seg;
  const uint32_t* nchunks;
  double* part;
  // wide V_dim, two passes (launch_bwd_fused with wsplit): a pass with one lane per key (entry,
  // g_w, FTRL) lists the keys whose V it must update {segment, V row, XXp}; a pass with G lanes
  // per listed key does the V sums and AdaGrad
  uint4* vlist;
  uint32_t* vcount;
  // the pass with one lane per key leaves its blocks' {new_w, n_init, n_keys} counts here and
  // the V pass's first block adds them to dsw (one atomic per counter instead of one per block)
  int4* wstat;
  int32_t nwstat;
  // the fused step's striped counters (DevState::bw_stripe; NULL: add to dsw directly)
  unsigned long long* stripes;
};

// occurrence i's row, and its value into *x: read directly, or (occ_rx: the bucket Localizer's
// gather left to the backward) through the input position occ_row holds
__device__ __forceinline__ uint32_t occ_get(const BwdArgs& a, uint64_t i, bool valued, bool nt,
                                            float* x) {
  const uint32_t r = ldnt(a.occ_row + i, nt);
  if (a.occ_rx) {
    const uint2 rv = a.occ_rx[r];
    *x = __uint_as_float(rv.y);
    return rv.x;
  }
  *x = valued ? ldnt(a.occ_x + i, nt) : 1.f;
  return r;
}

// the XVp row stride the workspace is sized for (step.hip): p rides in each row
int xvp_stride(const Context* c);
// fused forward; *nblk receives the number of loss partials written.  spread: probe mode
// with the lookups spread over the row's lanes (k_fm_fwd_probe) where the lane layout allows
int launch_fwd_fused(const FwdArgs& a, hipStream_t st, int* nblk, bool spread = true);
// fused backward + FTRL/AdaGrad update over at most nseg_bound segments; lds: bytes of LDS
// reserved per block (-1: the default cap)
int64_t bwd_fused_blocks(int d, int64_t nseg_bound, bool two_pass, int cpl);
// V_dim whose fused backward may run in two passes (>= 32 lanes per key)
bool bwd_two_pass(int d);
// the two-pass backward's list for nseg_bound keys, when the context runs it (else vlist NULL)
int bwd_two_pass_reserve(Context* c, Workspace& ws, int64_t nseg_bound, BwdArgs* g);
int sum_live(const uint2* part, int64_t n, DevState* ds, hipStream_t st);
int launch_bwd_fused(const BwdArgs& a, int64_t nseg_bound, hipStream_t st, long lds = -1);
// the chunk partials of long segments (before the backward reads them)
int launch_bwd_chunks(const BwdArgs& a, int64_t chunk_bound, hipStream_t st, bool aligned);

}  // namespace dfx
