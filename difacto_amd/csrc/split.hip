// Owner-computes FM over the key-range shards: SURVEY §8(e)'s synchronous semantics (one
// reference step, sgd_learner.cc:201-317, on the concatenation of the workers' batches) with the
// forward and backward run where the model rows live.
//
// The all-to-all-v schedule of dist.hip moves every touched key's model record to its worker
// and a gradient record back (~5.8 KB per row at d = 16), and each owner reads a key's entry and
// V twice per step.  Here the owners compute instead; only per-row quantities travel:
//   worker  k_split_count / k_split_scatter   each nnz's key (ReverseBytes(id % max_index)) to
//           its owner floor(key * N / 2^64), row order kept; nnz per (owner, row)
//   -> alltoallv keys (+ values), row counts
//   owner   owner_begin   the received sub-rows of all workers, concatenated in rank order, go
//           through the Localizer (sorted unique keys, occurrences in (worker, row, nnz) order =
//           the concatenated batch's order); epoch 0: Update(kFeaCount) + ranked InitV
//   owner   owner_forward per received row its partial [XV(d) | XXVV(d) | sum w x | 0 0 0] over
//           the owner's keys (the fused forward, fm.hip, in partial mode)
//   -> alltoallv partials back
//   worker  combine       per row the owners' partials summed in rank order -> pred (clip), p,
//           logloss, the AUC snapshot, and the row [XV*p (d) | p | 0 0 0] (fm_loss.h:67-203)
//   -> every owner receives every worker's rows
//   owner   owner_backward the fused backward + FTRL/AdaGrad over the owner's keys, reading the
//           rows' p and XV*p from the received records; ranked InitV
// Per row that is ~40 keys + N partials + N records (~1.9 KB at d = 16, N = 8) instead of
// ~5.8 KB, and each owner touches a key's entry and V once per step as the fused step does.
// At N = 1 the partial is the whole row and the step equals the fused step bit for bit; at
// N > 1 the forward's sums are regrouped by owner (within the 1e-5 tolerance), the gradients
// are summed over the occurrences in the concatenated batch's order.
#include "fm_args.h"

namespace dfx {

void sum_parts(Context* c, const double* part, int64_t n, double* out, bool accumulate);

constexpr int kSpNT = 256;
constexpr int kSpRows = 64;  // rows per partition block

__device__ inline uint32_t split_owner(uint64_t k, uint32_t n) {
  return (uint32_t)__umul64hi(k, (uint64_t)n);  // floor(k * n / 2^64), dist.hip owner_of
}

__device__ inline uint64_t split_key(uint64_t id, uint64_t max_index) {
  const uint64_t m = max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % max_index;
  return reverse_bytes(m);  // the Localizer's key (localize.hip k_loc_transform)
}

// nnz per (owner, row) -> row_cnt[owner * B + row]; per (owner, 64-row block) -> blk[owner *
// nblk + b].  A block owns one 64-row partition block and walks its nnz coalesced (one thread
// per nnz, its row by binary search over the block's offsets in LDS), counting into LDS
// [row][owner]; then the first wave, one thread per row, writes the counts and sums them.  (One
// thread per row walking its row serially: 62-66 us per step, 1.5 waves per SIMD waiting on
// 39-deep chains of strided loads.)
__global__ __launch_bounds__(kSpNT) void k_split_count(int64_t B, const uint64_t* offs,
                                                       const uint64_t* index, uint64_t max_index,
                                                       uint32_t n, uint32_t* row_cnt,
                                                       uint32_t* blk, int64_t nblk) {
  extern __shared__ uint32_t cnt[];  // [row of the block][owner]
  __shared__ uint64_t so[kSpRows + 1];
  static_assert(kSpRows == kWave, "a 64-row partition block is one wave");
  const int t = threadIdx.x;
  const int64_t rb = (int64_t)blockIdx.x * kSpRows;
  const int nr = (int)((B - rb) < kSpRows ? (B - rb) : kSpRows);
  for (int i = t; i <= nr; i += kSpNT) so[i] = offs[rb + i];
  for (int64_t i = t; i < (int64_t)kSpRows * n; i += kSpNT) cnt[i] = 0u;
  __syncthreads();
  const uint64_t j1 = so[nr];
  for (uint64_t j = so[0] + t; j < j1; j += kSpNT) {
    int lo = 0, hi = nr;  // row = upper_bound(j) - 1 over the block's offsets (empty rows skipped)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (so[mid] <= j) lo = mid; else hi = mid;
    }
    atomicAdd(&cnt[(int64_t)lo * n + split_owner(split_key(index[j], max_index), n)], 1u);
  }
  __syncthreads();
  if (t >= kWave) return;
  const int64_t r = rb + t;
  for (uint32_t o = 0; o < n; ++o) {
    uint32_t v = t < nr ? cnt[(int64_t)t * n + o] : 0u;
    if (r < B) row_cnt[(int64_t)o * B + r] = v;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    if (t == 0) blk[(int64_t)o * nblk + blockIdx.x] = v;
  }
}

// split counts per owner from the scanned block totals, into the pinned host words
__global__ void k_split_totals(const uint32_t* blk_excl, const uint32_t* total, int64_t nblk,
                               uint32_t n, unsigned long long* out) {
  const uint32_t o = threadIdx.x;
  if (o >= n) return;
  const uint32_t a = blk_excl[(int64_t)o * nblk];
  const uint32_t b = (o + 1 < n) ? blk_excl[(int64_t)(o + 1) * nblk] : *total;
  out[o] = (unsigned long long)(b - a);
}

// each nnz's key (and value) to its owner's run, in nnz order within each owner: the block's
// chunks of kSpNT nnz are ranked by owner with wave ballots (exact and order preserving)
__global__ __launch_bounds__(kSpNT) void k_split_scatter(int64_t B, const uint64_t* offs,
                                                         const uint64_t* index,
                                                         const float* value, uint64_t max_index,
                                                         uint32_t n, const uint32_t* blk_excl,
                                                         int64_t nblk, uint64_t* keys_out,
                                                         float* x_out) {
  constexpr int W = kSpNT / kWave;
  __shared__ uint32_t run[kMaxDistRanks];
  __shared__ uint32_t wc[W][kMaxDistRanks];
  const int t = threadIdx.x, w = t / kWave;
  const int64_t r0 = (int64_t)blockIdx.x * kSpRows;
  const int nr = (int)((B - r0) < kSpRows ? (B - r0) : kSpRows);
  const uint64_t j0 = offs[r0], j1 = offs[r0 + nr];
  for (int o = t; o < (int)n; o += kSpNT) run[o] = blk_excl[(int64_t)o * nblk + blockIdx.x];
  int bits = 0;
  while ((1u << bits) < n) ++bits;
  for (uint64_t c0 = j0; c0 < j1; c0 += kSpNT) {
    for (int i = t; i < W * (int)n; i += kSpNT) (&wc[0][0])[(i / n) * kMaxDistRanks + i % n] = 0;
    __syncthreads();
    const uint64_t j = c0 + t;
    const bool valid = j < j1;
    const uint64_t key = valid ? split_key(index[j], max_index) : 0ull;
    const uint32_t o = valid ? split_owner(key, n) : 0u;
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
      const bool bit = (o >> b) & 1u;
      const uint64_t mb = __ballot(valid && bit);
      peers &= bit ? mb : ~mb;
    }
    const uint32_t rk = (uint32_t)__popcll(peers & lanemask_lt());
    if (valid && rk == 0) wc[w][o] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = run[o] + rk;
      for (int v = 0; v < w; ++v) pos += wc[v][o];
      keys_out[pos] = key;
      if (x_out) x_out[pos] = value ? value[j] : 1.f;  // binary rows carry 1 when asked
    }
    __syncthreads();
    for (int oo = t; oo < (int)n; oo += kSpNT) {
      uint32_t s = 0;
      for (int v = 0; v < W; ++v) s += wc[v][oo];
      run[oo] += s;
    }
    __syncthreads();
  }
}

// owner: the received per-row counts (scanned in place) -> u64 row offsets
__global__ void k_split_offsets(const uint32_t* excl, const uint32_t* total, int64_t R,
                                uint64_t* offs) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) offs[r] = excl[r];
  if (r == R) offs[R] = *total;
}

// worker: the owners' partials of each row summed in rank order, then FMLoss::Predict's tail
// (fm_loss.h:110-119), Evaluate, the AUC snapshot and CalcGrad's per-row factors
// (fm_loss.h:155-199): pxv row [XV*p (d) | p | 0 0 0]
__global__ __launch_bounds__(kSpNT) void k_split_combine(int64_t row0, int64_t B, int64_t M,
                                                         int n, int d,
                                                         int PX, const float* __restrict__ parts,
                                                         const float* label, const float* rw,
                                                         float* pred_out, float* pxv,
                                                         double* loss_part, uint32_t* auc_key,
                                                         uint32_t* auc_lab) {
  __shared__ double red[kSpNT / kWave];
  const int64_t r = row0 + (int64_t)blockIdx.x * kSpNT + threadIdx.x;
  const int PS = split_part_floats(d, n);
  const bool compact = n > 1;  // [XV | sum w x | sum_l XXVV_l | 0 0] per owner
  double loss = 0;
  if (r < B) {
    float acc = 0.f;
    for (int o = 0; o < n; ++o) acc += parts[((int64_t)o * M + r) * PS + (compact ? d : 2 * d)];
    float pr = acc;
    if (d > 0 && compact) {
      // s = sum_l XV_l^2 - sum_owners sum_l XXVV_l (the owners' serial sums, in rank order)
      float s = 0.f, xx = 0.f;
      for (int l = 0; l < d; ++l) {
        float xv = 0.f;
        for (int o = 0; o < n; ++o) xv += parts[((int64_t)o * M + r) * PS + l];
        s += xv * xv;
      }
      for (int o = 0; o < n; ++o) xx += parts[((int64_t)o * M + r) * PS + d + 1];
      s -= xx;
      const double y = (double)acc + .5 * (double)s;
      pr = (float)y;
      pr = pr > 20.f ? 20.f : (pr < -20.f ? -20.f : pr);
    } else if (d > 0) {
      float s = 0.f;
      for (int l = 0; l < d; ++l) {
        float xv = 0.f, xx = 0.f;
        for (int o = 0; o < n; ++o) {
          const float* q = parts + ((int64_t)o * M + r) * PS;
          xv += q[l];
          xx += q[d + l];
        }
        s += xv * xv - xx;  // s = sum_l (XV_l^2 - XXVV_l), serially over l
      }
      const double y = (double)acc + .5 * (double)s;
      pr = (float)y;
      pr = pr > 20.f ? 20.f : (pr < -20.f ? -20.f : pr);
    }
    const float p = logit_p(label[r], pr, rw, r);
    if (pred_out) pred_out[r] = pr;
    float* x = pxv + r * PX;
    for (int l = 0; l < d; ++l) {
      float xv = 0.f;
      for (int o = 0; o < n; ++o) xv += parts[((int64_t)o * M + r) * PS + l];
      x[l] = xv * p;  // XV_ *= p (fm_loss.h:196-199)
    }
    x[d] = p;
    x[d + 1] = x[d + 2] = x[d + 3] = 0.f;
    const double yy = label[r] > 0 ? 1.0 : -1.0;
    loss = log(1.0 + exp(-yy * (double)pr));  // Loss::Evaluate (loss.h:57-66)
    if (auc_key) {
      const uint32_t u = __float_as_uint(pr + 0.0f);
      auc_key[r] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
      auc_lab[r] = label[r] > 0 ? 1u : 0u;
    }
  }
  for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int i = 0; i < kSpNT / kWave; ++i) s += red[i];
    loss_part[blockIdx.x] = s;
  }
}

// k_split_combine with G lanes per row (V_dim % 4 == 0, G = pow2 >= V_dim / 4): lane l sums
// coordinates [4l, 4l + 4) of the owners' partials with float4 loads, in rank order; the serial
// sum over l of the reference (fm_loss.h:110-113) is taken by every lane through shuffles in l
// order, so results are bit-identical to k_split_combine's, with coalesced row reads
template <int G>
__global__ __launch_bounds__(kSpNT) void k_split_combine_vec(int64_t row0, int64_t B,
                                                             int64_t M, int n, int d, int PX,
                                                             const float* __restrict__ parts,
                                                             const float* label, const float* rw,
                                                             float* pred_out, float* pxv,
                                                             double* loss_part, uint32_t* auc_key,
                                                             uint32_t* auc_lab) {
  __shared__ double red[kSpNT / kWave];
  constexpr int RPB = kSpNT / G;
  const int l = threadIdx.x % G;
  const int gbase = (threadIdx.x % kWave) - l;
  const int64_t r = row0 + (int64_t)blockIdx.x * RPB + threadIdx.x / G;
  const int PS = split_part_floats(d, n);
  const bool compact = n > 1;
  const bool mine = 4 * l < d;
  double loss = 0;
  if (r < B) {
    float acc = 0.f, xx1 = 0.f;
    float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), xx = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int o = 0; o < n; ++o) {
      const float* q = parts + ((int64_t)o * M + r) * PS;
      acc += q[compact ? d : 2 * d];
      if (compact) xx1 += q[d + 1];
      if (mine) {
        const float4 v = *reinterpret_cast<const float4*>(q + 4 * l);
        xv.x += v.x; xv.y += v.y; xv.z += v.z; xv.w += v.w;
        if (!compact) xx = *reinterpret_cast<const float4*>(q + d + 4 * l);  // one owner
      }
    }
    float t4[4];
    const float xk[4] = {xv.x, xv.y, xv.z, xv.w}, yk[4] = {xx.x, xx.y, xx.z, xx.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) t4[k] = compact ? xk[k] * xk[k] : xk[k] * xk[k] - yk[k];
    float s = 0.f;
    for (int q = 0; q < G; ++q) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float tk = __shfl(t4[k], gbase + q, kWave);
        if (4 * q + k < d) s += tk;
      }
    }
    if (compact) s -= xx1;
    const double y = (double)acc + .5 * (double)s;
    float pr = (float)y;
    pr = pr > 20.f ? 20.f : (pr < -20.f ? -20.f : pr);
    const float p = logit_p(label[r], pr, rw, r);
    float* x = pxv + r * PX;
    if (mine)  // XV_ *= p (fm_loss.h:196-199)
      *reinterpret_cast<float4*>(x + 4 * l) = make_float4(xv.x * p, xv.y * p, xv.z * p, xv.w * p);
    if (l == 0) {
      if (pred_out) pred_out[r] = pr;
      *reinterpret_cast<float4*>(x + d) = make_float4(p, 0.f, 0.f, 0.f);
      const double yy = label[r] > 0 ? 1.0 : -1.0;
      loss = log(1.0 + exp(-yy * (double)pr));  // Loss::Evaluate (loss.h:57-66)
      if (auc_key) {
        const uint32_t u = __float_as_uint(pr + 0.0f);
        auc_key[r] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        auc_lab[r] = label[r] > 0 ? 1u : 0u;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < kSpNT / kWave; ++i) t += red[i];
    loss_part[blockIdx.x] = t;
  }
}

// the received rows' p as a compact array (V_dim a multiple of 32: p would be a 128-byte line of
// its own per occurrence in the backward; fm.hip row_p)
__global__ void k_split_p_compact(const float* pxv, int64_t R, int xs, int d, float* p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) p[r] = pxv[r * xs + d];
}

// the combine's loss partials summed (k_sum_parts' order: 1024-strided, then the waves in
// order) and the worker's progress — one launch (round 6; was k_sum_parts + a one-thread
// finalize)
__global__ __launch_bounds__(1024) void k_split_worker_finalize(const double* part, int64_t n,
                                                                DevState* ds, int64_t B) {
  __shared__ double red[1024 / kWave];
  double a = 0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) a += part[i];
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = a;
  __syncthreads();
  if (threadIdx.x != 0) return;
  double s = 0;
  for (int k = 0; k < 1024 / kWave; ++k) s += red[k];
  ds->scratch[3] = s;
  ds->prog[0] += (double)B;  // sgd::Progress of this worker (sgd_learner.cc:213-229)
  ds->prog[1] += s;          // the AUC lane adds prog[2] itself
}

__global__ void k_split_zero_count(uint32_t* ftotal, int64_t* out) {
  *ftotal = 0u;
  *out = 0;
}

static Lane split_owner_lane(Context* c, int slot) {
  return Lane{c->stream, &c->ows[slot], c->ods[slot], &c->ds->err};
}

}  // namespace dfx

using namespace dfx;

extern "C" {

#define DFX_SPLIT_SLOT(slot) DFX_CHECK_ARG((slot) >= 0 && (slot) < kSlots, "split: slot must be 0 .. 3")

int dfx_split_part_floats(dfx_ctx* ctx, int nranks) {
  return ctx && nranks >= 1 ? split_part_floats(ctx->c.P.V_dim, nranks) : -1;
}

int dfx_split_pxv_floats(dfx_ctx* ctx) {
  return ctx ? split_pxv_floats(ctx->c.P.V_dim, 1) : -1;
}

int dfx_split_partition(dfx_ctx* ctx, int slot, const dfx_batch* b, uint64_t max_index,
                        int nranks, uint64_t* keys_out, float* x_out, uint32_t* row_cnt_out) {
  DFX_CHECK_ARG(ctx && b, "null argument");
  DFX_SPLIT_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxDistRanks, "split: 1 <= nranks <= 64");
  DFX_CHECK_ARG(b->size >= 0 && b->nnz >= 0, "split_partition: negative sizes");
  DFX_CHECK_ARG(b->size == 0 || b->offset, "split_partition: null offset");
  DFX_CHECK_ARG(b->nnz == 0 || (b->index && keys_out), "split_partition: null buffer");
  DFX_CHECK_ARG(!b->value || b->nnz == 0 || x_out, "split_partition: valued data needs x_out");
  if (b->nnz == 0) x_out = nullptr;
  DFX_CHECK_ARG(b->size == 0 || row_cnt_out, "split_partition: null row counts");
  DFX_CHECK_ARG(max_index != 0, "split_partition: max_index must be > 0");
  DFX_CHECK_ARG(b->nnz < 0xFFFFFFFFll, "split_partition: nnz must fit u32");
  Context* c = &ctx->c;
  DFX_TRY(pipeline_init(c));
  Workspace& bw = c->bws[slot];
  const int64_t B = b->size;
  const int64_t nblk = B > 0 ? (B + kSpRows - 1) / kSpRows : 0;
  DFX_TRY(bw.hist.ensure((size_t)(nblk * nranks + 1) * 4));
  uint32_t* blk = bw.hist.as<uint32_t>();
  uint32_t* total = &c->bds[slot]->totals[0];
  // on its own high-priority stream, after the batch's producer: it reads only the batch, so
  // it runs beside the previous step's owner Localizer (the Localizer lane) and forward /
  // backward, and the host has the next split counts as early as possible
  hipStream_t st = c->part_stream;
  DFX_HIP(hipEventRecord(c->ev_in, c->has_in_stream ? c->in_stream : c->stream));
  DFX_HIP(hipStreamWaitEvent(st, c->ev_in, 0));
  const Lane L{st, &bw, c->bds[slot], &c->ds->err};
  if (nblk > 0) {
    hipLaunchKernelGGL(k_split_count, dim3((unsigned)nblk), dim3(kSpNT),
                       (size_t)kSpRows * nranks * 4, st, B, b->offset, b->index, max_index,
                       (uint32_t)nranks, row_cnt_out, blk, nblk);
  }
  DFX_TRY(scan_u32(L, blk, nblk * nranks, total));
  if (nblk > 0) {
    hipLaunchKernelGGL(k_split_scatter, dim3((unsigned)nblk), dim3(kSpNT), 0, st, B, b->offset,
                       b->index, b->value, max_index, (uint32_t)nranks, blk, nblk, keys_out,
                       x_out);
    hipLaunchKernelGGL(k_split_totals, dim3(1), dim3(kMaxDistRanks), 0, st, blk, total, nblk,
                       (uint32_t)nranks, c->dist_host[slot]);
  } else {
    for (int o = 0; o < nranks; ++o) c->dist_host[slot][o] = 0;
  }
  DFX_HIP(hipEventRecord(c->ev_part[slot], st));
  DFX_HIP(hipGetLastError());
  c->split_B[slot] = B;
  c->split_nblk[slot] = nblk;
  return DFX_OK;
}

int dfx_split_partition_wait(dfx_ctx* ctx, int slot, int nranks, int64_t* split_counts) {
  DFX_CHECK_ARG(ctx && split_counts, "null argument");
  DFX_SPLIT_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxDistRanks, "split: 1 <= nranks <= 64");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(c->loc_stream, "split_partition_wait: no dfx_split_partition issued");
  DFX_HIP(hipEventSynchronize(c->ev_part[slot]));
  for (int o = 0; o < nranks; ++o) split_counts[o] = (int64_t)c->dist_host[slot][o];
  return DFX_OK;
}

int dfx_split_owner_begin(dfx_ctx* ctx, int slot, const uint64_t* keys, const float* x,
                          uint32_t* row_cnt, const int64_t* rows_per_rank,
                          const int64_t* keys_per_rank, int nranks, int job_type,
                          int push_cnt, int lane) {
  DFX_CHECK_ARG(ctx && rows_per_rank && keys_per_rank, "null argument");
  DFX_SPLIT_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxDistRanks, "split: 1 <= nranks <= 64");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(c->dist_sum, "split: needs push_agg=sum (one Update per key per step)");
  DFX_CHECK_ARG(!any_pending(c->split_initv_pending),
                "split_owner_begin: finish the pending InitV first (dfx_split_initv_*)");
  DFX_TRY(pipeline_init(c));
  int64_t R = 0, nnz = 0;
  for (int g = 0; g < nranks; ++g) {
    DFX_CHECK_ARG(rows_per_rank[g] >= 0 && keys_per_rank[g] >= 0, "split: negative sizes");
    R += rows_per_rank[g];
    nnz += keys_per_rank[g];
  }
  DFX_CHECK_ARG(R == 0 || row_cnt, "split_owner_begin: null row counts");
  DFX_CHECK_ARG(nnz == 0 || keys, "split_owner_begin: null keys");
  DFX_CHECK_ARG(nnz < 0xFFFFFFFFll && R < 0x7FFFFFFFll, "split_owner_begin: too many keys");
  DFX_CHECK_ARG(job_type == DFX_JOB_TRAINING || job_type == DFX_JOB_VALIDATION ||
                    job_type == DFX_JOB_PREDICTION,
                "split_owner_begin: bad job type");
  const bool cnt = push_cnt && job_type == DFX_JOB_TRAINING && c->P.V_dim > 0 && nnz > 0;
  const bool get = !cnt && job_type != DFX_JOB_TRAINING && nnz > 0;
  DFX_CHECK_ARG(!lane || (!cnt && !get),
                "split_owner_begin: a step that touches the table (count push, Get) runs on "
                "the context stream (lane = 0)");
  // this step inserts at most nnz keys and draws at most nnz V rows (slots are not carried
  // across steps here, so the store may grow at this point)
  DFX_TRY(cap_check(c, nnz));
  // a server of one of nranks key ranges: hash keys by their position inside the range
  DFX_TRY(table_set_ranges(c, nranks));
  Lane OL = split_owner_lane(c, slot);
  if (lane) {
    // the Localizer lane: the received keys are ready on the caller's current stream (the
    // library's lane, which the caller made wait for the exchange); the slot's buffers are free
    // once the main stream finished the step that used them before
    OL.stream = c->loc_stream;
    DFX_HIP(hipStreamWaitEvent(c->loc_stream, c->slot_free[slot] ? c->slot_free[slot]
                                                                  : c->ev_free[slot], 0));
  }
  Workspace& ows = c->ows[slot];
  DFX_TRY(loc_reserve(ows, nnz, OL.stream));
  DFX_TRY(ows.rowid.ensure((size_t)(R + 1) * 8));
  DFX_TRY(ows.oflags.ensure((size_t)(nnz + 1) * 4));
  uint64_t* offs = ows.rowid.as<uint64_t>();
  uint32_t* rtotal = &OL.ds->totals[4];
  DFX_TRY(scan_u32(OL, row_cnt, R, rtotal));
  hipLaunchKernelGGL(k_split_offsets, dim3((unsigned)((R + 1 + 255) / 256)), dim3(256), 0,
                     OL.stream, row_cnt, rtotal, R, offs);
  LocOut o;
  o.uniq = ows.uniq.as<uint64_t>();
  o.segstart = ows.segstart.as<uint32_t>();
  o.occ_row = ows.occ_row.as<uint32_t>();
  o.value = x;
  o.occ_x = x ? ows.occ_x.as<float>() : nullptr;
  o.keys_ready = true;
  DFX_TRY(localize_run(c, OL, R, nnz, offs, keys, ~0ull, o));
  // long segments (hot keys): their chunk plan, as the fused step's Localizer lane makes it
  DFX_TRY(chunk_plan(OL, nnz, o.segstart, ows.flags.as<uint32_t>(), ows.rowtmp.as<uint32_t>(),
                     &OL.ds->totals[1]));
  c->split_rows[slot] = R;
  c->split_nnz[slot] = nnz;
  c->split_keys[slot] = keys;
  c->split_x[slot] = x;
  c->split_resolved[slot] = false;
  if (get) {
    // a step without a backward: SGDUpdater::Get still inserts every key (model_[key],
    // sgd_updater.cc:34-58), as the fused step's probe does
    DFX_TRY(probe_keys_run(c, OL, nnz, o.uniq, ows.slot.as<uint32_t>()));
    c->split_resolved[slot] = true;
  }
  if (cnt) {
    // Update(kFeaCount) of the concatenated batch: find-or-insert every key (Get), add its
    // occurrence count; InitV requests in key order, drawn ranked over all owners
    DFX_TRY(probe_keys_run(c, OL, nnz, o.uniq, ows.slot.as<uint32_t>()));
    DFX_TRY(push_cnt_seg_flags(c, OL, nnz, o.segstart, ows.slot.as<uint32_t>(),
                               ows.oflags.as<uint32_t>(), OL.ds));
    c->split_resolved[slot] = true;
    c->split_initv_pending[slot] = true;
    c->split_initv_gated[slot] = false;
  }
  c->split_lane[slot] = lane != 0;
  c->split_job[slot] = job_type;
  if (lane) {
    // the combine writes the AUC lane's snapshot buffer (two, alternating) once the AUC that last
    // read it is done: the lane joins that AUC before it hands the slot over (the owner forward
    // waits for the lane), so the main stream waits on one event less per step (~4 us,
    // tools/membench/waitbench.hip).  The buffer is the next combine's when the driver begins a
    // step after the previous step's combine (split_host.cc); else the combine waits itself
    const int p = c->split_auc_par;
    DFX_HIP(hipStreamWaitEvent(c->loc_stream, c->ev_auc_p[p], 0));
    c->split_auc_joined_par[slot] = p;
    c->split_auc_joined[slot] = c->auc_seq_p[p];
    DFX_HIP(hipEventRecord(c->ev_loc[slot], c->loc_stream));
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// rows [lo, lo + len) of every source worker's M-row block (len = 0: every row, M unused)
int dfx_split_owner_forward_rows(dfx_ctx* ctx, int slot, float* part_out, int nranks, int64_t M,
                                 int64_t lo, int64_t len) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_SPLIT_SLOT(slot);
  Context* c = &ctx->c;
  DFX_CHECK_ARG(!c->split_initv_pending[slot],
                "split_owner_forward: the count push's InitV is pending (dfx_split_initv_*)");
  const int64_t R = c->split_rows[slot];
  const bool sliced = len > 0;
  DFX_CHECK_ARG(!sliced || (nranks >= 1 && M >= 1 && lo >= 0 && lo + len <= M &&
                            R == (int64_t)nranks * M),
                "split_owner_forward_rows: rows [lo, lo + len) of nranks blocks of M rows");
  if (c->split_lane[slot]) DFX_HIP(hipStreamWaitEvent(c->stream, c->ev_loc[slot], 0));
  const bool last = !sliced || lo + len == M;
  if (R > 0) {
    DFX_CHECK_ARG(part_out, "split_owner_forward: null buffer");
    Workspace& ows = c->ows[slot];
    FwdArgs a{};
    a.B = sliced ? (int64_t)nranks * len : R;
    a.offs = ows.rowid.as<uint64_t>(); a.val = c->split_x[slot];
    a.index = c->split_keys[slot]; a.max_index = ~0ull; a.keys_ready = 1;
    a.T = c->T; a.l1_shrk = c->P.l1_shrk; a.Vbase = c->T.V; a.zpad = c->zpad; a.d = c->P.V_dim;
    a.no_fat_fwd = !c->fat_fwd;
    a.cpl = c->fwd_cpl;
    a.part = part_out;
    a.part_n = (int)c->T.range_mul;  // the owners (dfx_split_owner_begin's table_set_ranges)
    if (sliced) {
      a.slice_m = M;
      a.slice_lo = lo;
      a.slice_len = len;
    }
    int nblk = 0;
    DFX_TRY(launch_fwd_fused(a, c->stream, &nblk, true));
  }
  if (!last) return DFX_OK;
  // a step without a backward is done with the slot (and the table) here (a training step's
  // InitV draw, or its backward at V_dim 0, frees it: an event record costs the stream ~5 us)
  if (c->split_job[slot] != DFX_JOB_TRAINING) {
    DFX_HIP(hipEventRecord(c->ev_free[slot], c->stream));
    c->slot_free[slot] = nullptr;
    DFX_TRY(cap_record(c));
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_split_owner_forward(dfx_ctx* ctx, int slot, float* part_out) {
  return dfx_split_owner_forward_rows(ctx, slot, part_out, 1, 0, 0, 0);
}

// rows [lo, lo + len) of this worker's batch (lo a multiple of 256); the call whose rows end
// at part_rows (or beyond) finishes the step: the loss of every row, the AUC lane, progress
int dfx_split_combine_rows(dfx_ctx* ctx, int slot, const dfx_batch* b, const float* parts,
                           int64_t part_rows, int nranks, float* pxv_out, float* pred_out,
                           int64_t lo, int64_t len) {
  DFX_CHECK_ARG(ctx && b, "null argument");
  DFX_SPLIT_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxDistRanks, "split: 1 <= nranks <= 64");
  DFX_CHECK_ARG(lo >= 0 && len >= 1 && lo % 256 == 0,
                "split_combine_rows: rows [lo, lo + len), lo a multiple of 256");
  Context* c = &ctx->c;
  const int64_t B = b->size;
  DFX_CHECK_ARG(B == c->split_B[slot], "split_combine: batch differs from split_partition's");
  DFX_CHECK_ARG(B == 0 || (b->label && parts && pxv_out), "split_combine: null buffer");
  DFX_CHECK_ARG(part_rows >= B, "split_combine: part_rows < the batch's rows");
  const int d = c->P.V_dim;
  Workspace& ws = c->ws;
  // V_dim % 4 == 0: G lanes per row, coalesced float4 rows (else one thread per row)
  int G = 0;
  if (d > 0 && d % 4 == 0 && d <= 256) {
    G = 1;
    while (4 * G < d) G <<= 1;
  }
  const int64_t rpb = G ? kSpNT / G : kSpNT;
  const int64_t nb = (B + rpb - 1) / rpb;
  const int PX = split_pxv_floats(d, 1);
  const bool first = lo == 0, last = lo + len >= part_rows;
  // one loss partial per block (the blocks of every call tile the batch), after the 8 doubles
  // the scratch keeps in front
  if (first) DFX_TRY(ws.dscratch.ensure((size_t)(nb + 16) * 8));
  double* loss_part = ws.dscratch.as<double>() + 8;
  // the AUC lane's snapshot: two buffers, alternating by step, each free once the AUC that last
  // read it is done — the AUC of two steps back (as the fused step's, step.hip auc_db_on)
  if (first) {
    c->split_auc_cur = c->split_auc_par;
    c->split_auc_par ^= 1;
  }
  const int ap = c->split_auc_cur;
  Workspace& aw = ap ? c->aws_alt : c->aws;
  const Lane AL{c->aux_stream, &aw, c->ads, &c->ds->err};
  if (first) {
    DFX_TRY(auc_reserve(aw, B, c->aux_stream));
    // (joined already when this slot's Localizer lane waited for that buffer's last reader and
    // no AUC read the buffer since: the owner forward before this combine waited for the lane)
    if (!(c->split_lane[slot] && c->split_auc_joined_par[slot] == ap &&
          c->split_auc_joined[slot] == c->auc_seq_p[ap]))
      DFX_HIP(hipStreamWaitEvent(c->stream, c->ev_auc_p[ap], 0));
  }
  const int64_t r1 = lo + len < B ? lo + len : B;
  if (r1 > lo) {
    uint32_t* ak = aw.ak0.as<uint32_t>();
    uint32_t* al = aw.av0.as<uint32_t>();
    const dim3 grid((unsigned)((r1 - lo + rpb - 1) / rpb));
    double* lp = loss_part + lo / rpb;
#define DFX_COMBINE(GG)                                                                        \
    if (G == GG)                                                                               \
      hipLaunchKernelGGL(k_split_combine_vec<GG>, grid, dim3(kSpNT), 0, c->stream, lo, r1,     \
                         part_rows, nranks, d, PX, parts, b->label, b->weight, pred_out,       \
                         pxv_out, lp, ak, al);
    DFX_COMBINE(1) DFX_COMBINE(2) DFX_COMBINE(4) DFX_COMBINE(8) DFX_COMBINE(16) DFX_COMBINE(32)
    DFX_COMBINE(64)
#undef DFX_COMBINE
    if (G == 0)
      hipLaunchKernelGGL(k_split_combine, grid, dim3(kSpNT), 0, c->stream, lo, r1, part_rows,
                         nranks, d, PX, parts, b->label, b->weight, pred_out, pxv_out, lp, ak,
                         al);
  }
  if (!last) {
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  DFX_HIP(hipEventRecord(c->ev_fwd, c->stream));
  DFX_HIP(hipStreamWaitEvent(c->aux_stream, c->ev_fwd, 0));
  DFX_TRY(auc_finish(AL, B, &c->ds->prog[2], true, c->auc_sort));
  DFX_HIP(hipEventRecord(c->ev_auc, c->aux_stream));
  DFX_HIP(hipEventRecord(c->ev_auc_p[ap], c->aux_stream));  // this buffer's last reader
  ++c->auc_seq_p[ap];
  hipLaunchKernelGGL(k_split_worker_finalize, dim3(1), dim3(1024), 0, c->stream, loss_part, nb,
                     c->ds, B);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_split_combine(dfx_ctx* ctx, int slot, const dfx_batch* b, const float* parts,
                      int64_t part_rows, int nranks, float* pxv_out, float* pred_out) {
  return dfx_split_combine_rows(ctx, slot, b, parts, part_rows, nranks, pxv_out, pred_out, 0,
                                part_rows > 0 ? part_rows : 1);
}

int dfx_split_owner_backward(dfx_ctx* ctx, int slot, const float* pxv) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_SPLIT_SLOT(slot);
  Context* c = &ctx->c;
  DFX_CHECK_ARG(!any_pending(c->split_initv_pending),
                "split_owner_backward: finish the pending InitV first (dfx_split_initv_*)");
  const int64_t R = c->split_rows[slot], nnz = c->split_nnz[slot];
  const int d = c->P.V_dim;
  if (nnz > 0) {
    DFX_CHECK_ARG(pxv, "split_owner_backward: null records");
    Workspace& ows = c->ows[slot];
    DevState* ods = c->ods[slot];
    BwdArgs g{};
    g.segstart = ows.segstart.as<uint32_t>(); g.ds = ods; g.nseg_host = -1; g.segcol = nullptr;
    g.occ_row = ows.occ_row.as<uint32_t>();
    g.occ_x = c->split_x[slot] ? ows.occ_x.as<float>() : nullptr;
    g.zpad = c->zpad; g.p = nullptr; g.XVp = pxv; g.xs = split_pxv_floats(d, 1); g.d = d;
    if (d >= 64 && d % 32 == 0 && R > 0) {  // p a line of its own in the rows: compact (row_p)
      DFX_TRY(ows.p.ensure((size_t)R * 4));
      hipLaunchKernelGGL(k_split_p_compact, dim3((unsigned)((R + 255) / 256)), dim3(256), 0,
                         c->stream, pxv, R, g.xs, d, ows.p.as<float>());
      g.p = ows.p.as<float>();
    }
    g.slot = ows.slot.as<uint32_t>(); g.T = c->T; g.Pm = c->P; g.no_fat_spec = false; g.cpl = c->bwd_cpl; g.cpl_from = c->bwd_cpl_from;
    g.flags = ows.oflags.as<uint32_t>(); g.dsw = c->ds;
    g.uniq = ows.uniq.as<uint64_t>(); g.insert_keys = c->split_resolved[slot] ? 0 : 1;
    g.choff = ows.flags.as<uint32_t>(); g.chunk_seg = ows.rowtmp.as<uint32_t>();
    g.nchunks = &ods->totals[1];
    DFX_TRY(ows.Vb.ensure((size_t)max_chunks(nnz) * (d + 2) * 8));
    g.part = ows.Vb.as<double>();
    DFX_TRY(bwd_two_pass_reserve(c, ows, nnz, &g));
    DFX_TRY(launch_bwd_chunks(g, max_chunks(nnz), c->stream, true));
    DFX_TRY(launch_bwd_fused(g, nnz, c->stream, c->bwd_lds));
  }
  // every owner takes part in the InitV ranking, with or without keys this step
  if (d > 0) {
    c->split_initv_pending[slot] = true;
    c->split_initv_gated[slot] = true;
  }
  // the slot is free and the store's counts final (capacity guard, cap_check) here at V_dim 0,
  // after the ranked InitV draws otherwise
  if (d == 0) {
    DFX_HIP(hipEventRecord(c->ev_free[slot], c->stream));
    c->slot_free[slot] = nullptr;
    DFX_TRY(cap_record(c));
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_split_owner_stats(dfx_ctx* ctx, int slot, int64_t* rows, int64_t* nnz,
                          int64_t* n_uniq) {
  DFX_CHECK_ARG(ctx && rows && nnz && n_uniq, "null argument");
  DFX_SPLIT_SLOT(slot);
  Context* c = &ctx->c;
  *rows = c->split_rows[slot];
  *nnz = c->split_nnz[slot];
  unsigned u = 0;
  if (c->ods[slot]) {
    DFX_HIP(hipMemcpyAsync(&u, &c->ods[slot]->u_count, sizeof(u), hipMemcpyDeviceToHost,
                           c->stream));
    DFX_HIP(hipStreamSynchronize(c->stream));
  }
  *n_uniq = u;
  return DFX_OK;
}

int dfx_split_initv_local(dfx_ctx* ctx, int slot, int64_t* count_dev) {
  DFX_CHECK_ARG(ctx && count_dev, "null argument");
  DFX_SPLIT_SLOT(slot);
  Context* c = &ctx->c;
  const Lane OL = split_owner_lane(c, slot);
  uint32_t* ftotal = &OL.ds->totals[2];
  const int64_t nnz = c->split_nnz[slot];
  if (!c->split_initv_pending[slot] || nnz == 0) {
    hipLaunchKernelGGL(k_split_zero_count, dim3(1), dim3(1), 0, OL.stream, ftotal, count_dev);
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  // the backward counts its requests in n_init: no requests (the steady state) skip the scan
  return initv_rank_count(OL, c->ows[slot].oflags.as<uint32_t>(), nnz, &OL.ds->u_count, ftotal,
                          c->split_initv_gated[slot] ? &c->ds->n_init : nullptr, count_dev);
}

int dfx_split_initv_draw(dfx_ctx* ctx, int slot, const int64_t* counts_all_dev, int rank,
                         int nranks) {
  DFX_CHECK_ARG(ctx && counts_all_dev, "null argument");
  DFX_SPLIT_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxDistRanks && rank >= 0 && rank < nranks,
                "split_initv_draw: bad rank");
  Context* c = &ctx->c;
  const Lane OL = split_owner_lane(c, slot);
  const bool pend = c->split_initv_pending[slot] && c->split_nnz[slot] > 0;
  const bool after_backward = c->split_initv_gated[slot];
  // after a backward: the draw's last block writes the store's counts for the capacity guard
  // (no copy on the stream), and the guard's event frees the slot too (one record)
  unsigned long long* cap = nullptr;
  if (after_backward) DFX_TRY(cap_record_slot(c, &cap));
  DFX_TRY(initv_rank_draw(c, OL, c->ows[slot].oflags.as<uint32_t>(), &OL.ds->totals[2],
                          &OL.ds->u_count, pend ? c->split_nnz[slot] : 0,
                          c->ows[slot].slot.as<uint32_t>(), counts_all_dev, rank, nranks,
                          &c->ds->n_init, cap));
  c->split_initv_pending[slot] = false;
  hipEvent_t fe = nullptr;
  if (cap) DFX_TRY(cap_record_commit(c, &fe));
  if (!fe) {
    DFX_HIP(hipEventRecord(c->ev_free[slot], c->stream));  // the slot's last reader
    fe = c->ev_free[slot];
  }
  c->slot_free[slot] = fe;
  return DFX_OK;
}

}  // extern "C"
