// Loss::Evaluate (include/difacto/loss.h:57-66) and BinClassMetric::AUC
// (src/loss/bin_class_metric.h:35-57) on the device, deterministic.
//
// AUC: stable radix sort of (orderable(pred), label>0) -> per-tile positive counts -> scan
// -> each negative adds the number of positives ranked below it.  The area is an exact
// integer (double up to 2^53); the reference accumulates it in float, so the two agree to
// float rounding (ties between equal predictions are implementation-defined in the
// reference's unstable std::sort; ours keep input order).
#include <vector>

#include "internal.h"

namespace dfx {

constexpr int kMNT = 256;
constexpr int kMItems = 8;
constexpr int kMTile = kMNT * kMItems;

__global__ void k_auc_keys(int64_t B, const float* label, const float* pred, uint32_t* k,
                           uint32_t* v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  uint32_t u = __float_as_uint(pred[i] + 0.0f);  // -0 == +0, as operator< sees them
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  k[i] = u;
  v[i] = label[i] > 0 ? 1u : 0u;
}

// the sorted labels: V0, or V1 when *sel (a radix sort's result buffer, known on the device)
__device__ inline const uint32_t* auc_labels(const uint32_t* V0, const uint32_t* V1,
                                             const unsigned* sel) {
  return (sel && *sel) ? V1 : V0;
}

__global__ __launch_bounds__(kMNT) void k_auc_tiles(const uint32_t* V0, const uint32_t* V1,
                                                    const unsigned* sel, int64_t n,
                                                    uint32_t* tiles) {
  __shared__ uint32_t lds[kMNT / kWave + 1];
  const uint32_t* V = auc_labels(V0, V1, sel);
  const int64_t base = (int64_t)blockIdx.x * kMTile + (int64_t)threadIdx.x * kMItems;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kMItems; ++i) s += (base + i < n) ? V[base + i] : 0u;
  uint32_t tot;
  block_excl_scan<kMNT>(s, lds, &tot);
  if (threadIdx.x == 0) tiles[blockIdx.x] = tot;
}

// per tile of the sorted labels: every negative adds the positives ranked below it (the
// tile's base from the scan of tile sums), summed exactly in double (integers below 2^53)
__global__ __launch_bounds__(kMNT) void k_auc_area_tiles(const uint32_t* V0, const uint32_t* V1,
                                                         const unsigned* sel, int64_t n,
                                                         const uint32_t* tilebase,
                                                         double* part) {
  __shared__ uint32_t lds[kMNT / kWave + 1];
  const uint32_t* V = auc_labels(V0, V1, sel);
  __shared__ double red[kMNT / kWave];
  const int64_t base = (int64_t)blockIdx.x * kMTile + (int64_t)threadIdx.x * kMItems;
  uint32_t lab[kMItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kMItems; ++i) {
    lab[i] = (base + i < n) ? V[base + i] : 0u;
    s += lab[i];
  }
  uint32_t cum = block_excl_scan<kMNT>(s, lds, nullptr) + tilebase[blockIdx.x];
  double area = 0;
#pragma unroll
  for (int i = 0; i < kMItems; ++i) {
    if (base + i >= n) break;
    if (lab[i]) cum += 1; else area += (double)cum;
  }
  for (int off = 32; off > 0; off >>= 1) area += __shfl_xor(area, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = area;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0;
    for (int i = 0; i < kMNT / kWave; ++i) a += red[i];
    part[blockIdx.x] = a;
  }
}

__global__ void k_auc_final(const double* part, int64_t ntiles, const uint32_t* npos_p,
                            int64_t n, double* out, int accumulate) {
  __shared__ double red[1024 / kWave];
  double a = 0;
  for (int64_t i = threadIdx.x; i < ntiles; i += blockDim.x) a += part[i];
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double area = 0;
    for (int i = 0; i < (int)(blockDim.x / kWave); ++i) area += red[i];
    const double P = (double)*npos_p;
    double r;
    if (P == 0 || P == (double)n) {
      r = 1.0;  // the reference returns 1 here (bin_class_metric.h:53), not 1*n
    } else {
      area /= P * ((double)n - P);
      r = (area < 0.5 ? 1 - area : area) * (double)n;
    }
    *out = accumulate ? *out + r : r;
  }
}

// snapshot of (orderable pred, label > 0) into the lane's sort buffers, on `st`
int auc_snapshot(const Lane& L, hipStream_t st, int64_t B, const float* label,
                 const float* pred) {
  Workspace& ws = *L.ws;
  if (B <= 0) return DFX_OK;
  DFX_TRY(auc_reserve(ws, B, L.stream));
  hipLaunchKernelGGL(k_auc_keys, dim3((B + 255) / 256), dim3(256), 0, st, B, label, pred,
                     ws.ak0.as<uint32_t>(), ws.av0.as<uint32_t>());
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// ---- the AUC lane: a stable sort, then a tiled counting pass ---------------------------------
// Beside the backward the AUC needs only to finish within a step, taking as few CU slots and
// as little memory traffic from the backward as possible.  Two sorts (context kwarg auc_sort):
//   radix (default)   the onesweep LSD radix sort (sort.hip) of (orderable pred, label) on the
//                     pred's four 8-bit digits (constant digits skipped): a B = 100 k snapshot
//                     is 25 tiles per pass, so the look-back blocks are few and short-lived
//   merge             k_auc_runs: one block per 4096-item tile (input order) sorts the tile in
//                     LDS into u64 keys (orderable pred << 32 | input index) and labels; then
//                     log2(tiles) rounds of LDS-tiled pairwise merges (sort.hip merge_runs):
//                     with the input index in the key every comparison is strict.  Each round
//                     waits on dependent global binary searches (~35 us per round at 100 k)
// Both are the global stable sort by pred (ties in input order), so the results are equal.
//   k_auc_tiles / k_auc_area_tiles / k_auc_final   positives per 2048-item tile, their scan,
//                     each negative's count of positives ranked below it (exact in double),
//                     AUC*n with the flip and the P = 0 / n rule
constexpr int kArNT = 256, kArItems = 16, kArTile = kArNT * kArItems;  // 4096

__global__ __launch_bounds__(kArNT) void k_auc_runs(int64_t n, const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ lab,
                                                   uint64_t* __restrict__ skey,
                                                   uint32_t* __restrict__ slab) {
  __shared__ uint32_t lk[2][kArTile];
  __shared__ uint16_t ll[2][kArTile];  // (index in the tile << 1) | label
  __shared__ uint32_t wcnt[kArNT / kWave][256];
  __shared__ uint32_t lds[kArNT / kWave + 1];
  const int t = threadIdx.x, w = t / kWave, l = lane_id();
  const int64_t tb = (int64_t)blockIdx.x * kArTile;
  const int m = (int)((n - tb) < kArTile ? (n - tb) : kArTile);
  for (int i = t; i < kArTile; i += kArNT) {
    lk[0][i] = i < m ? key[tb + i] : 0u;
    ll[0][i] = i < m ? (uint16_t)((i << 1) | (lab[tb + i] & 1u)) : (uint16_t)0;
  }
  __syncthreads();
  int src = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    for (int i = t; i < (kArNT / kWave) * 256; i += kArNT) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t dr[kArItems];
    const int wb = w * kWave * kArItems;
#pragma unroll
    for (int c = 0; c < kArItems; ++c) {
      const int idx = wb + c * kWave + l;
      const bool valid = idx < m;
      const uint32_t d = (lk[src][idx] >> shift) & 255u;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t mb = __ballot(valid && bit);
        peers &= bit ? mb : ~mb;
      }
      if (!valid) peers = 0;
      const uint32_t r = (uint32_t)__popcll(peers & lanemask_lt());
      const uint32_t old = valid ? wcnt[w][d] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (valid && r == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      dr[c] = d | ((old + r) << 8);
    }
    __syncthreads();
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < kArNT / kWave; ++i) {
      const uint32_t x = wcnt[i][t];
      wcnt[i][t] = cnt;
      cnt += x;
    }
    // digit d's start in the tile, folded into the waves' offsets: wcnt[w][d] += start(d)
    const uint32_t start = block_excl_scan<kArNT>(cnt, lds, nullptr);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kArNT / kWave; ++i) wcnt[i][t] += start;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kArItems; ++c) {
      const int idx = wb + c * kWave + l;
      if (idx < m) {
        const uint32_t d = dr[c] & 255u;
        const uint32_t pos = wcnt[w][d] + (dr[c] >> 8);
        lk[src ^ 1][pos] = lk[src][idx];
        ll[src ^ 1][pos] = ll[src][idx];
      }
    }
    __syncthreads();
    src ^= 1;
  }
  // the sorted tile out: the input index breaks ties, keeping the sort stable across tiles
  for (int i = t; i < m; i += kArNT) {
    const uint32_t q = ll[src][i];
    skey[tb + i] = ((uint64_t)lk[src][i] << 32) | (uint64_t)(tb + (q >> 1));
    slab[tb + i] = q & 1u;
  }
}

// Small snapshots (B <= kAbMax, e.g. B = 10^4 rows per GPU): ONE 1024-thread block sorts
// (orderable pred, input index << 1 | label) in LDS — four stable 8-bit LSD passes ranked by
// wave ballots as in k_auc_runs — then scans the sorted labels and adds, per negative, the
// positives ranked below it, and writes AUC*n (k_auc_final's rules): one launch, where the
// radix lane takes ~14 latency-bound launches (~0.12 ms of lane time at B = 10^4,
// profiles/r3/kernel_summary_b1e4_pipelined.md).  Same stable order, so the same AUC exactly.
constexpr int kAbNT = 1024, kAbItems = 12, kAbMax = kAbNT * kAbItems;  // 12288 rows, 152 KiB
static_assert(kAbMax == kAucBlockMax, "internal.h names the one-block AUC's limit");

__global__ __launch_bounds__(kAbNT) void k_auc_block(int64_t n, const uint32_t* __restrict__ key,
                                                     const uint32_t* __restrict__ lab,
                                                     double* out, int accumulate) {
  __shared__ uint32_t lk[2][kAbMax];
  __shared__ uint16_t ll[2][kAbMax];  // (input index << 1) | label
  __shared__ uint16_t wcnt[kAbNT / kWave][256];
  __shared__ uint32_t lds[kAbNT / kWave + 1];
  __shared__ double red[kAbNT / kWave];
  const int t = threadIdx.x, w = t / kWave, l = lane_id();
  const int m = (int)n;
  for (int i = t; i < m; i += kAbNT) {
    lk[0][i] = key[i];
    ll[0][i] = (uint16_t)((i << 1) | (lab[i] & 1u));
  }
  __syncthreads();
  int src = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 8 * pass;
    for (int i = t; i < (kAbNT / kWave) * 256; i += kAbNT) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t dr[kAbItems];
    const int wb = w * kWave * kAbItems;  // wave w ranks items [wb, wb + 64 * kAbItems) in order
#pragma unroll
    for (int c = 0; c < kAbItems; ++c) {
      const int idx = wb + c * kWave + l;
      const bool valid = idx < m;
      const uint32_t d = valid ? (lk[src][idx] >> shift) & 255u : 0u;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t mb = __ballot(valid && bit);
        peers &= bit ? mb : ~mb;
      }
      if (!valid) peers = 0;
      const uint32_t r = (uint32_t)__popcll(peers & lanemask_lt());
      const uint32_t old = valid ? wcnt[w][d] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (valid && r == 0) wcnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
      __builtin_amdgcn_wave_barrier();
      dr[c] = d | ((old + r) << 8);
    }
    __syncthreads();
    // per digit (threads 0..255): the waves' exclusive offsets, then the digits' starts
    uint32_t cnt = 0;
    if (t < 256) {
#pragma unroll
      for (int i = 0; i < kAbNT / kWave; ++i) {
        const uint32_t x = wcnt[i][t];
        wcnt[i][t] = (uint16_t)cnt;
        cnt += x;
      }
    }
    const uint32_t start = block_excl_scan<kAbNT>(cnt, lds, nullptr);
    if (t < 256) {
#pragma unroll
      for (int i = 0; i < kAbNT / kWave; ++i) wcnt[i][t] = (uint16_t)(wcnt[i][t] + start);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kAbItems; ++c) {
      const int idx = wb + c * kWave + l;
      if (idx < m) {
        const uint32_t d = dr[c] & 255u;
        const uint32_t pos = wcnt[w][d] + (dr[c] >> 8);
        lk[src ^ 1][pos] = lk[src][idx];
        ll[src ^ 1][pos] = ll[src][idx];
      }
    }
    __syncthreads();
    src ^= 1;
  }
  // the sorted labels: thread t holds items [t * kAbItems, ...); positives below each negative
  const int base = t * kAbItems;
  uint32_t lb[kAbItems], s = 0;
#pragma unroll
  for (int c = 0; c < kAbItems; ++c) {
    lb[c] = base + c < m ? (uint32_t)(ll[src][base + c] & 1u) : 0u;
    s += lb[c];
  }
  uint32_t npos = 0;
  uint32_t cum = block_excl_scan<kAbNT>(s, lds, &npos);
  double area = 0;
#pragma unroll
  for (int c = 0; c < kAbItems; ++c) {
    if (lb[c]) cum += 1;
    else if (base + c < m) area += (double)cum;
  }
  for (int off = 32; off > 0; off >>= 1) area += __shfl_xor(area, off, kWave);
  if (l == 0) red[w] = area;
  __syncthreads();
  if (t == 0) {
    double a = 0;
    for (int i = 0; i < kAbNT / kWave; ++i) a += red[i];
    const double P = (double)npos;
    double r;
    if (P == 0 || P == (double)n) {
      r = 1.0;  // the reference returns 1 here (bin_class_metric.h:53), not 1*n
    } else {
      a /= P * ((double)n - P);
      r = (a < 0.5 ? 1 - a : a) * (double)n;
    }
    *out = accumulate ? *out + r : r;
  }
}

// AUC*n of the snapshot (keys ak0, labels av0) into *out_dev (accumulate: += ), on the lane
int auc_finish(const Lane& L, int64_t B, double* out_dev, bool accumulate, int mode) {
  Workspace& ws = *L.ws;
  if (B <= 0) {
    if (!accumulate) DFX_HIP(hipMemsetAsync(out_dev, 0, sizeof(double), L.stream));
    return DFX_OK;
  }
  DFX_TRY(auc_reserve(ws, B, L.stream));
  if (B <= kAbMax) {  // one block in LDS (every auc_sort mode: the same stable order)
    hipLaunchKernelGGL(k_auc_block, dim3(1), dim3(kAbNT), 0, L.stream, B,
                       ws.ak0.as<uint32_t>(), ws.av0.as<uint32_t>(), out_dev,
                       accumulate ? 1 : 0);
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  const bool radix = mode != 0;
  const int64_t ntiles = (B + kArTile - 1) / kArTile;
  const uint32_t* V0 = nullptr;
  const uint32_t* V1 = nullptr;
  const unsigned* sel = nullptr;
  if (radix || ntiles > kMaxMergeRuns) {
    // the snapshot (ak0, av0) ping-pongs with (keys0, vals0) reinterpreted as u32; the
    // result's buffer follows the number of active passes: sortmeta[31], read on the device
    uint32_t* k1 = ws.keys0.as<uint32_t>();
    uint32_t* v1 = ws.vals0.as<uint32_t>();
    DFX_TRY((radix_sort_pairs<uint32_t, uint32_t>(L, ws.ak0.as<uint32_t>(), ws.av0.as<uint32_t>(),
                                                  k1, v1, B, 0, 32, nullptr, L.ds->sortmeta)));
    V0 = ws.av0.as<uint32_t>();
    V1 = v1;
    sel = &L.ds->sortmeta[31];
  } else {
    // runs into (keys1, vals1): merge_runs ping-pongs through keys0 / keys1
    uint64_t* kr = ws.keys1.as<uint64_t>();
    uint32_t* vr = ws.vals1.as<uint32_t>();
    hipLaunchKernelGGL(k_auc_runs, dim3((unsigned)ntiles), dim3(kArNT), 0, L.stream, B,
                       ws.ak0.as<uint32_t>(), ws.av0.as<uint32_t>(), kr, vr);
    const uint64_t* K = kr;
    const uint32_t* V = vr;
    if (ntiles > 1) {
      std::vector<int64_t> runs;
      for (int64_t r = 0; r < ntiles; ++r) runs.push_back(r * kArTile);
      runs.push_back(B);
      // merge_runs writes keys0 first: the runs in keys1 are read in the first round only
      merge_runs(L, runs, &K, &V);
    }
    V0 = V;
  }
  const int64_t nt = (B + kMTile - 1) / kMTile;
  DFX_TRY(ws.tiles.ensure(sizeof(uint32_t) * (nt + 2)));
  DFX_TRY(ws.dscratch.ensure(sizeof(double) * (nt + 8)));
  uint32_t* tiles = ws.tiles.as<uint32_t>();
  uint32_t* npos = tiles + nt + 1;
  hipLaunchKernelGGL(k_auc_tiles, dim3((unsigned)nt), dim3(kMNT), 0, L.stream, V0, V1, sel, B,
                     tiles);
  scan_tiles_top(L, tiles, nt, npos);
  double* part = ws.dscratch.as<double>();
  hipLaunchKernelGGL(k_auc_area_tiles, dim3((unsigned)nt), dim3(kMNT), 0, L.stream, V0, V1, sel,
                     B, tiles, part);
  hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1024), 0, L.stream, part, nt, npos, B, out_dev,
                     accumulate ? 1 : 0);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int auc_run(const Lane& L, int64_t B, const float* label, const float* pred, double* out_dev,
            int mode) {
  DFX_TRY(auc_snapshot(L, L.stream, B, label, pred));
  return auc_finish(L, B, out_dev, false, mode);
}

__global__ void k_eval_part(int64_t B, const float* label, const float* pred, double* part) {
  __shared__ double red[kMNT / kWave];
  const int64_t i = (int64_t)blockIdx.x * kMNT + threadIdx.x;
  double v = 0;
  if (i < B) {
    const double y = label[i] > 0 ? 1.0 : -1.0;
    v = log(1.0 + exp(-y * (double)pred[i]));
  }
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int k = 0; k < kMNT / kWave; ++k) s += red[k];
    part[blockIdx.x] = s;
  }
}

__global__ void k_sum_parts(const double* part, int64_t n, double* out, int accumulate) {
  __shared__ double red[1024 / kWave];
  double a = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) a += part[i];
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int k = 0; k < (int)(blockDim.x / kWave); ++k) s += red[k];
    *out = accumulate ? *out + s : s;
  }
}

int evaluate_run(Context* c, int64_t B, const float* label, const float* pred, double* out_dev) {
  if (B <= 0) {
    DFX_HIP(hipMemsetAsync(out_dev, 0, sizeof(double), c->stream));
    return DFX_OK;
  }
  const int64_t nb = (B + kMNT - 1) / kMNT;
  DFX_TRY(c->ws.dscratch.ensure(nb * 8 + 64));
  double* part = c->ws.dscratch.as<double>() + 8;
  hipLaunchKernelGGL(k_eval_part, dim3(nb), dim3(kMNT), 0, c->stream, B, label, pred, part);
  hipLaunchKernelGGL(k_sum_parts, dim3(1), dim3(1024), 0, c->stream, part, nb, out_dev, 0);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

void sum_parts(Context* c, const double* part, int64_t n, double* out, bool accumulate) {
  hipLaunchKernelGGL(k_sum_parts, dim3(1), dim3(1024), 0, c->stream, part, n, out,
                     accumulate ? 1 : 0);
}

}  // namespace dfx

using namespace dfx;

extern "C" int dfx_evaluate(dfx_ctx* ctx, int64_t B, const float* label, const float* pred,
                            double* objv) {
  DFX_CHECK_ARG(ctx && objv, "null argument");
  Context* c = &ctx->c;
  double* o = &c->ds->scratch[1];
  DFX_TRY(evaluate_run(c, B, label, pred, o));
  DFX_HIP(hipMemcpyAsync(objv, o, 8, hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  return DFX_OK;
}

extern "C" int dfx_auc(dfx_ctx* ctx, int64_t B, const float* label, const float* pred,
                       double* auc_n) {
  DFX_CHECK_ARG(ctx && auc_n, "null argument");
  Context* c = &ctx->c;
  double* o = &c->ds->scratch[2];
  DFX_TRY(auc_run(main_lane(c), B, label, pred, o, c->auc_sort));
  DFX_HIP(hipMemcpyAsync(auc_n, o, 8, hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  return DFX_OK;
}
