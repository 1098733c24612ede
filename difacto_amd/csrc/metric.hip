// Loss::Evaluate (include/difacto/loss.h:57-66) and BinClassMetric::AUC
// (src/loss/bin_class_metric.h:35-57) on the device, deterministic.
//
// AUC: stable radix sort of (orderable(pred), label>0) -> per-tile positive counts -> scan
// -> each negative adds the number of positives ranked below it.  The area is an exact
// integer (double up to 2^53); the reference accumulates it in float, so the two agree to
// float rounding (ties between equal predictions are implementation-defined in the
// reference's unstable std::sort; ours keep input order).
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

__global__ __launch_bounds__(kMNT) void k_auc_tiles(const uint32_t* v0, const uint32_t* v1,
                                                    int64_t n, const DevState* ds,
                                                    uint32_t* tiles) {
  __shared__ uint32_t lds[kMNT / kWave + 1];
  const uint32_t* V = ds->sortmeta[31] ? v1 : v0;
  const int64_t base = (int64_t)blockIdx.x * kMTile + (int64_t)threadIdx.x * kMItems;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kMItems; ++i) s += (base + i < n) ? V[base + i] : 0u;
  uint32_t tot;
  block_excl_scan<kMNT>(s, lds, &tot);
  if (threadIdx.x == 0) tiles[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kMNT) void k_auc_area(const uint32_t* v0, const uint32_t* v1,
                                                   int64_t n, const DevState* ds,
                                                   const uint32_t* tilebase, double* part) {
  __shared__ uint32_t lds[kMNT / kWave + 1];
  __shared__ double red[kMNT / kWave];
  const uint32_t* V = ds->sortmeta[31] ? v1 : v0;
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
  DFX_TRY(ws.ak0.ensure(B * 4));
  DFX_TRY(ws.ak1.ensure(B * 4));
  DFX_TRY(ws.av0.ensure(B * 4));
  DFX_TRY(ws.av1.ensure(B * 4));
  hipLaunchKernelGGL(k_auc_keys, dim3((B + 255) / 256), dim3(256), 0, st, B, label, pred,
                     ws.ak0.as<uint32_t>(), ws.av0.as<uint32_t>());
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// ---- the AUC lane: sorted runs + binary-search counting, no inter-block waits ----------
// Beside the backward the AUC needs only to finish within a step, and its blocks must never
// park on CUs the backward needs (a look-back sort's spinning blocks would).  So:
//   k_auc_runs   one block per 4096-item tile (input order): stable LSD sort of the tile in
//                LDS; sorted keys, the exclusive prefix count of positives, the tile's own
//                area (positives before each negative inside the tile) and positive count
//   k_auc_cross  one thread per (item, other tile): a negative with key x in tile r counts
//                the positives of tile r' < r with key <= x (they precede it in a stable
//                sort) and of tile r' > r with key < x — a binary search in the sorted tile
//   k_auc_sum    area and positives summed in a fixed order -> AUC*n (flip, P = 0 / n rule)
// Every partial is an integer held exactly in double, so the result is deterministic and
// equals the global stable sort's rank-sum.
constexpr int kArNT = 256, kArItems = 16, kArTile = kArNT * kArItems;  // 4096

__global__ __launch_bounds__(kArNT) void k_auc_runs(int64_t n, const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ lab,
                                                   uint32_t* __restrict__ skey,
                                                   uint32_t* __restrict__ ppre,
                                                   double* __restrict__ part,
                                                   uint32_t* __restrict__ npos) {
  __shared__ uint32_t lk[2][kArTile];
  __shared__ uint8_t ll[2][kArTile];
  __shared__ uint32_t wcnt[kArNT / kWave][256];
  __shared__ uint32_t lds[kArNT / kWave + 1];
  __shared__ double dred[kArNT / kWave];
  const int t = threadIdx.x, w = t / kWave, l = lane_id();
  const int64_t tb = (int64_t)blockIdx.x * kArTile;
  const int m = (int)((n - tb) < kArTile ? (n - tb) : kArTile);
  for (int i = t; i < kArTile; i += kArNT) {
    lk[0][i] = i < m ? key[tb + i] : 0u;
    ll[0][i] = i < m ? (uint8_t)lab[tb + i] : (uint8_t)0;
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
  // sorted tile out; exclusive prefix of positives; the tile's own area
  double area = 0;
  uint32_t carry = 0;
  uint32_t* pp = ppre + (int64_t)blockIdx.x * (kArTile + 1);
  for (int cb = 0; cb < kArTile; cb += kArNT) {
    const int i = cb + t;
    const uint32_t y = i < m ? (uint32_t)ll[src][i] : 0u;
    uint32_t tot;
    const uint32_t before = block_excl_scan<kArNT>(y, lds, &tot) + carry;
    if (i < m) {
      skey[tb + i] = lk[src][i];
      pp[i] = before;
      if (!y) area += (double)before;
    }
    carry += tot;
  }
  if (t == 0) pp[m] = carry;
  for (int off = 32; off > 0; off >>= 1) area += __shfl_xor(area, off, kWave);
  if (l == 0) dred[w] = area;
  __syncthreads();
  if (t == 0) {
    double a = 0;
    for (int i = 0; i < kArNT / kWave; ++i) a += dred[i];
    part[blockIdx.x] = a;
    npos[blockIdx.x] = carry;
  }
}

__global__ __launch_bounds__(256) void k_auc_cross(int64_t n, int ntiles,
                                                   const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ lab,
                                                   const uint32_t* __restrict__ skey,
                                                   const uint32_t* __restrict__ ppre,
                                                   double* __restrict__ part2) {
  __shared__ double dred[256 / kWave];
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = g / ntiles;
  const int rr = (int)(g % ntiles);
  double add = 0;
  if (i < n && !lab[i]) {
    const int r = (int)(i / kArTile);
    if (rr != r) {
      const uint32_t x = key[i];
      const int64_t b = (int64_t)rr * kArTile;
      const int len = (int)((n - b) < kArTile ? (n - b) : kArTile);
      const uint32_t* sk = skey + b;
      int lo = 0, hi = len;  // first index with sk > x (rr < r) or sk >= x (rr > r)
      if (rr < r) {
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (sk[mid] <= x) lo = mid + 1; else hi = mid; }
      } else {
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (sk[mid] < x) lo = mid + 1; else hi = mid; }
      }
      add = (double)ppre[(int64_t)rr * (kArTile + 1) + lo];
    }
  }
  for (int off = 32; off > 0; off >>= 1) add += __shfl_xor(add, off, kWave);
  if (lane_id() == 0) dred[threadIdx.x / kWave] = add;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0;
    for (int k = 0; k < 256 / kWave; ++k) a += dred[k];
    part2[blockIdx.x] = a;
  }
}

__global__ __launch_bounds__(1024) void k_auc_sum(int64_t n, int ntiles, const double* part,
                                                  const uint32_t* npos, int64_t nb2,
                                                  const double* part2, double* out,
                                                  int accumulate) {
  __shared__ double red[1024 / kWave];
  __shared__ uint32_t pred_[1024 / kWave];
  double a = 0;
  uint32_t P = 0;
  for (int64_t i = threadIdx.x; i < nb2; i += 1024) a += part2[i];
  for (int i = threadIdx.x; i < ntiles; i += 1024) { a += part[i]; P += npos[i]; }
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, kWave);
    P += __shfl_xor(P, off, kWave);
  }
  if (lane_id() == 0) { red[threadIdx.x / kWave] = a; pred_[threadIdx.x / kWave] = P; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double area = 0;
    double Pd = 0;
    for (int i = 0; i < 1024 / kWave; ++i) { area += red[i]; Pd += (double)pred_[i]; }
    double r;
    if (Pd == 0 || Pd == (double)n) {
      r = 1.0;  // the reference returns 1 here (bin_class_metric.h:53), not 1*n
    } else {
      area /= Pd * ((double)n - Pd);
      r = (area < 0.5 ? 1 - area : area) * (double)n;
    }
    *out = accumulate ? *out + r : r;
  }
}

// AUC*n of the snapshot into *out_dev (accumulate: += ), on the lane's stream
int auc_finish(const Lane& L, int64_t B, double* out_dev, bool accumulate) {
  Workspace& ws = *L.ws;
  if (B <= 0) {
    if (!accumulate) DFX_HIP(hipMemsetAsync(out_dev, 0, sizeof(double), L.stream));
    return DFX_OK;
  }
  const int ntiles = (int)((B + kArTile - 1) / kArTile);
  const int64_t pairs = B * (int64_t)ntiles;
  const int64_t nb2 = (pairs + 255) / 256;
  // ak1: sorted keys; av1: per-tile positive prefixes (ntiles * (kArTile + 1) u32); atiles:
  // per-tile area + positive count, then the cross partials
  DFX_TRY(ws.ak1.ensure(B * 4));
  DFX_TRY(ws.av1.ensure((size_t)ntiles * (kArTile + 1) * 4));
  DFX_TRY(ws.atiles.ensure(ntiles * 8 + ntiles * 4 + nb2 * 8 + 64));
  double* part = ws.atiles.as<double>();
  uint32_t* npos = reinterpret_cast<uint32_t*>(part + ntiles);
  double* part2 = reinterpret_cast<double*>(ws.atiles.as<char>() +
                                            ((ntiles * 12 + 15) / 16) * 16);
  const uint32_t* k0 = ws.ak0.as<uint32_t>();
  const uint32_t* v0 = ws.av0.as<uint32_t>();
  hipLaunchKernelGGL(k_auc_runs, dim3(ntiles), dim3(kArNT), 0, L.stream, B, k0, v0,
                     ws.ak1.as<uint32_t>(), ws.av1.as<uint32_t>(), part, npos);
  hipLaunchKernelGGL(k_auc_cross, dim3((unsigned)nb2), dim3(256), 0, L.stream, B, ntiles, k0, v0,
                     ws.ak1.as<uint32_t>(), ws.av1.as<uint32_t>(), part2);
  hipLaunchKernelGGL(k_auc_sum, dim3(1), dim3(1024), 0, L.stream, B, ntiles, part, npos, nb2,
                     part2, out_dev, accumulate ? 1 : 0);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int auc_run(const Lane& L, int64_t B, const float* label, const float* pred, double* out_dev) {
  DFX_TRY(auc_snapshot(L, L.stream, B, label, pred));
  return auc_finish(L, B, out_dev, false);
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
  DFX_TRY(auc_run(main_lane(c), B, label, pred, o));
  DFX_HIP(hipMemcpyAsync(auc_n, o, 8, hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  return DFX_OK;
}
