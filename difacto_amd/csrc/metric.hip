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
  const uint32_t* V = ds->sortmeta2[31] ? v1 : v0;
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
  const uint32_t* V = ds->sortmeta2[31] ? v1 : v0;
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
                            int64_t n, double* out) {
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
    *out = r;
  }
}

int auc_run(Context* c, int64_t B, const float* label, const float* pred, double* out_dev) {
  Workspace& ws = c->ws;
  if (B <= 0) {
    DFX_HIP(hipMemsetAsync(out_dev, 0, sizeof(double), c->stream));
    return DFX_OK;
  }
  DFX_TRY(ws.ak0.ensure(B * 4));
  DFX_TRY(ws.ak1.ensure(B * 4));
  DFX_TRY(ws.av0.ensure(B * 4));
  DFX_TRY(ws.av1.ensure(B * 4));
  const int64_t ntiles = (B + kMTile - 1) / kMTile;
  DFX_TRY(ws.atiles.ensure(ntiles * 4 + ntiles * 8 + 64));
  uint32_t* tiles = ws.atiles.as<uint32_t>();
  double* part = reinterpret_cast<double*>(ws.atiles.as<char>() + ((ntiles * 4 + 15) / 16) * 16);
  uint32_t* k0 = ws.ak0.as<uint32_t>();
  uint32_t* v0 = ws.av0.as<uint32_t>();
  hipLaunchKernelGGL(k_auc_keys, dim3((B + 255) / 256), dim3(256), 0, c->stream, B, label, pred,
                     k0, v0);
  DFX_TRY(radix_sort_pairs<uint32_t>(c, k0, v0, ws.ak1.as<uint32_t>(), ws.av1.as<uint32_t>(), B,
                                     0, 32, nullptr, c->ds->sortmeta2));
  hipLaunchKernelGGL(k_auc_tiles, dim3(ntiles), dim3(kMNT), 0, c->stream, v0,
                     ws.av1.as<uint32_t>(), B, c->ds, tiles);
  uint32_t* npos = &c->ds->totals[7];
  scan_tiles_top(c, tiles, ntiles, npos);
  hipLaunchKernelGGL(k_auc_area, dim3(ntiles), dim3(kMNT), 0, c->stream, v0,
                     ws.av1.as<uint32_t>(), B, c->ds, tiles, part);
  hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1024), 0, c->stream, part, ntiles, npos, B,
                     out_dev);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
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
  DFX_TRY(auc_run(c, B, label, pred, o));
  DFX_HIP(hipMemcpyAsync(auc_n, o, 8, hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  return DFX_OK;
}
