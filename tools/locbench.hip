// The fused step's Localizer alone, on the GPU: a C3-shaped batch (B rows of k ids uniform
// below 2^kbits, generated on the device) localized `iters` times on the context stream, as
// the fused step's lane does (no col: the bucket Localizer, or the radix one with
// loc_bucket=0), timed with events; run it under rocprofv3 --kernel-trace for per-kernel
// times.  With a sixth argument "auc": the AUC lane's sort + area of a B-row (pred, label)
// snapshot instead (auc_sort from the kwargs).  Measurement tool (links the library's
// internals), not a test.
//   build/locbench [B] [k] [kbits] [iters] [context kwargs] [auc | valued | zipf]
// zipf: Zipf(1.1) keys, a fresh batch every iteration (untimed), the chunk plan timed with the
// Localizer as the fused step's lane runs it
#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "../difacto_amd/csrc/internal.h"

__global__ void k_gen(int64_t B, int k, int kbits, uint64_t* offs, uint64_t* ids, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= B) offs[i] = (uint64_t)i * k;
  if (i >= B * k) return;
  uint64_t x = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;  // splitmix64
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  ids[i] = x >> (64 - kbits);
}

// Zipf(s) ranks over [1, 2^kbits] by the continuous inverse CDF (C5's keys, approximately)
__global__ void k_gen_zipf(int64_t B, int k, int kbits, double zs, uint64_t* offs, uint64_t* ids,
                           uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= B) offs[i] = (uint64_t)i * k;
  if (i >= B * k) return;
  uint64_t x = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;  // splitmix64
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
  const double N = (double)(1ull << kbits), a = 1.0 - zs;
  double r = pow((pow(N + 1.0, a) - 1.0) * u + 1.0, 1.0 / a);
  uint64_t rk = (uint64_t)r;
  ids[i] = rk < 1 ? 1 : (rk > (1ull << kbits) ? (1ull << kbits) : rk);
}

__global__ void k_gen_pred(int64_t B, float* pred, float* lab, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  uint64_t x = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = (float)(x >> 40) * (1.0f / 16777216.0f);
  lab[i] = ((x >> 8) & 3) == 0 ? 1.0f : 0.0f;
  pred[i] = 6.0f * (u - 0.5f) + (lab[i] > 0 ? 0.7f : 0.0f);  // overlapping classes
}

static int auc_bench(dfx::Context* c, int64_t B, int iters, const char* kw) {
  float *pred, *lab;
  double* out;
  hipMalloc(&pred, B * 4);
  hipMalloc(&lab, B * 4);
  hipMalloc(&out, 8);
  hipLaunchKernelGGL(k_gen_pred, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, c->stream, B,
                     pred, lab, 7ull);
  dfx::Lane L = dfx::main_lane(c);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double tot = 0;
  for (int it = 0; it < iters + 2; ++it) {
    hipEventRecord(e0, c->stream);
    if (dfx::auc_run(L, B, lab, pred, out, c->auc_sort) != DFX_OK) {
      fprintf(stderr, "auc: %s\n", dfx_last_error());
      return 1;
    }
    hipEventRecord(e1, c->stream);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (it >= 2) tot += ms;
  }
  double r = 0;
  hipMemcpy(&r, out, 8, hipMemcpyDeviceToHost);
  printf("aucbench B=%lld kwargs='%s': %.4f ms per AUC (snapshot + sort + area), AUC*n=%.1f\n",
         (long long)B, kw, tot / iters, r);
  return 0;
}

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? atoll(argv[1]) : 100000;
  const int k = argc > 2 ? atoi(argv[2]) : 39;
  const int kbits = argc > 3 ? atoi(argv[3]) : 24;
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  const char* kw = argc > 5 ? argv[5] : "";
  const int64_t nnz = B * k;
  dfx_ctx* ctx = nullptr;
  if (dfx_ctx_create(0, kw, &ctx) != DFX_OK) {
    fprintf(stderr, "ctx: %s\n", dfx_last_error());
    return 1;
  }
  dfx::Context* c = &ctx->c;
  if (argc > 6 && std::string(argv[6]) == "auc") {
    const int rc = auc_bench(c, B, iters, kw);
    dfx_ctx_destroy(ctx);
    return rc;
  }
  const bool valued = argc > 6 && std::string(argv[6]) == "valued";
  const bool zipf = argc > 6 && std::string(argv[6]) == "zipf";
  uint32_t *choff = nullptr, *chseg = nullptr, *nch = nullptr;
  if (zipf) {
    hipMalloc(&choff, (nnz + 1) * 4);
    hipMalloc(&chseg, dfx::max_chunks(nnz) * 4);
    hipMalloc(&nch, 4);
  }
  uint64_t *offs, *ids, *uniq;
  uint32_t *seg, *occ;
  float *val = nullptr, *occx = nullptr;
  hipMalloc(&offs, (B + 1) * 8);
  hipMalloc(&ids, nnz * 8);
  hipMalloc(&uniq, nnz * 8);
  hipMalloc(&seg, (nnz + 1) * 4);
  hipMalloc(&occ, nnz * 4);
  if (valued) {  // values 1.0 (their bits travel as well as any)
    hipMalloc(&val, nnz * 4);
    hipMalloc(&occx, nnz * 4);
    hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(val), 0x3f800000u, nnz);
  }
  hipLaunchKernelGGL(k_gen, dim3((unsigned)((nnz + 256) / 256)), dim3(256), 0, c->stream, B, k,
                     kbits, offs, ids, 42ull);
  dfx::Lane L = dfx::main_lane(c);
  dfx::LocOut o;
  o.uniq = uniq;
  o.segstart = seg;
  o.occ_row = occ;
  o.value = val;
  o.occ_x = occx;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double tot = 0;
  for (int it = 0; it < iters + 2; ++it) {
    if (zipf)
      hipLaunchKernelGGL(k_gen_zipf, dim3((unsigned)((nnz + 256) / 256)), dim3(256), 0, c->stream,
                         B, k, kbits, 1.1, offs, ids, 42ull + 7919ull * it);
    hipEventRecord(e0, c->stream);
    if (dfx::localize_run(c, L, B, nnz, offs, ids, ~0ull, o) != DFX_OK) {
      fprintf(stderr, "localize: %s\n", dfx_last_error());
      return 1;
    }
    if (zipf && dfx::chunk_plan(L, nnz, seg, choff, chseg, nch) != DFX_OK) {
      fprintf(stderr, "chunk plan: %s\n", dfx_last_error());
      return 1;
    }
    hipEventRecord(e1, c->stream);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (it >= 2) tot += ms;
  }
  unsigned u = 0;
  hipMemcpy(&u, &c->ds->u_count, 4, hipMemcpyDeviceToHost);
  int err = 0;
  hipMemcpy(&err, &c->ds->err, 4, hipMemcpyDeviceToHost);
  printf("locbench B=%lld k=%d kbits=%d kwargs='%s'%s: %.4f ms per Localizer, U=%u, err=%d\n",
         (long long)B, k, kbits, kw, valued ? " valued" : zipf ? " zipf (+ chunk plan)" : "",
         tot / iters, u, err);
  dfx_ctx_destroy(ctx);
  return 0;
}
