// Layout microbenchmark for the model store: a key's 32-B entry and its [V | Vaux] row in two
// arrays (the entry carries the row index) versus one "fat" slot holding the entry and the row
// together.  Two access shapes at the bench config (d = 16):
//   fwd: per nnz (3.9 M, random keys) read the entry's {w, vrow} and the 64-B V     (read only)
//   bwd: per unique key (3.48 M, key order = slot order when SORTED) read-modify-write the
//        entry's 16-B state and the 128-B [V | Vaux] row
// Build: hipcc --offload-arch=gfx950 -O3 slotbench.hip -o slotbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s\n", hipGetErrorString(e));                 \
      exit(1);                                              \
    }                                                       \
  } while (0)

// split: ent (32 B per slot), rows (128 B per row, row = permuted slot)
__global__ void fwd_split(const float4* ent, const float4* rows, const unsigned* idx, int n,
                          float* out) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  const float2 wv = *reinterpret_cast<const float2*>(ent + (size_t)s * 2);
  unsigned vr = __float_as_uint(wv.y);
  float4 v = rows[(size_t)vr * 8 + l];
  float acc = wv.x + v.x + v.y + v.z + v.w;
  if (acc == 12345.f) out[g] = acc;
}
// split, V row indexed by the slot: both loads issue at once
__global__ void fwd_split_par(const float4* ent, const float4* rows, const unsigned* idx, int n,
                              float* out) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  const float2 wv = *reinterpret_cast<const float2*>(ent + (size_t)s * 2);
  float4 v = rows[(size_t)s * 8 + l];
  if (__float_as_int(wv.y) < 0) v = make_float4(0.f, 0.f, 0.f, 0.f);
  float acc = wv.x + v.x + v.y + v.z + v.w;
  if (acc == 12345.f) out[g] = acc;
}
// fat: slot of SF float4s: entry (2 float4) then V (4) then Vaux (4)
template <int SF>
__global__ void fwd_fat(const float4* slots, const unsigned* idx, int n, float* out) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  const float4* p = slots + (size_t)s * SF;
  const float2 wv = *reinterpret_cast<const float2*>(p);
  float4 v = p[2 + l];
  float acc = wv.x + v.x + v.y + v.z + v.w;
  if (acc == 12345.f) out[g] = acc;
}
__global__ void bwd_split(float4* ent, float4* rows, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  float4 e = ent[(size_t)s * 2];
  unsigned vr = __float_as_uint(e.y);
  float4* p = rows + (size_t)vr * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += 1.f;
  c.y += 1.f;
  p[l] = v;
  p[4 + l] = c;
  if (l == 0) {
    e.x += 1.f;
    ent[(size_t)s * 2] = e;
  }
}
// split with V rows indexed by the slot: both arrays walked in address order
__global__ void bwd_split_slot(float4* ent, float4* rows, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  float4 e = ent[(size_t)s * 2];
  float4* p = rows + (size_t)s * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += e.x;
  c.y += 1.f;
  p[l] = v;
  p[4 + l] = c;
  if (l == 0) {
    e.x += 1.f;
    ent[(size_t)s * 2] = e;
  }
}
template <int SF>
__global__ void bwd_fat(float4* slots, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  float4* p = slots + (size_t)s * SF;
  float4 e = p[0];
  float4 v = p[2 + l], c = p[6 + l];
  v.x += e.x;
  c.y += 1.f;
  p[2 + l] = v;
  p[6 + l] = c;
  if (l == 0) {
    e.x += 1.f;
    p[0] = e;
  }
}
// fat 128 B: slot = [entry (2 float4) | V (4 float4) | pad (2)]; Vaux in a pool of 64-B rows,
// indexed by the slot (AUXSLOT) or by the entry's vrow (a permutation: allocation order)
template <bool AUXSLOT>
__global__ void bwd_fat128(float4* slots, float4* aux, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  float4* p = slots + (size_t)s * 8;
  float4 e = p[0];
  float4 v = p[2 + l];
  float4* q = aux + (AUXSLOT ? (size_t)s : (size_t)__float_as_uint(e.y)) * 4;
  float4 c = q[l];
  v.x += e.x;
  c.y += 1.f;
  p[2 + l] = v;
  q[l] = c;
  if (l == 0) {
    e.x += 1.f;
    p[0] = e;
  }
}
// fat 128 B, V first: slot = [V (4 float4) | entry (2 float4) | pad (2)] — V is one whole 64-B
// sector; E32: the entry is written back whole (32 B) instead of its 16-B hot half
template <bool E32>
__global__ void bwd_fatv(float4* slots, float4* aux, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  float4* p = slots + (size_t)s * 8;
  float4 e = p[4], e1 = p[5];
  float4 v = p[l];
  float4* q = aux + (size_t)s * 4;
  float4 c = q[l];
  v.x += e.x;
  c.y += 1.f;
  p[l] = v;
  q[l] = c;
  if (l == 0) {
    e.x += 1.f;
    p[4] = e;
    if (E32) p[5] = e1;
  }
}
__global__ void fwd_fatv(const float4* slots, const unsigned* idx, int n, float* out) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  const float4* p = slots + (size_t)s * 8;
  const float2 wv = *reinterpret_cast<const float2*>(p + 4);
  const float2 kk = *reinterpret_cast<const float2*>(p + 5) ;
  float4 v = p[l];
  float acc = wv.x + kk.y + v.x + v.y + v.z + v.w;
  if (acc == 12345.f) out[g] = acc;
}
// current layout, the entry written back whole (32 B)
__global__ void bwd_split32(float4* ent, float4* rows, const unsigned* idx, int n) {
  int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  unsigned s = idx[g];
  float4 e = ent[(size_t)s * 2], e1 = ent[(size_t)s * 2 + 1];
  unsigned vr = __float_as_uint(e.y);
  float4* p = rows + (size_t)vr * 8;
  float4 v = p[l], c = p[4 + l];
  v.x += 1.f;
  c.y += 1.f;
  p[l] = v;
  p[4 + l] = c;
  if (l == 0) {
    e.x += 1.f;
    ent[(size_t)s * 2] = e;
    ent[(size_t)s * 2 + 1] = e1;
  }
}
__global__ void init_fat128(float4* slots, const unsigned* perm, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) slots[i * 8] = make_float4(0.f, __uint_as_float(perm[i]), 0.f, 0.f);
}
__global__ void init_split(float4* ent, const unsigned* perm, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ent[i * 2] = make_float4(0.f, __uint_as_float(perm[i]), 0.f, 0.f);
}

int main() {
  const long CAP = 1L << 25;  // slots (the bench's table: 16.7 M keys at load 0.5)
  const int nfwd = 3900000, nbwd = 3480000;
  float4 *ent, *rows, *fat;
  unsigned *ifwd, *ibwd, *perm;
  float* out;
  CK(hipMalloc(&ent, CAP * 32));
  CK(hipMalloc(&rows, CAP * 128));
  CK(hipMalloc(&fat, CAP * 256));
  float4 *fat128, *aux;
  CK(hipMalloc(&fat128, CAP * 128));
  CK(hipMalloc(&aux, CAP * 64));
  CK(hipMemset(fat128, 0, CAP * 128));
  CK(hipMemset(aux, 0, CAP * 64));
  CK(hipMalloc(&ifwd, nfwd * 4));
  CK(hipMalloc(&ibwd, nbwd * 4));
  CK(hipMalloc(&perm, CAP * 4));
  CK(hipMalloc(&out, nfwd * 4));
  CK(hipMemset(rows, 0, CAP * 128));
  CK(hipMemset(fat, 0, CAP * 256));
  srand(1);
  {
    // V rows in insertion order: a random permutation of the slots
    std::vector<unsigned> p(CAP);
    for (long i = 0; i < CAP; ++i) p[i] = (unsigned)i;
    for (long i = CAP - 1; i > 0; --i) std::swap(p[i], p[((long)rand() << 16 ^ rand()) % (i + 1)]);
    CK(hipMemcpy(perm, p.data(), CAP * 4, hipMemcpyHostToDevice));
  }
  init_split<<<(CAP + 255) / 256, 256>>>(ent, perm, CAP);
  init_fat128<<<(CAP + 255) / 256, 256>>>(fat128, perm, CAP);
  std::vector<unsigned> h(nfwd);
  for (int i = 0; i < nfwd; ++i) h[i] = (unsigned)(((long)rand() << 16 ^ rand()) % CAP);
  CK(hipMemcpy(ifwd, h.data(), nfwd * 4, hipMemcpyHostToDevice));
  h.resize(nbwd);
  for (int i = 0; i < nbwd; ++i) h[i] = (unsigned)(((long)rand() << 16 ^ rand()) % CAP);
  std::sort(h.begin(), h.end());  // the backward walks keys in slot order
  h.erase(std::unique(h.begin(), h.end()), h.end());
  const int nb = (int)h.size();
  CK(hipMemcpy(ibwd, h.data(), nb * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, auto launch) {
    float best = 1e9;
    for (int rep = 0; rep < 8; ++rep) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%-34s %8.1f us\n", name, best * 1e3);
  };
  const int gf = (nfwd * 4 + 255) / 256, gb = (nb * 4 + 255) / 256;
  timeit("fwd split (entry + pool row)", [&] { fwd_split<<<gf, 256>>>(ent, rows, ifwd, nfwd, out); });
  timeit("fwd split, row = slot", [&] { fwd_split_par<<<gf, 256>>>(ent, rows, ifwd, nfwd, out); });
  timeit("fwd fat 192 B", [&] { fwd_fat<12><<<gf, 256>>>(fat, ifwd, nfwd, out); });
  timeit("fwd fat 160 B", [&] { fwd_fat<10><<<gf, 256>>>(fat, ifwd, nfwd, out); });
  timeit("fwd fat 256 B", [&] { fwd_fat<16><<<gf, 256>>>(fat, ifwd, nfwd, out); });
  timeit("fwd fat 128 B", [&] { fwd_fat<8><<<gf, 256>>>(fat128, ifwd, nfwd, out); });
  timeit("bwd fat 128 B, aux by slot", [&] { bwd_fat128<true><<<gb, 256>>>(fat128, aux, ibwd, nb); });
  timeit("bwd fat 128 B, aux by vrow", [&] { bwd_fat128<false><<<gb, 256>>>(fat128, aux, ibwd, nb); });
  timeit("fwd fat 128 B, V first", [&] { fwd_fatv<<<gf, 256>>>(fat128, ifwd, nfwd, out); });
  timeit("bwd fat 128 B V first, 16-B entry", [&] { bwd_fatv<false><<<gb, 256>>>(fat128, aux, ibwd, nb); });
  timeit("bwd fat 128 B V first, 32-B entry", [&] { bwd_fatv<true><<<gb, 256>>>(fat128, aux, ibwd, nb); });
  timeit("bwd split, 32-B entry", [&] { bwd_split32<<<gb, 256>>>(ent, rows, ibwd, nb); });
  timeit("bwd split (sorted slots)", [&] { bwd_split<<<gb, 256>>>(ent, rows, ibwd, nb); });
  timeit("bwd split, row = slot (sorted)", [&] { bwd_split_slot<<<gb, 256>>>(ent, rows, ibwd, nb); });
  timeit("bwd fat 160 B (sorted slots)", [&] { bwd_fat<10><<<gb, 256>>>(fat, ibwd, nb); });
  timeit("bwd fat 256 B (sorted slots)", [&] { bwd_fat<16><<<gb, 256>>>(fat, ibwd, nb); });
  return 0;
}
