// Does a key's state in ONE 256-byte-aligned span read-modify-write faster than in two unrelated
// 128-byte chunks?  ("next" 3; DESIGN.md (d): the backward is priced at 2 random chunk
// read-modify-writes per key because a key's 144 B of hot state — entry 16 B, V 64 B, Vaux 64 B
// at d = 16 — cannot fit one 128-B chunk.)
//
// The backward's pattern at the bench config: 3.48 M distinct table slots out of 2^25, walked in
// slot order (the ordered hash), 4 lanes per key, each lane a float4 of V and of Vaux, lane 0 the
// entry's hot 16 B.  Layouts:
//   cur      128-B slot [entry 32 | V 64 | pad 32] + Vaux in a pool of 64-B rows, row = slot (today)
//   s256     256-B slot [entry 32 | V 64 | pad 32][Vaux 64 | pad 64]: two 128-B halves of one span
//   s256p    256-B slot [entry 32 | V 64 | Vaux 64 | pad 96]: the 160 B packed from the start
//   s128v    128-B slot, entry + V only (no Vaux): the 1-chunk-per-key lower bound
//   pairD    two 128-B lines D bytes apart (D = 256 ... 8192) in a slot of 2D: where the second
//            chunk of a key stops being cheap (the memory's interleave granularity)
// and the forward's read of a slot's first 128 B, 3.9 M random slots, 4-GiB (128-B slots) vs
// 8-GiB (256-B slots) tables.
// Build: hipcc --offload-arch=gfx950 -O3 spanbench.hip -o spanbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s line %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                              \
    }                                                       \
  } while (0)

// entry (hot 16 B) at float4 0 of line A, V at float4 2..5 of line A (4 lanes), Vaux at float4
// AUX + l of a second address: the same slot (in-span) or a pool row
template <int SF, int AUX>
__global__ void rmw_slot(float4* slots, const unsigned* idx, int n) {
  const int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  float4* p = slots + (size_t)idx[g] * SF;
  float4 e = p[0];
  float4 v = p[2 + l];
  float4 c = AUX > 0 ? p[AUX + l] : make_float4(0.f, 0.f, 0.f, 0.f);
  v.x += e.x;
  c.y += 1.f;
  p[2 + l] = v;
  if (AUX > 0) p[AUX + l] = c;
  if (l == 0) {
    e.x += 1.f;
    p[0] = e;
  }
}
// today's layout: 128-B slot + Vaux pool row = slot
__global__ void rmw_cur(float4* slots, float4* aux, const unsigned* idx, int n) {
  const int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  const size_t s = idx[g];
  float4* p = slots + s * 8;
  float4* q = aux + s * 4;
  float4 e = p[0];
  float4 v = p[2 + l];
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
// two 128-B lines (entry + V, then Vaux) DF float4s apart, in slots of SF float4s (DF = 0: the
// first line only)
__global__ void rmw_pair(float4* slots, const unsigned* idx, int n, int SF, int DF) {
  const int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  float4* p = slots + (size_t)idx[g] * SF;
  float4 e = p[0];
  float4 v = p[2 + l];
  float4 c = DF ? p[DF + l] : make_float4(0.f, 0.f, 0.f, 0.f);
  v.x += e.x;
  c.y += 1.f;
  p[2 + l] = v;
  if (DF) p[DF + l] = c;
  if (l == 0) {
    e.x += 1.f;
    p[0] = e;
  }
}
// the forward: a slot's first 128 B (entry halves + V), 4 lanes
__global__ void rd_slot(const float4* slots, const unsigned* idx, int n, int SF, float* out) {
  const int g = (blockIdx.x * blockDim.x + threadIdx.x) / 4, l = threadIdx.x & 3;
  if (g >= n) return;
  const float4* p = slots + (size_t)idx[g] * SF;
  const float2 wv = reinterpret_cast<const float2*>(p)[(l & 1) ? 3 : 0];
  const float4 v = p[2 + l];
  const float acc = wv.x + wv.y + v.x + v.y + v.z + v.w;
  if (acc == 12345.f) out[g] = acc;
}

// evicts the 256-MiB Infinity Cache (and the L2s) between timed reps: a 1-GiB streaming read
// (no dirty lines left to write back inside the timed kernel), so every rep starts cold, as a
// bench step does on fresh keys
__global__ void flush_caches(float4* buf, size_t n) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc += buf[i].x;
  if (acc == 1234.5f) buf[0].y = acc;
}

int main(int argc, char** argv) {
  float4* fbuf = nullptr;
  const size_t fbytes = 1ull << 30;
  CK(hipMalloc(&fbuf, fbytes));
  CK(hipMemset(fbuf, 0, fbytes));

  const long CAP = 1L << 25;  // slots: the bench's table (16.7 M keys at load 0.5)
  const int nfwd = 3900000, nbwd = 3480000;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  srand(1);
  std::vector<unsigned> h(nbwd);
  for (int i = 0; i < nbwd; ++i) h[i] = (unsigned)(((long)rand() << 16 ^ rand()) % CAP);
  std::sort(h.begin(), h.end());
  h.erase(std::unique(h.begin(), h.end()), h.end());
  const int nb = (int)h.size();
  std::vector<unsigned> hf(nfwd);
  for (int i = 0; i < nfwd; ++i) hf[i] = (unsigned)(((long)rand() << 16 ^ rand()) % CAP);
  unsigned *ibwd, *ifwd;
  float* out;
  CK(hipMalloc(&ibwd, (size_t)nb * 4));
  CK(hipMalloc(&ifwd, (size_t)nfwd * 4));
  CK(hipMalloc(&out, (size_t)nfwd * 4));
  CK(hipMemcpy(ibwd, h.data(), (size_t)nb * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(ifwd, hf.data(), (size_t)nfwd * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, double keys, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int rep = 0; rep < reps; ++rep) {
      flush_caches<<<4096, 256>>>(fbuf, fbytes / 16);
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-40s best %7.1f us  median %7.1f us  %6.2f G keys/s\n", name, t[0] * 1e3,
           t[t.size() / 2] * 1e3, keys / (t[0] * 1e-3) / 1e9);
    fflush(stdout);
  };
  const int gb = (nb * 4 + 255) / 256, gf = (nfwd * 4 + 255) / 256;
  float4 *s128, *aux;
  CK(hipMalloc(&s128, CAP * 128));
  CK(hipMalloc(&aux, CAP * 64));
  CK(hipMemset(s128, 0, CAP * 128));
  CK(hipMemset(aux, 0, CAP * 64));
  timeit("fwd read 128-B slot (4 GiB table)", nfwd, [&] { rd_slot<<<gf, 256>>>(s128, ifwd, nfwd, 8, out); });
  timeit("bwd cur: 128-B slot + 64-B Vaux row", nb, [&] { rmw_cur<<<gb, 256>>>(s128, aux, ibwd, nb); });
  timeit("bwd s128v: 128-B slot, no Vaux", nb, [&] { rmw_slot<8, 0><<<gb, 256>>>(s128, ibwd, nb); });
  CK(hipFree(aux));
  CK(hipFree(s128));
  float4* s256;
  CK(hipMalloc(&s256, CAP * 256));
  CK(hipMemset(s256, 0, CAP * 256));
  timeit("fwd read 256-B slot (8 GiB table)", nfwd, [&] { rd_slot<<<gf, 256>>>(s256, ifwd, nfwd, 16, out); });
  timeit("bwd s256: [entry|V|pad][Vaux|pad]", nb, [&] { rmw_slot<16, 8><<<gb, 256>>>(s256, ibwd, nb); });
  timeit("bwd s256p: [entry|V|Vaux|pad]", nb, [&] { rmw_slot<16, 6><<<gb, 256>>>(s256, ibwd, nb); });
  CK(hipFree(s256));
  // where the second chunk stops being cheap: pairs D bytes apart, slots of 2D (CAP / 8 slots of
  // the same index set scaled down so the tables stay <= 32 GiB)
  for (int D = 256; D <= 8192; D *= 2) {
    const long S = 2L * D;
    const long cap = std::min<long>(CAP, (32L << 30) / S);
    std::vector<unsigned> hs(nb);
    for (int i = 0; i < nb; ++i) hs[i] = (unsigned)((long)h[i] * cap / CAP);
    hs.erase(std::unique(hs.begin(), hs.end()), hs.end());
    const int ns = (int)hs.size();
    CK(hipMemcpy(ibwd, hs.data(), (size_t)ns * 4, hipMemcpyHostToDevice));
    float4* t;
    CK(hipMalloc(&t, cap * S));
    CK(hipMemset(t, 0, cap * S));
    char name[96];
    snprintf(name, sizeof name, "bwd pair D=%d (slots %ld B, %d keys)", D, S, ns);
    const int g2 = (ns * 4 + 255) / 256;
    timeit(name, ns, [&] { rmw_pair<<<g2, 256>>>(t, ibwd, ns, (int)(S / 16), D / 16); });
    snprintf(name, sizeof name, "bwd one line (slots %ld B)", S);
    timeit(name, ns, [&] { rmw_pair<<<g2, 256>>>(t, ibwd, ns, (int)(S / 16), 0); });
    CK(hipFree(t));
  }
  return 0;
}
