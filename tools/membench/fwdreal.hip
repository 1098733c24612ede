// The library's own fat forward (fm.hip k_fm_fwd_walk, compiled into this harness) on the bench's
// table shape, alone: 2^25 fat slots of 128 B, every key of a 2^24 id space at its ordered-hash
// home slot (ids ~ U[0, 2^24): distinct home slots, no probe chains — the bench's table), B
// rows of 39 binary ids.  Against tools/membench/fwdbench's stripped-down walks it tells what
// the real kernel's extra work costs.  Build: tools/membench/fwdreal.sh (links libdifacto_amd
// for the host helpers fm.hip references; the kernels come from this translation unit).
#include "../../difacto_amd/csrc/fm.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("%s line %d\n", hipGetErrorString(e), __LINE__);     \
      exit(1);                                                    \
    }                                                             \
  } while (0)

using namespace dfx;

__global__ void fill_table(Entry* ent, const uint64_t* ids, int n, int logcap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = reverse_bytes(ids[i]);
  const uint64_t s = k >> (64 - logcap);
  Entry* e = ent + (s << 2);
  e->key = k;
  e->w = 0.25f;
  e->vrow = (int32_t)s;
  float* v = reinterpret_cast<float*>(e + 1);
  for (int q = 0; q < 16; ++q) v[q] = 0.01f * (float)((i + q) % 7);
}

template <auto K>
static int resident(int want) {
  int per = 0, cus = 0, dev = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, K, kFmNT, 0));
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return std::min(want, per * cus);
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

  const int B = argc > 1 ? atoi(argv[1]) : 100000, Kn = 39;
  const int nnz = B * Kn, logcap = 25;
  const long cap = 1L << logcap;
  srand(3);
  std::vector<uint64_t> hid(nnz), ho(B + 1);
  for (int i = 0; i < nnz; ++i) hid[i] = (uint64_t)(((long)rand() << 16 ^ rand()) % (1L << 24));
  for (int r = 0; r <= B; ++r) ho[r] = (uint64_t)r * Kn;
  std::vector<float> hl(B);
  for (int r = 0; r < B; ++r) hl[r] = (r % 4) ? -1.f : 1.f;
  Entry* ent;
  float *V, *label, *pred, *p, *XVp;
  uint64_t *ids, *offs;
  uint32_t *ak, *al;
  double* lp;
  CK(hipMalloc(&ent, cap * 128));
  CK(hipMemset(ent, 0xFF, cap * 128));  // key ~0: free slots
  CK(hipMalloc(&V, 64));
  CK(hipMalloc(&ids, (size_t)nnz * 8));
  CK(hipMalloc(&offs, (size_t)(B + 1) * 8));
  CK(hipMalloc(&label, (size_t)B * 4));
  CK(hipMalloc(&pred, (size_t)B * 4));
  CK(hipMalloc(&p, (size_t)B * 4));
  CK(hipMalloc(&XVp, (size_t)B * 128));
  CK(hipMalloc(&ak, (size_t)B * 4));
  CK(hipMalloc(&al, (size_t)B * 4));
  CK(hipMalloc(&lp, (size_t)(B / 4 + 64) * 8));
  CK(hipMemcpy(ids, hid.data(), (size_t)nnz * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(offs, ho.data(), (size_t)(B + 1) * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(label, hl.data(), (size_t)B * 4, hipMemcpyHostToDevice));
  fill_table<<<(nnz + 255) / 256, 256>>>(ent, ids, nnz, logcap);
  CK(hipDeviceSynchronize());
  FwdArgs a{};
  a.B = B; a.offs = offs; a.index = ids; a.max_index = ~0ull; a.val = nullptr;
  a.T.ent = ent; a.T.V = V; a.T.mask = cap - 1; a.T.logcap = logcap; a.T.d = 16; a.T.vcap = cap;
  a.T.ordered = 1; a.T.range_mul = 1; a.T.es = 2;
  a.l1_shrk = 0; a.d = 16; a.label = label; a.pred = pred; a.p_out = p; a.XVp = XVp; a.xs = 32;
  a.loss_part = lp; a.auc_key = ak; a.auc_lab = al;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int rep = 0; rep < 10; ++rep) {
      flush_caches<<<4096, 256>>>(fbuf, fbytes / 16);
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-36s best %7.1f us  median %7.1f us\n", name, t[0] * 1e3, t[t.size() / 2] * 1e3);
    fflush(stdout);
  };
  const int nb = (B + 63) / 64;
  {
    const int g = resident<k_fm_fwd_walk<4, false>>(nb);
    timeit("k_fm_fwd_walk", [&] {
      hipLaunchKernelGGL((k_fm_fwd_walk<4, false>), dim3(g), dim3(kFmNT), 0, 0, a);
    });
    float h0[4];
    CK(hipMemcpy(h0, XVp, 16, hipMemcpyDeviceToHost));
    printf("walk XVp[0..3] %g %g %g %g\n", h0[0], h0[1], h0[2], h0[3]);
  }
  {
    const int g = resident<k_fm_fwd_walk<4, false, 2>>(nb);
    timeit("k_fm_fwd_walk (MINB 2)", [&] {
      hipLaunchKernelGGL((k_fm_fwd_walk<4, false, 2>), dim3(g), dim3(kFmNT), 0, 0, a);
    });
  }
  float h[4];
  CK(hipMemcpy(h, pred, 16, hipMemcpyDeviceToHost));
  printf("pred[0..3] %g %g %g %g\n", h[0], h[1], h[2], h[3]);
  return 0;
}
