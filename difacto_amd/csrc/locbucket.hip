// Localizer::Compact (src/data/localizer.cc:11-107) as a bucket sort, for the callers that need
// no per-nnz col: the fused step and the split owner, whose forward finds each key in the model
// table itself and whose backward walks each key's occurrences in sorted order.  Five launches
// where the radix Localizer (localize.hip + sort.hip) takes ~17, and about half its traffic:
//
//   k_lb_init     the batch's key statistics and the bucket tickets reset
//   k_lb_hist     per tile of rows: every nnz's key (ReverseBytes(id % max_index),
//                 localizer.cc:24) and its bucket into the tile's histogram (LDS); OR / AND /
//                 min / max of the keys.  A key's bucket is a monotone map of the key,
//                 clamp((key - base) >> s), fitted to the key range of the previous batch on this
//                 lane: buckets are ranges of keys in key order whatever the batch holds, and a
//                 batch like the previous one spreads evenly over them
//   k_lb_colscan  per bucket: the exclusive prefix of its counts over the tiles, and its total
//   k_lb_scatter  per tile: the buckets' starts (a scan of the totals), then every nnz's item
//                 into its bucket's range through an LDS cursor per bucket.  An item packs the
//                 key's varying bits above the row (binary data) or the position (valued data,
//                 {value, row} beside it) in one u64 when they fit; else the key and the row /
//                 position travel apart
//   k_lb_bucket   one block per bucket, in bucket order (tickets): the bucket sorted in LDS —
//                 bitonic, on the whole item: (key, row) resp. (key, position) is a total order
//                 and equal items are the same occurrence data, so the scatter's order inside a
//                 bucket never shows — then its heads (CountUniqIndex's run-length pass), the
//                 heads of the buckets before it by decoupled look-back (RemapIndex's ranks),
//                 and the outputs: per rank its key and segment start, per occurrence in sorted
//                 order its row (and value).  A bucket beyond the LDS capacity (skewed keys, or a
//                 key range that moved) is sorted by its block through global memory in stable
//                 8-bit LSD passes: slower, the same result; the workspace's hint then sends
//                 the next batches to the radix Localizer and retries every kLbRetry batches.
//
// The occurrence order is the radix Localizer's stable (key, position) order: positions ascend
// with rows, and a binary row's repeats of one key are identical items.  So the outputs are
// bit-identical to localize.hip's (test_gpu_r4.py compares the two).
#include <algorithm>

#include "lookback.h"

namespace dfx {

constexpr int kLbNT = 256;
constexpr int kLbWaves = kLbNT / kWave;
constexpr int kLbCap = 2048;         // items of a bucket sorted in LDS
constexpr int kLbMaxBits = 13;       // at most 8192 buckets
constexpr int64_t kLbMaxRows = 2048; // rows per hist / scatter tile (their offsets sit in LDS)
constexpr int kLbIT = 8;             // items per thread of a chunk (heads, the global-memory passes)
constexpr unsigned kLbOverRadix = 2; // more buckets than this over kLbCap: radix Localizer next
constexpr unsigned kLbRetry = 64;    // ... and the bucket Localizer tried again after this many

struct LbArgs {
  int64_t B, nnz;
  const uint64_t* offset;
  const uint64_t* index;
  uint64_t max_index;
  int keys_ready;        // index holds the final keys (the split owner's received keys)
  const float* value;    // valued data: {value bits, row << 32} rides beside each item
  int64_t rt, ntiles;    // rows per tile, tiles
  int wbits;             // log2 of the bucket count
  int nt;                // streaming policy for the ids and the items (kwarg nt & 1)
  uint32_t* tilecnt;     // [ntiles][nbk]: counts, then exclusive prefixes over the tiles
  uint32_t* totals;      // [nbk]
  uint32_t* bstart;      // [nbk + 1]
  uint64_t* kbuf;        // items
  uint32_t* qbuf;        // rows / positions of unpacked items
  uint64_t* sbuf;        // side payloads (valued)
  uint64_t* kscr;        // scratch of the global-memory passes
  uint32_t* qscr;
  uint64_t* sscr;
  DevState* ds;
  unsigned long long* hstat;  // per bucket its tagged look-back word
  uint64_t* uniq;
  uint32_t* segstart;
  uint32_t* occ_row;
  float* occ_x;
  unsigned int* hint;    // pinned: Workspace::lb_hint
};

__device__ inline uint64_t lb_key(uint64_t id, uint64_t max_index, int keys_ready) {
  if (keys_ready) return id;
  const uint64_t m = max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % max_index;
  return reverse_bytes(m);
}

__device__ inline int lb_bitlen(uint64_t x) { return x ? 64 - __clzll((long long)x) : 0; }

// the bucket map: bucket(k) = clamp((k - base) >> s, 0, nbk - 1), monotone in k
struct LbMap {
  uint64_t base;
  int s;
  uint32_t nbk;
};
__device__ inline LbMap lb_map(const DevState* ds, int wbits) {
  LbMap m;
  m.nbk = 1u << wbits;
  if (ds->pk_valid) {
    m.base = ds->pk_min;
    const int bl = lb_bitlen(ds->pk_max - ds->pk_min);
    m.s = bl > wbits ? bl - wbits : 0;
  } else {  // no batch seen yet: the top bits of the key
    m.base = 0;
    m.s = 64 - wbits;
  }
  return m;
}
__device__ inline uint32_t lb_bucket(uint64_t k, const LbMap& m) {
  if (k <= m.base) return 0u;
  const uint64_t x = (k - m.base) >> m.s;
  return x < m.nbk ? (uint32_t)x : m.nbk - 1u;
}

// the item form of this batch: ((key - kmin) >> lo) << rb | q when the key's varying bits and q's
// rb bits fit 63 bits (the top bit stays clear, so no item equals the sort's padding ~0);
// else the raw key (never ~0: common.h kEmptyKey) with q apart
struct LbPack {
  uint64_t kmin;
  int lo, rb;
  bool packed;
};
__device__ inline LbPack lb_pack(const DevState* ds, uint64_t qmax) {
  LbPack p;
  p.kmin = ds->kmin;
  const uint64_t diff = ds->or_mask ^ ds->and_mask;
  p.lo = diff ? __ffsll((long long)diff) - 1 : 0;
  p.rb = lb_bitlen(qmax);
  p.packed = lb_bitlen((ds->kmax - ds->kmin) >> p.lo) + p.rb <= 63;
  return p;
}
__device__ inline uint64_t lb_keybits(const LbPack& p, uint64_t it) {
  return p.packed ? it >> p.rb : it;
}

__global__ void k_lb_init(DevState* ds) {
  ds->or_mask = 0;
  ds->and_mask = ~0ull;
  ds->kmin = ~0ull;
  ds->kmax = 0;
  ds->n_init = 0;  // long segments of the batch (chunk_plan's gate)
  unsigned* meta = ds->sortmeta;
  meta[kSortMetaEpoch] = ++ds->sort_epoch;  // tags this Localizer's look-back words
  meta[kSortMetaHwTile] = 0;                // bucket tickets
  meta[kSortMetaCpTile] = 0;                // the chunk plan's tile tickets
}

__device__ inline unsigned long long lb_wave_or(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off, kWave);
  return v;
}
__device__ inline unsigned long long lb_wave_and(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) v &= __shfl_xor(v, off, kWave);
  return v;
}
__device__ inline unsigned long long lb_wave_min(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off, kWave);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline unsigned long long lb_wave_max(unsigned long long v) {
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

constexpr int kLbUnr = 4;  // ids in flight per thread

__global__ __launch_bounds__(kLbNT) void k_lb_hist(LbArgs a) {
  extern __shared__ uint32_t lb_dyn[];
  uint32_t* hist = lb_dyn;
  __shared__ unsigned long long red[4][kLbWaves];
  const LbMap m = lb_map(a.ds, a.wbits);
  const int t = threadIdx.x;
  for (uint32_t d = t; d < m.nbk; d += kLbNT) hist[d] = 0;
  const int64_t r0 = (int64_t)blockIdx.x * a.rt;
  const int64_t r1 = r0 + a.rt < a.B ? r0 + a.rt : a.B;
  const uint64_t j0 = a.offset[r0], j1 = a.offset[r1];
  __syncthreads();
  unsigned long long vor = 0, vand = ~0ull, vmin = ~0ull, vmax = 0;
  for (uint64_t jb = j0; jb < j1; jb += (uint64_t)kLbUnr * kLbNT) {
    uint64_t id[kLbUnr];
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t j = jb + (uint64_t)u * kLbNT + t;
      id[u] = j < j1 ? ldnt(a.index + j, a.nt != 0) : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      if (jb + (uint64_t)u * kLbNT + t < j1) {
        const uint64_t k = lb_key(id[u], a.max_index, a.keys_ready);
        vor |= k;
        vand &= k;
        vmin = k < vmin ? k : vmin;
        vmax = k > vmax ? k : vmax;
        atomicAdd(&hist[lb_bucket(k, m)], 1u);
      }
    }
  }
  vor = lb_wave_or(vor);
  vand = lb_wave_and(vand);
  vmin = lb_wave_min(vmin);
  vmax = lb_wave_max(vmax);
  const int w = t / kWave;
  if (lane_id() == 0) {
    red[0][w] = vor;
    red[1][w] = vand;
    red[2][w] = vmin;
    red[3][w] = vmax;
  }
  __syncthreads();
  uint32_t* dst = a.tilecnt + (size_t)blockIdx.x * m.nbk;
  for (uint32_t d = t; d < m.nbk; d += kLbNT) dst[d] = hist[d];
  if (t == 0 && j1 > j0) {
    for (int i = 1; i < kLbWaves; ++i) {
      vor |= red[0][i];
      vand &= red[1][i];
      vmin = red[2][i] < vmin ? red[2][i] : vmin;
      vmax = red[3][i] > vmax ? red[3][i] : vmax;
    }
    atomicOr(&a.ds->or_mask, vor);
    atomicAnd(&a.ds->and_mask, vand);
    atomicMin(&a.ds->kmin, vmin);
    atomicMax(&a.ds->kmax, vmax);
  }
}

// 64 buckets per block (one per lane), the tiles split over 16 waves
constexpr int kLbScanWaves = 16;
__global__ __launch_bounds__(kLbScanWaves * kWave) void k_lb_colscan(LbArgs a) {
  __shared__ uint32_t part[kLbScanWaves][kWave];
  const int l = lane_id(), w = threadIdx.x / kWave;
  const uint32_t nbk = 1u << a.wbits;
  const uint32_t b = blockIdx.x * kWave + l;
  const bool ok = b < nbk;
  const int64_t T = a.ntiles, tt = (T + kLbScanWaves - 1) / kLbScanWaves;
  const int64_t t0 = (int64_t)w * tt < T ? (int64_t)w * tt : T;
  const int64_t t1 = t0 + tt < T ? t0 + tt : T;
  uint32_t s = 0;
  if (ok)
    for (int64_t i = t0; i < t1; ++i) s += a.tilecnt[(size_t)i * nbk + b];
  part[w][l] = s;
  __syncthreads();
  if (w == 0) {
    uint32_t run = 0;
    for (int i = 0; i < kLbScanWaves; ++i) {
      const uint32_t x = part[i][l];
      part[i][l] = run;
      run += x;
    }
    if (ok) a.totals[b] = run;
  }
  __syncthreads();
  if (ok) {
    uint32_t run = part[w][l];
    for (int64_t i = t0; i < t1; ++i) {
      uint32_t* p = a.tilecnt + (size_t)i * nbk + b;
      const uint32_t c = *p;
      *p = run;
      run += c;
    }
  }
}

template <bool S>
__global__ __launch_bounds__(kLbNT) void k_lb_scatter(LbArgs a) {
  extern __shared__ uint64_t lb_dyn64[];
  __shared__ uint32_t lds[kLbWaves + 1];
  const LbMap m = lb_map(a.ds, a.wbits);
  uint32_t* cur = reinterpret_cast<uint32_t*>(lb_dyn64);  // per bucket: this tile's next slot
  uint64_t* offs = lb_dyn64 + (m.nbk + 1u) / 2;
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * a.rt;
  const int nr = (int)(a.B - r0 < a.rt ? a.B - r0 : a.rt);
  // the buckets' starts: thread t holds buckets [t * per, (t + 1) * per)
  const uint32_t per = (m.nbk + kLbNT - 1) / kLbNT;
  uint32_t mine = 0, over = 0;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t d = t * per + i;
    if (d < m.nbk) {
      const uint32_t c = a.totals[d];
      mine += c;
      over += c > (uint32_t)kLbCap ? 1u : 0u;
    }
  }
  uint32_t total;
  uint32_t ex = block_excl_scan<kLbNT>(mine, lds, &total);
  const uint32_t* pre = a.tilecnt + (size_t)blockIdx.x * m.nbk;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t d = t * per + i;
    if (d < m.nbk) {
      cur[d] = ex + pre[d];
      if (blockIdx.x == 0) a.bstart[d] = ex;
      ex += a.totals[d];
    }
  }
  const uint64_t qmax = S ? (uint64_t)(a.nnz - 1) : (uint64_t)(a.B - 1);
  const LbPack p = lb_pack(a.ds, qmax);
  if (blockIdx.x == 0) {
    uint32_t nover;
    (void)block_excl_scan<kLbNT>(over, lds, &nover);
    if (t == 0) {
      a.bstart[m.nbk] = total;
      // the next batches' choice (pinned host words, vector stores)
      a.hint[0] = nover;
      a.hint[2] = p.packed ? 1u : 2u;
    }
  }
  for (int i = t; i <= nr; i += kLbNT) offs[i] = a.offset[r0 + i];
  __syncthreads();
  const uint64_t j0 = offs[0], j1 = offs[nr];
  const uint64_t qmask = p.rb ? (~0ull >> (64 - p.rb)) : 0ull;
  for (uint64_t jb = j0; jb < j1; jb += (uint64_t)kLbUnr * kLbNT) {
    uint64_t id[kLbUnr];
    float x[kLbUnr];
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t j = jb + (uint64_t)u * kLbNT + t;
      id[u] = j < j1 ? ldnt(a.index + j, a.nt != 0) : 0ull;
      if (S) x[u] = j < j1 ? ldnt(a.value + j, a.nt != 0) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t j = jb + (uint64_t)u * kLbNT + t;
      if (j >= j1) continue;
      const uint64_t k = lb_key(id[u], a.max_index, a.keys_ready);
      // row = upper_bound(j) - 1 over the tile's offsets (empty rows skipped)
      int lo = 0, hi = nr;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (offs[mid] <= j) lo = mid; else hi = mid;
      }
      const uint32_t row = (uint32_t)(r0 + lo);
      const uint64_t q = S ? j : (uint64_t)row;
      const uint32_t pos = atomicAdd(&cur[lb_bucket(k, m)], 1u);
      stnt(a.kbuf + pos, p.packed ? ((((k - p.kmin) >> p.lo) << p.rb) | (q & qmask)) : k,
           a.nt != 0);
      if (!p.packed) a.qbuf[pos] = (uint32_t)q;
      if (S) a.sbuf[pos] = (uint64_t)__float_as_uint(x[u]) | ((uint64_t)row << 32);
    }
  }
}

// ---- the per-bucket sort --------------------------------------------------------------------
// One stable 8-bit LSD pass of a bucket's n items through global memory (X -> Y) by its block:
// per chunk of kLbNT * kLbIT items the waves rank their items with ballots (wave w owns a
// contiguous run, items in order), and the digit's running base places them
template <bool S>
__device__ void lb_global_pass(const uint64_t* Xk, const uint32_t* Xq, const uint64_t* Xs,
                               uint64_t* Yk, uint32_t* Yq, uint64_t* Ys, int64_t n, bool on_q,
                               int shift, uint32_t (*wcnt)[256], uint32_t* base, uint32_t* lds) {
  const int t = threadIdx.x, w = t / kWave, l = lane_id();
  base[t] = 0;
  __syncthreads();
  for (int64_t i = t; i < n; i += kLbNT) {
    const uint32_t d = on_q ? (Xq[i] >> shift) & 255u : (uint32_t)(Xk[i] >> shift) & 255u;
    atomicAdd(&base[d], 1u);
  }
  __syncthreads();
  {
    const uint32_t c = base[t];
    const uint32_t ex = block_excl_scan<kLbNT>(c, lds, nullptr);
    base[t] = ex;
  }
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += (int64_t)kLbNT * kLbIT) {
    for (int i = t; i < kLbWaves * 256; i += kLbNT) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t dr[kLbIT];
    const int64_t wb = c0 + (int64_t)w * kWave * kLbIT;
#pragma unroll
    for (int j = 0; j < kLbIT; ++j) {
      const int64_t idx = wb + j * kWave + l;
      const bool valid = idx < n;
      const uint32_t d = !valid ? 0u
                         : on_q ? (Xq[idx] >> shift) & 255u
                                : (uint32_t)(Xk[idx] >> shift) & 255u;
      uint64_t peers = __ballot(valid);
#pragma unroll
      for (int bt = 0; bt < 8; ++bt) {
        const bool bit = (d >> bt) & 1u;
        const uint64_t mb = __ballot(valid && bit);
        peers &= bit ? mb : ~mb;
      }
      if (!valid) peers = 0;
      const uint32_t rk = (uint32_t)__popcll(peers & lanemask_lt());
      const uint32_t old = valid ? wcnt[w][d] : 0u;
      __builtin_amdgcn_wave_barrier();
      if (valid && rk == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
      dr[j] = valid ? (d | ((old + rk) << 8)) : 0xFFFFFFFFu;
    }
    __syncthreads();
    {  // the waves' offsets inside the chunk, on the digit's running base
      uint32_t run = base[t];
      for (int i = 0; i < kLbWaves; ++i) {
        const uint32_t x = wcnt[i][t];
        wcnt[i][t] = run;
        run += x;
      }
      base[t] = run;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kLbIT; ++j) {
      if (dr[j] == 0xFFFFFFFFu) continue;
      const int64_t idx = wb + j * kWave + l;
      const uint32_t dst = wcnt[w][dr[j] & 255u] + (dr[j] >> 8);
      Yk[dst] = Xk[idx];
      if (Xq) Yq[dst] = Xq[idx];
      if (S) Ys[dst] = Xs[idx];
    }
    __syncthreads();
  }
  __threadfence();  // this pass's stores, read by the whole block in the next (L1 invalidated)
  __syncthreads();
}

template <bool Q, bool S>
__global__ __launch_bounds__(kLbNT) void k_lb_bucket(LbArgs a) {
  __shared__ uint64_t sk[kLbCap];
  __shared__ uint32_t sq[Q ? kLbCap : 1];
  __shared__ uint64_t ss[S ? kLbCap : 1];
  __shared__ uint32_t wcnt[kLbWaves][256];
  __shared__ uint32_t base[256];
  __shared__ uint32_t lds[kLbWaves + 1];
  __shared__ uint32_t s_b, s_pre;
  __shared__ unsigned long long s_red[4][kLbWaves];
  static_assert(kLbNT == 256, "one thread per 8-bit digit in the global-memory passes");
  DevState* ds = a.ds;
  unsigned* meta = ds->sortmeta;
  const int t = threadIdx.x;
  if (t == 0) s_b = atomicAdd(&meta[kSortMetaHwTile], 1u);
  __syncthreads();
  const uint32_t b = s_b;
  const uint32_t nbk = 1u << a.wbits;
  if (b >= nbk) return;  // every later ticket exits too: no waiter is left behind
  const int64_t start = a.bstart[b];
  const int64_t n = (int64_t)a.bstart[b + 1] - start;
  const uint64_t qmax = S ? (uint64_t)(a.nnz - 1) : (uint64_t)(a.B - 1);
  const LbPack p = lb_pack(ds, qmax);
  const bool hasq = !p.packed;
  const bool fast = n <= kLbCap && (p.packed || Q);
  // where the sorted bucket is read from by the heads / outputs below
  const uint64_t* gk = a.kbuf + start;
  const uint32_t* gq = a.qbuf + start;
  const uint64_t* gs = a.sbuf + start;
  if (fast) {
    int n2 = 2;
    while (n2 < n) n2 <<= 1;
    for (int i = t; i < n2; i += kLbNT) {
      if (i < n) {
        sk[i] = ldnt(gk + i, a.nt != 0);
        if (Q && hasq) sq[i] = gq[i];
        if (S) ss[i] = gs[i];
      } else {  // padding sorts last: no real item is ~0 (lb_pack)
        sk[i] = ~0ull;
        if (Q && hasq) sq[i] = ~0u;
      }
    }
    __syncthreads();
    for (int size = 2; size <= n2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = t; i < (n2 >> 1); i += kLbNT) {
          const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
          const int hi = lo + stride;
          const int x = (lo & size) == 0 ? lo : hi;  // x must not exceed y
          const int y = x == lo ? hi : lo;
          const uint64_t kx = sk[x], ky = sk[y];
          bool sw = kx > ky;
          if (Q && hasq && kx == ky) sw = sq[x] > sq[y];
          if (sw) {
            sk[x] = ky;
            sk[y] = kx;
            if (Q && hasq) {
              const uint32_t qx = sq[x];
              sq[x] = sq[y];
              sq[y] = qx;
            }
            if (S) {
              const uint64_t sx = ss[x];
              ss[x] = ss[y];
              ss[y] = sx;
            }
          }
        }
        __syncthreads();
      }
    }
  } else if (n > 1) {
    // through global memory: stable 8-bit LSD over the digits that vary inside the bucket — q's
    // first (the less significant part of an unpacked item), then the key's
    unsigned long long kor = 0, kand = ~0ull, qor = 0, qand = ~0ull;
    for (int64_t i = t; i < n; i += kLbNT) {
      const uint64_t x = gk[i];
      kor |= x;
      kand &= x;
      if (hasq) {
        qor |= gq[i];
        qand &= gq[i];
      }
    }
    kor = lb_wave_or(kor);
    kand = lb_wave_and(kand);
    qor = lb_wave_or(qor);
    qand = lb_wave_and(qand);
    if (lane_id() == 0) {
      s_red[0][t / kWave] = kor;
      s_red[1][t / kWave] = kand;
      s_red[2][t / kWave] = qor;
      s_red[3][t / kWave] = qand;
    }
    __syncthreads();
    for (int i = 0; i < kLbWaves; ++i) {
      kor |= s_red[0][i];
      kand &= s_red[1][i];
      qor |= s_red[2][i];
      qand &= s_red[3][i];
    }
    __syncthreads();
    uint64_t* Xk = a.kbuf + start;
    uint32_t* Xq = hasq ? a.qbuf + start : nullptr;
    uint64_t* Xs = S ? a.sbuf + start : nullptr;
    uint64_t* Yk = a.kscr + start;
    uint32_t* Yq = hasq ? a.qscr + start : nullptr;
    uint64_t* Ys = S ? a.sscr + start : nullptr;
    for (int pass = 0; pass < 12; ++pass) {
      const bool on_q = pass < 4;
      const int shift = 8 * (on_q ? pass : pass - 4);
      const unsigned long long vary = on_q ? (hasq ? (qor ^ qand) : 0ull) : (kor ^ kand);
      if (((vary >> shift) & 255ull) == 0) continue;
      lb_global_pass<S>(Xk, Xq, Xs, Yk, Yq, Ys, n, on_q, shift, wcnt, base, lds);
      uint64_t* tk = Xk; Xk = Yk; Yk = tk;
      uint32_t* tq = Xq; Xq = Yq; Yq = tq;
      uint64_t* ts = Xs; Xs = Ys; Ys = ts;
    }
    gk = Xk;
    gq = Xq;
    gs = Xs;
  }
  auto item = [&](int64_t i) -> uint64_t { return fast ? sk[i] : gk[i]; };
  // ---- heads: an item whose key differs from the one before it (the bucket's first always);
  // a segment longer than kChunkOcc raises the chunk plan's gate
  uint32_t mine = 0;
  bool longseg = false;
  for (int64_t i = t; i < n; i += kLbNT) {
    const uint64_t kb = lb_keybits(p, item(i));
    mine += (i == 0 || kb != lb_keybits(p, item(i - 1))) ? 1u : 0u;
    if (i >= kChunkOcc && kb == lb_keybits(p, item(i - kChunkOcc))) longseg = true;
  }
  if (__syncthreads_or(longseg) && t == 0 &&
      __hip_atomic_load(&ds->n_init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    atomicOr(&ds->n_init, 1u);
  uint32_t tot;
  (void)block_excl_scan<kLbNT>(mine, lds, &tot);
  uint32_t rank0 = tile_lookback(a.hstat, (int64_t)b, hw_tag(meta), tot, &ds->err, &s_pre);
  // ---- outputs, per thread kLbIT consecutive items of a chunk
  const uint64_t qmask = p.rb ? (~0ull >> (64 - p.rb)) : 0ull;
  for (int64_t c0 = 0; c0 < n; c0 += (int64_t)kLbNT * kLbIT) {
    const int64_t ib = c0 + (int64_t)t * kLbIT;
    uint32_t h[kLbIT], s = 0;
#pragma unroll
    for (int j = 0; j < kLbIT; ++j) {
      const int64_t i = ib + j;
      h[j] = (i < n && (i == 0 || lb_keybits(p, item(i)) != lb_keybits(p, item(i - 1)))) ? 1u
                                                                                        : 0u;
      s += h[j];
    }
    uint32_t ctot;
    uint32_t incl = block_excl_scan<kLbNT>(s, lds, &ctot) + rank0;
#pragma unroll
    for (int j = 0; j < kLbIT; ++j) {
      const int64_t i = ib + j;
      if (i >= n) break;
      incl += h[j];
      const uint64_t it = item(i);
      if (h[j]) {
        const uint64_t key = p.packed ? (((it >> p.rb) << p.lo) + p.kmin) : it;
        if (a.uniq) a.uniq[incl - 1] = key;
        if (a.segstart) a.segstart[incl - 1] = (uint32_t)(start + i);
      }
      uint32_t row;
      if (S) {
        const uint64_t sv = fast ? ss[i] : gs[i];
        row = (uint32_t)(sv >> 32);
        if (a.occ_x) a.occ_x[start + i] = __uint_as_float((uint32_t)sv);
      } else {
        row = p.packed ? (uint32_t)(it & qmask) : (fast ? sq[i] : gq[i]);
      }
      a.occ_row[start + i] = row;
    }
    rank0 += ctot;
  }
  if (b == nbk - 1u && t == 0) {  // the last bucket closes the segments
    ds->u_count = rank0;
    if (a.segstart) a.segstart[rank0] = (uint32_t)a.nnz;
    // the next batch on this lane fits its bucket map to this batch's key range
    ds->pk_min = ds->kmin;
    ds->pk_max = ds->kmax;
    ds->pk_valid = 1u;
  }
}

int localize_bucket(Context* c, const Lane& L, int64_t B, int64_t nnz, const uint64_t* offset,
                    const uint64_t* index, uint64_t max_index, const LocOut& o, bool* used) {
  *used = false;
  Workspace& ws = *L.ws;
  if (!ws.lb_hint) {
    DFX_HIP(hipHostMalloc(reinterpret_cast<void**>(&ws.lb_hint), 4 * sizeof(unsigned int),
                          hipHostMallocDefault));
    for (int i = 0; i < 4; ++i) ws.lb_hint[i] = 0;
  }
  volatile unsigned int* hint = ws.lb_hint;
  if (hint[0] > kLbOverRadix) {  // the last bucket Localizer here had skewed buckets
    if (++hint[1] < kLbRetry) return DFX_OK;
    hint[0] = 0;
    hint[1] = 0;
  }
  const bool valued = o.value != nullptr && o.occ_x != nullptr;
  int wbits = 1;
  while (wbits < kLbMaxBits && ((int64_t)1024 << wbits) < nnz) ++wbits;
  const uint32_t nbk = 1u << wbits;
  int64_t ntiles = std::min<int64_t>(256, std::max<int64_t>(1, nnz / 4096));
  int64_t rt = std::min<int64_t>(kLbMaxRows, std::max<int64_t>(1, (B + ntiles - 1) / ntiles));
  ntiles = (B + rt - 1) / rt;
  DFX_TRY(ws.keys0.ensure(nnz * 8));
  DFX_TRY(ws.keys1.ensure(nnz * 8));
  DFX_TRY(ws.vals0.ensure(nnz * 8));
  DFX_TRY(ws.vals1.ensure(nnz * 8));
  DFX_TRY(ws.lbq.ensure(nnz * 8));
  DFX_TRY(ws.lbcnt.ensure(sizeof(uint32_t) * ((size_t)ntiles * nbk + 2 * (nbk + 1))));
  {
    void* before = ws.hstat.p;
    DFX_TRY(ws.hstat.ensure(sizeof(unsigned long long) * std::max<int64_t>(nbk, 256)));
    if (ws.hstat.p != before)  // fresh words read as unpublished (tag 0, flag 0)
      DFX_HIP(hipMemsetAsync(ws.hstat.p, 0, ws.hstat.bytes, L.stream));
  }
  LbArgs a{};
  a.B = B; a.nnz = nnz; a.offset = offset; a.index = index; a.max_index = max_index;
  a.keys_ready = o.keys_ready ? 1 : 0;
  a.value = valued ? o.value : nullptr;
  a.rt = rt; a.ntiles = ntiles; a.wbits = wbits;
  a.nt = (c->nt_mask & kNtLane) ? 1 : 0;
  a.tilecnt = ws.lbcnt.as<uint32_t>();
  a.totals = a.tilecnt + (size_t)ntiles * nbk;
  a.bstart = a.totals + nbk + 1;
  a.kbuf = ws.keys0.as<uint64_t>();
  a.kscr = ws.keys1.as<uint64_t>();
  a.sbuf = ws.vals0.as<uint64_t>();
  a.sscr = ws.vals1.as<uint64_t>();
  a.qbuf = ws.lbq.as<uint32_t>();
  a.qscr = a.qbuf + nnz;
  a.ds = L.ds;
  a.hstat = ws.hstat.as<unsigned long long>();
  a.uniq = o.uniq; a.segstart = o.segstart; a.occ_row = o.occ_row;
  a.occ_x = valued ? o.occ_x : nullptr;
  a.hint = ws.lb_hint;
  hipLaunchKernelGGL(k_lb_init, dim3(1), dim3(1), 0, L.stream, L.ds);
  hipLaunchKernelGGL(k_lb_hist, dim3((unsigned)ntiles), dim3(kLbNT), nbk * sizeof(uint32_t),
                     L.stream, a);
  hipLaunchKernelGGL(k_lb_colscan, dim3((nbk + kWave - 1) / kWave), dim3(kLbScanWaves * kWave), 0,
                     L.stream, a);
  const size_t scatter_lds = ((nbk + 1) & ~1u) * sizeof(uint32_t) + (rt + 1) * sizeof(uint64_t);
  if (valued)
    hipLaunchKernelGGL(k_lb_scatter<true>, dim3((unsigned)ntiles), dim3(kLbNT), scatter_lds,
                       L.stream, a);
  else
    hipLaunchKernelGGL(k_lb_scatter<false>, dim3((unsigned)ntiles), dim3(kLbNT), scatter_lds,
                       L.stream, a);
  // the LDS form of the per-bucket sort follows the last batch's item form (a batch whose items
  // do not pack while the launch expected packed ones sorts through global memory: correct)
  const bool q_lds = hint[2] == 2u;
  const dim3 bg(nbk), bb(kLbNT);
  if (valued) {
    if (q_lds) hipLaunchKernelGGL((k_lb_bucket<true, true>), bg, bb, 0, L.stream, a);
    else hipLaunchKernelGGL((k_lb_bucket<false, true>), bg, bb, 0, L.stream, a);
  } else {
    if (q_lds) hipLaunchKernelGGL((k_lb_bucket<true, false>), bg, bb, 0, L.stream, a);
    else hipLaunchKernelGGL((k_lb_bucket<false, false>), bg, bb, 0, L.stream, a);
  }
  DFX_HIP(hipGetLastError());
  *used = true;
  return DFX_OK;
}

}  // namespace dfx
