// Localizer::Compact (src/data/localizer.cc:11-107) as a bucket sort, for the callers that need
// no per-nnz col: the fused step and the split owner, whose forward finds each key in the model
// table itself and whose backward walks each key's occurrences in sorted order.  Eight short
// launches where the radix Localizer (localize.hip + sort.hip) takes ~17, and about half its
// traffic; no look-back chain and no ticket counter (blocks take their tile / bucket by block
// index — device-scope atomics on one word serialise at ~88 per microsecond on MI355X):
//
//   k_lb_init     the batch's key statistics reset
//   k_lb_hist     per tile of rows: every nnz's key (ReverseBytes(id % max_index),
//                 localizer.cc:24) and its bucket into the tile's histogram (LDS); OR / AND /
//                 min / max of the keys.  A key's bucket is a monotone map of the key,
//                 clamp((key - base) >> s), fitted to the key range of the previous batch on this
//                 lane: buckets are ranges of keys in key order whatever the batch holds, and a
//                 batch like the previous one spreads evenly over them
//   k_lb_colscan  per bucket: the exclusive prefix of its counts over the tiles, its total, and
//                 the count of buckets beyond the LDS sort's capacity
//   k_lb_scatter  per tile: the buckets' starts (a scan of the totals), then every nnz's item
//                 into its bucket's range through an LDS cursor per bucket.  An item packs the
//                 key's varying bits above the row (binary data) or the position (valued data,
//                 {value, row} beside it) in one u64 when they fit; else the key and the row /
//                 position travel apart
//   k_lb_big      (exits at once unless a bucket is oversize: skewed keys, or a key range that
//                 moved) such buckets sorted in place through global memory by a few looping
//                 blocks, stable 8-bit LSD passes — slower, the same result; the workspace's hint
//                 then sends the next batches to the radix Localizer and retries every kLbRetry
//   k_lb_wbucket  one wave per bucket: the bucket sorted in LDS — LSD radix over the digits
//                 that vary inside it, on the whole item: (key, row) resp. (key, position) is a
//                 total order and equal items are the same occurrence data, so the scatter's
//                 order inside a bucket never shows — then its heads (CountUniqIndex's run-length
//                 pass) at the bucket's own offset in scratch lists, per occurrence in sorted
//                 order its row (and value), and the bucket's head count
//   k_lb_bscan    one block: the exclusive scan of the head counts (RemapIndex's ranks), U
//   k_lb_out      per bucket its heads to their ranks: per rank its key and segment start
//
// The occurrence order is the radix Localizer's stable (key, position) order: positions ascend
// with rows, and a binary row's repeats of one key are identical items.  So the outputs are
// bit-identical to localize.hip's (test_gpu_r3.py test_bucket_localizer_equals_lsd).
#include <algorithm>
#include <mutex>
#include <set>

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
constexpr int kLbBigBlocks = 64;     // blocks sorting the oversize buckets through global memory

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
  uint32_t* bheads;      // [nbk]: unique keys per bucket (k_lb_wbucket)
  uint32_t* brank;       // [nbk]: the bucket's first rank (k_lb_bscan)
  uint64_t* kbuf;        // items
  uint32_t* qbuf;        // rows / positions of unpacked items
  uint64_t* sbuf;        // side payloads (valued, carried: kwarg lb_gather=0)
  uint2* rowof;          // valued, gathered (lb_gather=1): each position's {row, value bits},
                         // written in input order by k_lb_scatter
  uint64_t* kscr;        // scratch of the global-memory passes
  uint32_t* qscr;
  uint64_t* sscr;
  DevState* ds;
  uint64_t* uniq;
  uint32_t* segstart;
  uint32_t* occ_row;
  float* occ_x;
  unsigned int* hint;    // pinned: Workspace::lb_hint
  int diag;              // Context::lb_diag (measurement only)
  // the hot-key map (Workspace::lbsplit): the previous batch's hot keys (runs of >= hot_th),
  // listed, then laid out over the buckets; per bucket its first and last key and whether its
  // first key continues the previous non-empty bucket's last (a hot key's run over buckets)
  uint64_t* hl_key;      // [kLbHotMax] the list (k_lb_hotlist, unordered)
  uint32_t* hl_len;
  uint64_t* hm_key;      // [kLbHotMax] the map (k_lb_hotmap): hot keys in order,
  uint32_t* hm_p;        // [kLbHotMax + 1] exclusive prefix of (W + 1),
  uint32_t* hm_w;        // [kLbHotMax] buckets per hot key,
  uint32_t* hm_ic;       // [nbk / 2 + 1] per coarse bucket its first hot key
  uint64_t* bfk;
  uint64_t* blk;
  uint32_t* bcont;
  int hm_lds;            // the histogram / scatter launches hold LDS for the map
  int wbits_hot;         // the bucket bits a map is built for (one more than the key map's)
  uint32_t hot_th;       // a hot key's occurrences, at least
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

// The hot-key map, for binary batches after one with hot keys (Zipf keys: C5's top key holds
// ~11 % of a batch's nnz, ~600 buckets' worth, which no map of the key alone can split).  The
// previous batch's keys of >= hot_th occurrences, in key order, each get W_h = ceil(len_h /
// target) buckets of their own; a coarse key map (half the buckets, the key map's form) places
// every other key.  In key order, coarse bucket c holds [cold keys below its first hot key]
// [hot key 1: W_1 buckets] [cold keys between] ... [cold keys above its last hot key]: with
// P_i = sum over the hot keys before i of (W + 1), a cold key of coarse bucket c above q of its
// hot keys (the first being i_c) goes to c + P[i_c + q], and occurrence j of hot key i to
// c + P[i] + 1 + min(W_i - 1, floor(j * W_i / nnz)) — by position, so by row: the map is
// monotone in (key, row) and the buckets still concatenate in sorted order.  Per item a coarse
// bucket, its hot-key range and a compare or two, from LDS.
constexpr int kLbHotMax = 1024;
struct LbHot {
  const uint64_t* hk;
  const uint32_t* hp;
  const uint32_t* hw;
  const uint32_t* ic;
  LbMap cm;
  double inv_nnz;
};
__device__ inline bool lb_hot_on(const LbArgs& a) {
  return a.hm_lds && a.value == nullptr && a.ds->lb_sp_use &&
         a.ds->lb_sp_wbits == (unsigned)a.wbits;
}
__host__ __device__ constexpr size_t lb_hot_lds(uint32_t nbk) {
  return (size_t)kLbHotMax * 8 + ((size_t)kLbHotMax + 1) * 4 + (size_t)kLbHotMax * 4 +
         ((size_t)nbk / 2 + 1) * 4;
}
__device__ inline LbHot lb_stage_hot(const LbArgs& a, void* lds, int t, int nt) {
  LbHot h;
  uint64_t* hk = reinterpret_cast<uint64_t*>(lds);
  uint32_t* hp = reinterpret_cast<uint32_t*>(hk + kLbHotMax);
  uint32_t* hw = hp + kLbHotMax + 1;
  uint32_t* ic = hw + kLbHotMax;
  const uint32_t n = a.ds->lb_hm_n, C = (1u << a.wbits) / 2;
  for (uint32_t i = t; i < n; i += nt) {
    hk[i] = a.hm_key[i];
    hw[i] = a.hm_w[i];
  }
  for (uint32_t i = t; i <= n; i += nt) hp[i] = a.hm_p[i];
  for (uint32_t c = t; c <= C; c += nt) ic[c] = a.hm_ic[c];
  h.hk = hk;
  h.hp = hp;
  h.hw = hw;
  h.ic = ic;
  h.cm.nbk = C;
  h.cm.base = a.ds->lb_hm_base;
  h.cm.s = (int)a.ds->lb_hm_s;
  h.inv_nnz = 1.0 / (double)a.nnz;
  return h;
}
__device__ inline uint32_t lb_hot_bucket(uint64_t k, uint64_t j, const LbHot& h) {
  const uint32_t c = lb_bucket(k, h.cm);
  uint32_t i = h.ic[c];
  const uint32_t i1 = h.ic[c + 1];
  for (; i < i1; ++i) {
    const uint64_t hkey = h.hk[i];
    if (hkey >= k) {
      if (hkey == k) {
        const uint32_t W = h.hw[i];
        uint32_t sub = (uint32_t)((double)j * (double)W * h.inv_nnz);
        sub = sub < W - 1 ? sub : W - 1;
        return c + h.hp[i] + 1 + sub;
      }
      break;
    }
  }
  return c + h.hp[i];
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
  ds->lb_over = 0;
  ds->lb_hot = 0;
  ds->lb_nhot = 0;
  unsigned* meta = ds->sortmeta;
  meta[kSortMetaEpoch] = ++ds->sort_epoch;  // tags this Localizer's look-back words
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

constexpr int kLbUnr = 8;  // ids in flight per thread

// the histogram and scatter kernels' blocks: 16 waves on a tile by default, for the loads in
// flight (kwarg lb_hnt = 256 | 512 | 1024)

// HOT: instantiated with the hot-key map's lookup (the key map's launches keep their registers)
template <int HNT, bool HOT>
__global__ __launch_bounds__(HNT) void k_lb_hist(LbArgs a) {
  constexpr int kLbHNT = HNT, kLbHWaves = HNT / kWave;
  extern __shared__ uint64_t lb_dyn64[];  // 8-byte aligned: the splitter keys follow hist
  uint32_t* hist = reinterpret_cast<uint32_t*>(lb_dyn64);
  __shared__ unsigned long long red[4][kLbHWaves];
  const LbMap m = lb_map(a.ds, a.wbits);
  const int t = threadIdx.x;
  for (uint32_t d = t; d < m.nbk; d += kLbHNT) hist[d] = 0;
  const bool qs = HOT && lb_hot_on(a);
  LbHot hm{};
  if (qs) hm = lb_stage_hot(a, hist + m.nbk, t, kLbHNT);
  const int64_t tile = blockIdx.x;
  const int64_t r0 = tile * a.rt;
  const int64_t r1 = r0 + a.rt < a.B ? r0 + a.rt : a.B;
  const uint64_t j0 = a.offset[r0], j1 = a.offset[r1];
  __syncthreads();
  unsigned long long vor = 0, vand = ~0ull, vmin = ~0ull, vmax = 0;
  for (uint64_t jb = j0; jb < j1; jb += (uint64_t)kLbUnr * kLbHNT) {
    uint64_t id[kLbUnr];
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t j = jb + (uint64_t)u * kLbHNT + t;
      id[u] = j < j1 ? ldnt(a.index + j, a.nt != 0) : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t j = jb + (uint64_t)u * kLbHNT + t;
      if (j < j1) {
        const uint64_t k = lb_key(id[u], a.max_index, a.keys_ready);
        vor |= k;
        vand &= k;
        vmin = k < vmin ? k : vmin;
        vmax = k > vmax ? k : vmax;
        atomicAdd(&hist[qs ? lb_hot_bucket(k, j, hm) : lb_bucket(k, m)], 1u);
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
  uint32_t* dst = a.tilecnt + (size_t)tile * m.nbk;
  for (uint32_t d = t; d < m.nbk; d += kLbHNT) dst[d] = hist[d];
  if (t == 0 && j1 > j0) {
    for (int i = 1; i < kLbHWaves; ++i) {
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
    if (ok) {
      a.totals[b] = run;
      // (rare) k_lb_big's gate; the AUC's view of this scan has no state
      if (a.ds && run > (uint32_t)kLbCap) atomicAdd(&a.ds->lb_over, 1u);
    }
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

template <bool S, int HNT, bool HOT>
__global__ __launch_bounds__(HNT) void k_lb_scatter(LbArgs a) {
  constexpr int kLbHNT = HNT, kLbHWaves = HNT / kWave;
  extern __shared__ uint64_t lb_dyn64[];
  __shared__ uint32_t lds[kLbHWaves + 1];
  __shared__ uint32_t whist[kLbHWaves][kWave];
  const LbMap m = lb_map(a.ds, a.wbits);
  uint32_t* cur = reinterpret_cast<uint32_t*>(lb_dyn64);  // per bucket: this tile's next slot
  uint64_t* offs = lb_dyn64 + (m.nbk + 1u) / 2;
  const int t = threadIdx.x;
  const bool qs = HOT && lb_hot_on(a);
  LbHot hm{};
  if (qs) hm = lb_stage_hot(a, offs + a.rt + 1, t, kLbHNT);
  // (lb_diag 512, measurement only) each XCD a contiguous range of tiles
  const int64_t tile = ((a.diag & 512) && a.ntiles % 8 == 0)
                           ? (int64_t)(blockIdx.x % 8) * (a.ntiles / 8) + blockIdx.x / 8
                           : (int64_t)blockIdx.x;
  const int64_t r0 = tile * a.rt;
  const int nr = (int)(a.B - r0 < a.rt ? a.B - r0 : a.rt);
  // the buckets' starts: thread t holds buckets [t * per, (t + 1) * per)
  const uint32_t per = (m.nbk + kLbHNT - 1) / kLbHNT;
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
  uint32_t ex = block_excl_scan<kLbHNT>(mine, lds, &total);
  const uint32_t* pre = a.tilecnt + (size_t)tile * m.nbk;
  const bool mid4 = (a.diag & 512) && per == 4;  // (measurement only) 4 buckets per cursor
  uint32_t msum = 0;
  const uint32_t mex = ex;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t d = t * per + i;
    if (d < m.nbk) {
      if (!mid4) cur[d] = ex + pre[d];
      msum += pre[d];
      if (blockIdx.x == 0) a.bstart[d] = ex;
      ex += a.totals[d];
    }
  }
  if (mid4) {
    __syncthreads();
    cur[t] = mex + msum;
  }
  if (a.diag & 256) {  // (measurement only) tile-local positions: the tile's items by bucket
    auto tcnt = [&](uint32_t d) {
      const uint32_t nx = tile + 1 < a.ntiles ? a.tilecnt[(size_t)(tile + 1) * m.nbk + d]
                                              : a.totals[d];
      return nx - pre[d];
    };
    uint32_t lm = 0;
    for (uint32_t i = 0; i < per; ++i)
      if (t * per + i < m.nbk) lm += tcnt(t * per + i);
    uint32_t lex = block_excl_scan<kLbHNT>(lm, lds, nullptr);
    for (uint32_t i = 0; i < per; ++i) {
      const uint32_t d = t * per + i;
      if (d < m.nbk) {
        const uint32_t cd = tcnt(d);
        cur[d] = lex;
        lex += cd;
      }
    }
  }
  const uint64_t qmax = (S || a.rowof) ? (uint64_t)(a.nnz - 1) : (uint64_t)(a.B - 1);
  const LbPack p = lb_pack(a.ds, qmax);
  if (blockIdx.x == 0) {
    uint32_t nover;
    (void)block_excl_scan<kLbHNT>(over, lds, &nover);
    if (t == 0) {
      a.bstart[m.nbk] = total;
      // the next batches' choice (pinned host words, vector stores)
      a.hint[0] = nover;
      a.hint[2] = p.packed ? 1u : 2u;
    }
  }
  for (int i = t; i <= nr; i += kLbHNT) offs[i] = a.offset[r0 + i];
  __syncthreads();
  const uint64_t j0 = offs[0], j1 = offs[nr];
  const uint64_t qmask = p.rb ? (~0ull >> (64 - p.rb)) : 0ull;
  // Each wave takes a contiguous segment of kLbUnr * 64 items per round, 64 per step, and
  // carries the row of its window's first item from step to step: the rows of a window's
  // items are that row plus the count of the next 64 rows' starts at or before each item — a
  // histogram of the starts' offsets in the window (LDS) and a wave scan, one LDS round trip
  // where a binary search over the tile's offsets took nine.  When all of the next 64 rows
  // start inside the window (rows of one item, or empty rows) the step searches instead.
  const int w = t / kWave, l = lane_id();
  uint32_t* wh = whist[w];
  auto search = [&](uint64_t j) {  // the row of item j: upper_bound(j) - 1 over offs[0..nr]
    int lo = 0, hi = (a.diag & 8) ? 0 : nr;  // (diag 8, measurement only: no search)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offs[mid] <= j) lo = mid; else hi = mid;
    }
    return lo;
  };
  for (uint64_t jb = j0; jb < j1; jb += (uint64_t)kLbUnr * kLbHNT) {
    const uint64_t wj = jb + (uint64_t)w * kLbUnr * kWave;
    uint64_t id[kLbUnr];
    float x[kLbUnr];
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t j = wj + (uint64_t)u * kWave + l;
      id[u] = j < j1 ? ldnt(a.index + j, a.nt != 0) : 0ull;
      if (S) x[u] = j < j1 ? ldnt(a.value + j, a.nt != 0) : 0.f;
    }
    if (wj >= j1) continue;  // wave-uniform
    int ra = search(wj);     // the row of the window's first item (wave-uniform)
#pragma unroll
    for (int u = 0; u < kLbUnr; ++u) {
      const uint64_t J = wj + (uint64_t)u * kWave;
      if (J >= j1) break;  // wave-uniform
      const int rl = ra + 1 + l;
      const uint64_t sl = rl <= nr ? offs[rl] : ~0ull;  // > J
      wh[l] = 0;
      __builtin_amdgcn_wave_barrier();
      if (sl - J < (uint64_t)kWave) atomicAdd(&wh[sl - J], 1u);
      __builtin_amdgcn_wave_barrier();
      const uint32_t before = wave_incl_scan(wh[l]);  // the next rows starting at <= J + l
      __builtin_amdgcn_wave_barrier();
      const bool full = __shfl(sl, kWave - 1, kWave) <= J + kWave;
      const uint64_t j = J + l;
      const int lo = full ? search(j) : ra + (int)before;
      ra = full ? search(J + kWave)
                : ra + (int)__popcll(__ballot(sl <= J + kWave));
      if (j >= j1) continue;
      const uint64_t k = lb_key(id[u], a.max_index, a.keys_ready);
      const uint32_t row = (uint32_t)(r0 + lo);
      const uint64_t q = S ? j : (uint64_t)row;
      const uint32_t bk = qs ? lb_hot_bucket(k, j, hm) : lb_bucket(k, m);
      const uint32_t pos = atomicAdd(&cur[mid4 ? bk >> 2 : bk], 1u);
      // (lb_diag 128, measurement only: the same items written contiguously, by input
      // position, to a scratch buffer — the scatter's work without its scattered writes)
      stnt((a.diag & 128) ? a.sscr + j : (a.diag & (256 | 512)) ? a.sscr + (a.diag & 256 ? j0 : 0) + pos : a.kbuf + pos,
           p.packed ? ((((k - p.kmin) >> p.lo) << p.rb) | (q & qmask)) : k, a.nt != 0);
      if (!p.packed) a.qbuf[pos] = (uint32_t)q;
      if (S && a.rowof) a.rowof[j] = make_uint2(row, __float_as_uint(x[u]));  // input order
      else if (S) a.sbuf[pos] = (uint64_t)__float_as_uint(x[u]) | ((uint64_t)row << 32);
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

// ---- a bucket's stable LSD radix sort in LDS (n <= kLbCap items) ------------------------------
// The items stay in registers, kLbIT per thread — thread (wave w, lane l) holds positions
// w * 64 * kLbIT + c * 64 + l, c < kLbIT — and each pass over an 8-bit digit that varies inside
// the bucket ranks them with wave ballots (wave w's items before wave w+1's, in order: stable),
// scatters them through the LDS buffers and reads them back in the new order; the last pass
// leaves the sorted bucket in the LDS buffers.  q's digits go first when the items are not packed
// (q is the less significant part of (key, q)).  About 16 bytes of LDS traffic per item and pass,
// where a bitonic network over 1024 items moved ~880 (LDS-bound at 4096 buckets: ~220 us).
constexpr int kLbRadixIT = kLbCap / kLbNT;  // 8

template <bool Q, bool S>
__device__ inline void lb_lds_sort(uint64_t (&k)[kLbRadixIT], uint32_t (&q)[kLbRadixIT],
                                   uint64_t (&sv)[kLbRadixIT], int n, bool hasq,
                                   uint64_t* sk, uint32_t* sq, uint64_t* ss,
                                   uint32_t (*wcnt)[256], uint32_t* lds,
                                   unsigned long long (*red)[kLbWaves]) {
  const int t = threadIdx.x, w = t / kWave, l = lane_id();
  const int wb = w * kWave * kLbRadixIT;
  // the digits that vary inside the bucket
  unsigned long long kor = 0, kand = ~0ull, qor = 0, qand = ~0ull;
#pragma unroll
  for (int c = 0; c < kLbRadixIT; ++c) {
    if (wb + c * kWave + l < n) {
      kor |= k[c];
      kand &= k[c];
      if (Q && hasq) {
        qor |= q[c];
        qand &= q[c];
      }
    }
  }
  kor = lb_wave_or(kor);
  kand = lb_wave_and(kand);
  if (Q) {
    qor = lb_wave_or(qor);
    qand = lb_wave_and(qand);
  }
  if (l == 0) {
    red[0][w] = kor;
    red[1][w] = kand;
    red[2][w] = qor;
    red[3][w] = qand;
  }
  __syncthreads();
  for (int i = 0; i < kLbWaves; ++i) {
    kor |= red[0][i];
    kand &= red[1][i];
    qor |= red[2][i];
    qand &= red[3][i];
  }
  const unsigned long long kvary = kor ^ kand, qvary = (Q && hasq) ? (qor ^ qand) : 0ull;
  int last = -1;  // the last active pass (0..3: q's digits, 4..11: the key's)
  for (int pass = 0; pass < 12; ++pass) {
    const unsigned long long vary = pass < 4 ? qvary : kvary;
    const int shift = 8 * (pass < 4 ? pass : pass - 4);
    if ((vary >> shift) & 255ull) last = pass;
  }
  if (last < 0) {  // one item value (or none): in place
#pragma unroll
    for (int c = 0; c < kLbRadixIT; ++c) {
      const int idx = wb + c * kWave + l;
      if (idx < n) {
        sk[idx] = k[c];
        if (Q && hasq) sq[idx] = q[c];
        if (S) ss[idx] = sv[c];
      }
    }
    __syncthreads();
    return;
  }
  for (int pass = 0; pass <= last; ++pass) {
    const bool on_q = pass < 4;
    const unsigned long long vary = on_q ? qvary : kvary;
    const int shift = 8 * (on_q ? pass : pass - 4);
    if (((vary >> shift) & 255ull) == 0) continue;
#pragma unroll
    for (int i = 0; i < 256 / kWave; ++i) wcnt[w][i * kWave + l] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t dr[kLbRadixIT];
#pragma unroll
    for (int c = 0; c < kLbRadixIT; ++c) {
      const bool valid = wb + c * kWave + l < n;
      const uint32_t d = !valid ? 0u : on_q ? (q[c] >> shift) & 255u
                                            : (uint32_t)(k[c] >> shift) & 255u;
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
      dr[c] = d | ((old + rk) << 8);
    }
    __syncthreads();
    {  // digit t: the waves' exclusive offsets, then the digit's start in the bucket
      uint32_t run = 0;
#pragma unroll
      for (int i = 0; i < kLbWaves; ++i) {
        const uint32_t x = wcnt[i][t];
        wcnt[i][t] = run;
        run += x;
      }
      const uint32_t st = block_excl_scan<kLbNT>(run, lds, nullptr);
#pragma unroll
      for (int i = 0; i < kLbWaves; ++i) wcnt[i][t] += st;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kLbRadixIT; ++c) {
      if (wb + c * kWave + l < n) {
        const uint32_t pos = wcnt[w][dr[c] & 255u] + (dr[c] >> 8);
        sk[pos] = k[c];
        if (Q && hasq) sq[pos] = q[c];
        if (S) ss[pos] = sv[c];
      }
    }
    __syncthreads();
    if (pass == last) break;  // the sorted bucket stays in LDS
#pragma unroll
    for (int c = 0; c < kLbRadixIT; ++c) {
      const int idx = wb + c * kWave + l;
      if (idx < n) {
        k[c] = sk[idx];
        if (Q && hasq) q[c] = sq[idx];
        if (S) sv[c] = ss[idx];
      }
    }
    __syncthreads();
  }
}

// Buckets the LDS sort cannot take — beyond kLbCap items (skewed keys, or a key range that
// moved), or unpacked items while the launch expected packed ones (q_lds = 0) — sorted in place by
// a few looping blocks, through global memory, before k_lb_wbucket reads them: stable 8-bit LSD
// passes over the digits that vary inside the bucket, q's first (the less significant part of an
// unpacked item), then the key's; the result copied back when it ends in the scratch buffers.
// Kept out of k_lb_wbucket, whose registers would otherwise be sized for it.
__device__ inline bool lb_needs_global(int64_t n, bool packed, int q_lds) {
  return n > kLbCap || (!packed && !q_lds);
}

template <bool S>
__global__ __launch_bounds__(kLbNT) void k_lb_big(LbArgs a, int q_lds) {
  __shared__ uint32_t wcnt[kLbWaves][256];
  __shared__ uint32_t base[256];
  __shared__ uint32_t lds[kLbWaves + 1];
  __shared__ unsigned long long s_red[4][kLbWaves];
  const int t = threadIdx.x;
  const uint32_t nbk = 1u << a.wbits;
  const uint64_t qmax = (S || a.rowof) ? (uint64_t)(a.nnz - 1) : (uint64_t)(a.B - 1);
  const LbPack p = lb_pack(a.ds, qmax);
  const bool hasq = !p.packed;
  // nothing to do unless a bucket is oversize or the items did not pack as the launch expected
  if (__hip_atomic_load(&a.ds->lb_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
      (p.packed || q_lds))
    return;
  __shared__ uint32_t s_list[kLbNT];
  __shared__ uint32_t s_nlist;
  uint32_t listed = 0;  // buckets needing this kernel so far; block i takes the list's i, i + G, ...
  for (uint32_t b0 = 0; b0 < nbk; b0 += kLbNT) {
    const uint32_t bb = b0 + t;
    const int64_t nb = bb < nbk ? (int64_t)a.bstart[bb + 1] - (int64_t)a.bstart[bb] : 0;
    const uint32_t need = (bb < nbk && nb > 1 && lb_needs_global(nb, p.packed, q_lds)) ? 1u : 0u;
    uint32_t cnt;
    const uint32_t ex = block_excl_scan<kLbNT>(need, lds, &cnt);
    if (t == 0) s_nlist = 0;
    __syncthreads();
    if (need && (listed + ex) % gridDim.x == blockIdx.x) s_list[atomicAdd(&s_nlist, 1u)] = bb;
    __syncthreads();
    listed += cnt;
    const uint32_t nl = s_nlist;
    // (the order of a block's own buckets does not matter: each is sorted on its own)
    for (uint32_t li = 0; li < nl; ++li) {
    const uint32_t b = s_list[li];
    const int64_t start = a.bstart[b];
    const int64_t n = (int64_t)a.bstart[b + 1] - start;
    unsigned long long kor = 0, kand = ~0ull, qor = 0, qand = ~0ull;
    for (int64_t i = t; i < n; i += kLbNT) {
      const uint64_t x = a.kbuf[start + i];
      kor |= x;
      kand &= x;
      if (hasq) {
        qor |= a.qbuf[start + i];
        qand &= a.qbuf[start + i];
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
    int np = 0;
    for (int pass = 0; pass < 12; ++pass) {
      const bool on_q = pass < 4;
      const int shift = 8 * (on_q ? pass : pass - 4);
      const unsigned long long vary = on_q ? (hasq ? (qor ^ qand) : 0ull) : (kor ^ kand);
      if (((vary >> shift) & 255ull) == 0) continue;
      lb_global_pass<S>(Xk, Xq, Xs, Yk, Yq, Ys, n, on_q, shift, wcnt, base, lds);
      uint64_t* tk = Xk; Xk = Yk; Yk = tk;
      uint32_t* tq = Xq; Xq = Yq; Yq = tq;
      uint64_t* ts = Xs; Xs = Ys; Ys = ts;
      ++np;
    }
    if (np & 1) {  // the sorted bucket sits in the scratch buffers: back into place
      for (int64_t i = t; i < n; i += kLbNT) {
        Yk[i] = Xk[i];
        if (hasq) Yq[i] = Xq[i];
        if (S) Ys[i] = Xs[i];
      }
    }
    __syncthreads();
    }
    __syncthreads();  // s_list is rewritten by the next chunk
  }
}

// ---- the per-bucket sort and outputs, one wave per bucket, no block barrier.  The wave holds up to kLbCap items, kLbWIT per lane (lane l's slot c is the
// bucket's position c * 64 + l), ranks each pass's digits with ballots against its own 256
// counters, scans them across its lanes, scatters through LDS and reads back; the heads' ranks
// are a ballot prefix per slot.  A 64-thread block per bucket: ~17 KiB of LDS and one wave, so
// the buckets pack the CUs around the backward's blocks, and no pass waits on other waves.
constexpr int kLbWIT = kLbCap / kWave;  // 32

// a bucket's n <= kLbCap items (+ rows / positions, side payloads) sorted by one wave into LDS:
// LSD radix over the digits that vary inside the bucket, q's first when the items are not
// packed; positions >= n of the last slot hold padding ~0.

template <bool Q, bool S>
__device__ __attribute__((always_inline)) inline void lb_wave_sort(
    const uint64_t* gk, const uint32_t* gq, const uint64_t* gs, int n, bool hasq, int ntp,
    int diag, uint64_t* sk, uint32_t* sq, uint64_t* ss, uint32_t* cnt) {
  const int l = threadIdx.x;
  const int nc = (n + kWave - 1) / kWave;  // slots in use (wave-uniform)
  // the last slot's lanes past n hold padding ~0, which sorts after every item (packed items
  // keep the top bit clear; raw keys are never kEmptyKey): every pass then runs on whole
  // slots with no lane masks, and the padding ends at positions >= n
  uint64_t k[kLbWIT], sv[kLbWIT];
  uint32_t q[kLbWIT];
#pragma unroll
  for (int c = 0; c < kLbWIT; ++c) {  // every load in flight at once
    const int i = c * kWave + l;
    const bool v = c < nc && i < n;
    k[c] = v ? ldnt(gk + i, ntp != 0) : ~0ull;
    q[c] = (Q && hasq) ? (v ? gq[i] : ~0u) : 0u;
    sv[c] = (S && v) ? gs[i] : 0ull;
  }
  unsigned long long kor = 0, kand = ~0ull, qor = 0, qand = ~0ull;
#pragma unroll
  for (int c = 0; c < kLbWIT; ++c) {
    if (c < nc) {  // (no item and no q equals its padding, all ones: no lane masks)
      kor |= k[c] == ~0ull ? 0ull : k[c];
      kand &= k[c];
      if (Q && hasq) {
        qor |= q[c] == ~0u ? 0u : q[c];
        qand &= q[c];
      }
    }
  }
  kor = lb_wave_or(kor);
  kand = lb_wave_and(kand);
  if (Q) {
    qor = lb_wave_or(qor);
    qand = lb_wave_and(qand);
  }
  const unsigned long long kvary = kor ^ kand, qvary = (Q && hasq) ? (qor ^ qand) : 0ull;
  // the passes (wave-uniform): q's 4 digits, then the item's 8 (an item's low rb bits are its
  // row / position when the items are packed)
  auto passes = [&]() {
    auto pass_at = [&](int pass, bool* on_q, int* shift) {
      *on_q = pass < 4;
      *shift = 8 * (*on_q ? pass : pass - 4);
      return true;
    };
    int last = -1;  // the last active pass
    if (!(diag & 1))
      for (int pass = 0; pass < 12; ++pass) {
        bool on_q;
        int shift;
        if (!pass_at(pass, &on_q, &shift)) break;
        if (((on_q ? qvary : kvary) >> shift) & 255ull) last = pass;
      }
    if (last < 0) {  // one item value (or none; or diag 1): in place
#pragma unroll
      for (int c = 0; c < kLbWIT; ++c) {
        if (c < nc) {
          const int i = c * kWave + l;
          sk[i] = k[c];
          if (Q && hasq) sq[i] = q[c];
          if (S) ss[i] = sv[c];
        }
      }
    }
    for (int pass = 0; pass <= last; ++pass) {
      bool on_q;
      int shift;
      (void)pass_at(pass, &on_q, &shift);
      const unsigned long long vary = on_q ? qvary : kvary;
      if (((vary >> shift) & 255ull) == 0) continue;
#pragma unroll
      for (int i = 0; i < 256 / kWave; ++i) cnt[i * kWave + l] = 0;
      __builtin_amdgcn_wave_barrier();
      // the digits' counts (LDS adds, no return), their starts, then each slot's items ranked
      // by ballots on the digit's running start and scattered
#pragma unroll
      for (int c = 0; c < kLbWIT; ++c) {
        if (c < nc) {
          const uint32_t d = on_q ? (q[c] >> shift) & 255u : (uint32_t)(k[c] >> shift) & 255u;
          atomicAdd(&cnt[d], 1u);
        }
      }
      __builtin_amdgcn_wave_barrier();
      {  // lane l holds digits 4l .. 4l + 3
        const uint32_t c0 = cnt[4 * l], c1 = cnt[4 * l + 1], c2 = cnt[4 * l + 2],
                       c3 = cnt[4 * l + 3];
        const uint32_t s4 = c0 + c1 + c2 + c3;
        const uint32_t ex = wave_incl_scan(s4) - s4;
        __builtin_amdgcn_wave_barrier();
        cnt[4 * l] = ex;
        cnt[4 * l + 1] = ex + c0;
        cnt[4 * l + 2] = ex + c0 + c1;
        cnt[4 * l + 3] = ex + c0 + c1 + c2;
        __builtin_amdgcn_wave_barrier();
      }
      uint32_t pos[kLbWIT];
#pragma unroll
      for (int c = 0; c < kLbWIT; ++c) {
        pos[c] = 0;
        if (c < nc) {
          const uint32_t d = on_q ? (q[c] >> shift) & 255u : (uint32_t)(k[c] >> shift) & 255u;
          uint64_t peers = ~0ull;
#pragma unroll
          for (int bt = 0; bt < 8; ++bt) {
            const bool bit = (d >> bt) & 1u;
            const uint64_t mb = __ballot(bit);
            peers &= bit ? mb : ~mb;
          }
          const uint32_t rk = (uint32_t)__popcll(peers & lanemask_lt());
          const uint32_t base = cnt[d];
          __builtin_amdgcn_wave_barrier();
          if (rk == 0) cnt[d] = base + (uint32_t)__popcll(peers);
          __builtin_amdgcn_wave_barrier();
          pos[c] = base + rk;
        }
      }
      // all reads of this pass's items are done (they are in registers): scatter
#pragma unroll
      for (int c = 0; c < kLbWIT; ++c) {
        if (c < nc) {
          sk[pos[c]] = k[c];
          if (Q && hasq) sq[pos[c]] = q[c];
          if (S) ss[pos[c]] = sv[c];
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (pass == last) break;  // the sorted bucket stays in LDS
#pragma unroll
      for (int c = 0; c < kLbWIT; ++c) {
        if (c < nc) {
          const int i = c * kWave + l;
          k[c] = sk[i];
          if (Q && hasq) q[c] = sq[i];
          if (S) sv[c] = ss[i];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
  };
  passes();
}

template <bool Q, bool S>
__global__ __launch_bounds__(kWave) void k_lb_wbucket(LbArgs a) {
  __shared__ uint64_t sk[kLbCap];
  __shared__ uint32_t sq[Q ? kLbCap : 1];
  __shared__ uint64_t ss[S ? kLbCap : 1];
  __shared__ uint32_t cnt[256];
  DevState* ds = a.ds;
  const int l = threadIdx.x;
  const uint32_t b = blockIdx.x;
  const int64_t start = a.bstart[b];
  const int n = (int)((int64_t)a.bstart[b + 1] - start);
  const uint64_t qmax = (S || a.rowof) ? (uint64_t)(a.nnz - 1) : (uint64_t)(a.B - 1);
  const LbPack p = lb_pack(ds, qmax);
  const bool hasq = !p.packed;
  // sorted in LDS here, or already in place (k_lb_big)
  const bool fast = !lb_needs_global(n, p.packed, Q ? 1 : 0);
  const uint64_t* gk = a.kbuf + start;
  const uint32_t* gq = a.qbuf + start;
  const uint64_t* gs = a.sbuf + start;
  const int nc = (n + kWave - 1) / kWave;  // slots in use (wave-uniform)
  if (fast)
    lb_wave_sort<Q, S>(gk, gq, gs, n, hasq, a.nt, a.diag, sk, sq, ss, cnt);
  // ---- per occurrence its row (and value); per head its key and segment start at the
  // bucket's own offset in the scratch lists (k_lb_out moves them to their ranks); a segment
  // longer than kChunkOcc raises the chunk plan's gate.  Instantiated for the LDS and for the
  // global-memory copy apart: one pointer chosen at run time would make every read a flat load.
  const uint64_t qmask = p.rb ? (~0ull >> (64 - p.rb)) : 0ull;
  uint32_t* tseg = a.qscr + start;
  uint64_t* tkey = a.kscr + start;
  uint32_t run = 0;
  bool longseg = false, hot = false;
  const int th = (int)a.hot_th;  // a run this long inside the bucket: the batch has a hot key
  auto fullkey = [&](uint64_t it) { return p.packed ? (((it >> p.rb) << p.lo) + p.kmin) : it; };
  auto heads = [&](const uint64_t* K, const uint32_t* Qs, const uint64_t* Ss) {
    uint64_t prev = 0;  // the key bits of the item before this slot's first
    for (int c = 0; c < nc; ++c) {
      const int i = c * kWave + l;
      const bool valid = i < n;
      const uint64_t it = valid ? K[i] : 0ull;
      const uint64_t kb = lb_keybits(p, it);
      const uint64_t up = __shfl_up(kb, 1, kWave);
      const bool h = valid && (i == 0 || kb != (l == 0 ? prev : up));
      if (valid && i >= kChunkOcc && kb == lb_keybits(p, K[i - kChunkOcc])) longseg = true;
      // (a run of >= th is a long one first: uniform batches never read the extra item)
      if (longseg && valid && i >= th && kb == lb_keybits(p, K[i - th])) hot = true;
      prev = __shfl(kb, kWave - 1, kWave);
      const uint64_t hb = __ballot(h);
      if (!(a.diag & 4) && valid) {
        if (h) {
          const uint32_t r = run + (uint32_t)__popcll(hb & lanemask_lt());
          tkey[r] = fullkey(it);
          tseg[r] = (uint32_t)(start + i);
        }
        uint32_t row;
        if (S) {
          const uint64_t sw = Ss[i];
          row = (uint32_t)(sw >> 32);
          if (a.occ_x) a.occ_x[start + i] = __uint_as_float((uint32_t)sw);
        } else if (a.rowof) {  // valued: the position now, its row and value by k_lb_gather
          row = p.packed ? (uint32_t)(it & qmask) : Qs[i];
        } else {
          row = p.packed ? (uint32_t)(it & qmask) : Qs[i];
        }
        a.occ_row[start + i] = row;
      }
      run += (uint32_t)__popcll(hb);
    }
  };
  if (fast) heads(sk, sq, ss);
  else heads(gk, gq, gs);
  // the bucket's first and last key (k_lb_bscan's continuations)
  if (n > 0 && l == 0) {
    a.bfk[b] = fullkey(fast ? sk[0] : gk[0]);
    a.blk[b] = fullkey(fast ? sk[n - 1] : gk[n - 1]);
  }
  // (each flag raised once or so: one-word atomics serialise)
  if (__ballot(hot) && l == 0 &&
      __hip_atomic_load(&ds->lb_hot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    atomicOr(&ds->lb_hot, 1u);
  if (__ballot(longseg) && l == 0 &&
      __hip_atomic_load(&ds->n_init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    atomicOr(&ds->n_init, 1u);
  if (l == 0) a.bheads[b] = run;
}

// the buckets' first ranks: an exclusive scan of their head counts (one block); U, the closing
// segment start, and the bucket map of the next batch on this lane
constexpr int kLbScanNT = 1024;
__global__ __launch_bounds__(kLbScanNT) void k_lb_bscan(LbArgs a) {
  __shared__ uint32_t lds[kLbScanNT / kWave + 1];
  __shared__ int s_last[kLbScanNT];
  const int t = threadIdx.x;
  const uint32_t nbk = 1u << a.wbits;
  const uint32_t per = (nbk + kLbScanNT - 1) / kLbScanNT;
  // a bucket whose first key is the previous non-empty bucket's last continues that key's run
  // (the hot-key map spreads a hot key over buckets): its first head is no new rank.  Only
  // under the hot-key map (a key map keeps a key in one bucket)
  const bool hm = lb_hot_on(a);
  int lastne = -1;
  for (uint32_t i = 0; hm && i < per; ++i) {
    const uint32_t d = t * per + i;
    if (d < nbk && a.bstart[d + 1] > a.bstart[d]) lastne = (int)d;
  }
  s_last[t] = lastne;
  __syncthreads();
  for (int off = 1; hm && off < kLbScanNT; off <<= 1) {  // inclusive max scan
    const int v = t >= off ? s_last[t - off] : -1;
    __syncthreads();
    if (v > s_last[t]) s_last[t] = v;
    __syncthreads();
  }
  int prev = t > 0 && hm ? s_last[t - 1] : -1;
  uint32_t mine = 0, anycont = 0;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t d = t * per + i;
    if (d < nbk) {
      uint32_t c = 0;
      if (hm && a.bstart[d + 1] > a.bstart[d]) {
        if (prev >= 0 && a.bfk[d] == a.blk[prev]) c = 1;
        prev = (int)d;
      }
      a.bcont[d] = c;
      anycont |= c;
      mine += a.bheads[d] - c;
    }
  }
  uint32_t U;
  uint32_t ex = block_excl_scan<kLbScanNT>(mine, lds, &U);
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t d = t * per + i;
    if (d < nbk) {
      a.brank[d] = ex;
      ex += a.bheads[d] - a.bcont[d];
    }
  }
  // a continued run may be long although no bucket's part is: the chunk plan's gate opens (an
  // open gate with no long segment plans no chunk — the same result)
  if (anycont && __hip_atomic_load(&a.ds->n_init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    atomicOr(&a.ds->n_init, 1u);
  if (t == 0) {
    DevState* ds = a.ds;
    ds->u_count = U;
    if (a.segstart) a.segstart[U] = (uint32_t)a.nnz;
    ds->pk_min = ds->kmin;
    ds->pk_max = ds->kmax;
    ds->pk_valid = 1u;
  }
}

// every bucket's heads to their ranks: uniq[rank] and segstart[rank] (RemapIndex's ranks,
// localizer.cc:53-107), a contiguous run per bucket
__global__ __launch_bounds__(kLbNT) void k_lb_out(LbArgs a) {
  const uint32_t b = blockIdx.x;
  const int64_t start = a.bstart[b];
  const uint32_t h = a.bheads[b], r0 = a.brank[b], c = a.bcont[b];
  for (uint32_t j = threadIdx.x + c; j < h; j += kLbNT) {
    if (a.uniq) a.uniq[r0 + j - c] = a.kscr[start + j];
    if (a.segstart) a.segstart[r0 + j - c] = a.qscr[start + j];
  }
}

// binary batches with a hot key (k_lb_wbucket's flag): every segment of >= hot_th occurrences
// listed (key, length), for the next batch's hot-key map; a grid-stride pass over the U segments
constexpr int kLbHotGrid = 512;
__global__ __launch_bounds__(kLbNT) void k_lb_hotlist(LbArgs a) {
  DevState* ds = a.ds;
  // under the hot-key map a hot key's run is split over buckets in parts of <= target, which may
  // be below hot_th, so no bucket raises lb_hot: a batch placed by the map lists its hot keys
  // whatever the flag says (else the map would switch off every other batch)
  if (ds->lb_hot == 0u && !lb_hot_on(a)) return;
  const int64_t U = ds->u_count;
  for (int64_t i = (int64_t)blockIdx.x * kLbNT + threadIdx.x; i < U;
       i += (int64_t)gridDim.x * kLbNT) {
    const uint32_t len = a.segstart[i + 1] - a.segstart[i];
    if (len >= a.hot_th) {
      const uint32_t x = atomicAdd(&ds->lb_nhot, 1u);
      if (x < (uint32_t)kLbHotMax) {
        a.hl_key[x] = a.uniq[i];
        a.hl_len[x] = len;
      }
    }
  }
}

// the next batch's hot-key map from the list (one block): the hot keys sorted (bitonic, LDS),
// W_h = ceil(len_h / target) with target sized so the buckets needed, nbk / 2 coarse plus
// sum (W_h + 1), fit 2^wbits_hot; P (the exclusive prefix of W + 1); per coarse bucket its first
// hot key.  No list, a list past kLbHotMax, or no room: the key map next.  A batch that was
// skewed under the key map sends the next one to the bucket Localizer again (hint[0]).
__global__ __launch_bounds__(kLbHotMax) void k_lb_hotmap(LbArgs a) {
  __shared__ uint64_t sk[kLbHotMax];
  __shared__ uint32_t sl[kLbHotMax];
  __shared__ uint32_t lds[kLbHotMax / kWave + 1];
  DevState* ds = a.ds;
  const int t = threadIdx.x;
  const bool was = lb_hot_on(a);
  const uint32_t nh = (ds->lb_hot || was) ? ds->lb_nhot : 0u;  // (k_lb_hotlist's condition)
  if (t == 0 && was) ds->lb_map_steps += 1u;  // diagnostic: batches placed by the map
  const int wb = a.wbits_hot;
  const uint32_t nbk = 1u << wb, C = nbk / 2;
  if (nh == 0u || nh > (uint32_t)kLbHotMax || wb < 2 || 2 * nh >= nbk - C) {
    if (t == 0) {
      ds->lb_sp_use = 0u;
      a.hint[3] = 0u;
    }
    return;
  }
  sk[t] = (uint32_t)t < nh ? a.hl_key[t] : ~0ull;
  sl[t] = (uint32_t)t < nh ? a.hl_len[t] : 0u;
  __syncthreads();
  {  // sorted by key: a key's place is the count of smaller keys (keys are distinct; every
     // thread reads the same key at a time, an LDS broadcast)
    const uint64_t mk = sk[t];
    const uint32_t ml = sl[t];
    uint32_t r = 0;
    if ((uint32_t)t < nh)
      for (uint32_t i = 0; i < nh; ++i) r += sk[i] < mk ? 1u : 0u;
    __syncthreads();
    if ((uint32_t)t < nh) {
      sk[r] = mk;
      sl[r] = ml;
    }
    __syncthreads();
  }
  const uint32_t len = sl[t];
  uint32_t mass;
  (void)block_excl_scan<kLbHotMax>(len, lds, &mass);
  const uint32_t room = nbk - C - 2 * nh;  // sum W_h <= mass / target + nh <= nbk - C - nh
  const uint32_t target = (mass + room - 1) / room;
  const uint32_t W = (uint32_t)t < nh ? (len + target - 1) / target : 0u;
  uint32_t tot;
  const uint32_t P = block_excl_scan<kLbHotMax>((uint32_t)t < nh ? W + 1 : 0u, lds, &tot);
  if ((uint32_t)t < nh) {
    a.hm_key[t] = sk[t];
    a.hm_w[t] = W;
    a.hm_p[t] = P;
  }
  if (t == 0) a.hm_p[nh] = tot;
  // the coarse map: the key map's form over C buckets, fitted to this batch's key range (the
  // parameters travel with the map: the next batch's own fit may move)
  LbMap cm;
  cm.nbk = C;
  cm.base = ds->kmin;
  {
    const int bl = lb_bitlen(ds->kmax - ds->kmin), cb = wb - 1;
    cm.s = bl > cb ? bl - cb : 0;
  }
  for (uint32_t c = t; c <= C; c += kLbHotMax) {  // the first hot key of coarse bucket >= c
    uint32_t lo = 0, hi = nh;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (lb_bucket(sk[mid], cm) < c) lo = mid + 1;
      else hi = mid;
    }
    a.hm_ic[c] = lo;
  }
  if (t == 0) {
    ds->lb_hm_n = nh;
    ds->lb_hm_base = cm.base;
    ds->lb_hm_s = (unsigned)cm.s;
    ds->lb_sp_wbits = (unsigned)wb;
    ds->lb_sp_use = 1u;
    a.hint[3] = 1u;
    if (!was) a.hint[0] = 0u;
  }
}

// valued data (lb_gather=1): each occurrence's position (left in occ_row by the bucket kernel)
// replaced by its row and its value, one 8-byte {row, value} read per occurrence — one thread
// per occurrence, so the random reads are all in flight at once (inside the bucket kernel's
// slot loop each waited)
__global__ __launch_bounds__(kLbNT) void k_lb_gather(LbArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kLbNT + threadIdx.x;
  if (i >= a.nnz) return;
  const uint2 rv = a.rowof[a.occ_row[i]];  // one 8-byte read per occurrence
  a.occ_row[i] = rv.x;
  if (a.occ_x) a.occ_x[i] = __uint_as_float(rv.y);
}

// Workspace::lbsplit: the hot list and map, the buckets' first / last keys and continuations
static size_t lb_split_bytes() {
  constexpr size_t kNb = (size_t)1 << kLbMaxBits;
  return (size_t)kLbHotMax * 8 * 2 + kNb * 8 * 2 + (size_t)kLbHotMax * 4 * 3 + 4 + (kNb / 2 + 1) * 4 +
         kNb * 4;
}

// dynamic LDS past 64 KiB (the splitters at 8192 buckets): allowed once per kernel
static void lb_lds_attr(const void* f) {
  static std::mutex mu;
  static std::set<const void*> done;
  std::lock_guard<std::mutex> g(mu);
  if (!done.insert(f).second) return;
  hipFuncAttributes at{};
  if (hipFuncGetAttributes(&at, f) == hipSuccess)
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - (int)at.sharedSizeBytes);
  (void)hipGetLastError();  // a refusal leaves the default (64 KiB): no sticky error
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
  uint32_t nbk = 1u << wbits;
  // past ~3/4 of the LDS sort's capacity per bucket on average (beyond ~12.6 M nnz) most buckets
  // would be oversize: the radix Localizer outright, not a bucket pass that falls back
  if (nnz > (int64_t)nbk * (kLbCap * 3 / 4)) return DFX_OK;
  if (hint[2] == 0u) {
    // no batch seen on this workspace yet: seed the item form from what the host knows, so a
    // first batch whose items cannot pack (64-bit hashed ids, received keys) takes the LDS form
    // rather than sending every bucket through k_lb_big.  Varying key bits are at
    // most the bytes of max_index - 1 (ReverseBytes moves them, localizer.cc:24)
    int kb = 64;
    if (!o.keys_ready && max_index != ~0ull) {
      kb = 0;
      for (uint64_t m = max_index - 1; m; m >>= 8) kb += 8;
    }
    const uint64_t qmax = valued ? (uint64_t)(nnz - 1) : (uint64_t)(B - 1);
    int rb = 0;
    for (uint64_t q = qmax; q; q >>= 1) ++rb;
    hint[2] = kb + rb <= 63 ? 1u : 2u;
  }
  // the hot-key map (binary batches, after one that built it here): one more bucket bit, and
  // LDS for the map in the histogram / scatter launches (the device decides whether to use it;
  // without the LDS it keeps the key map).  Hot keys: runs of at least half a bucket's average
  // under the key map (and >= 64)
  const int hm_lds = (!valued && hint[3]) ? 1 : 0;
  const int wbits_key = wbits, wbits_hot = wbits + 1 < kLbMaxBits ? wbits + 1 : kLbMaxBits;
  if (hm_lds) {
    wbits = wbits_hot;
    nbk = 1u << wbits;
  }
  // at most kLbTiles row tiles (same-box A/B at C3: 256 -> 128 tiles 131.5 -> 132.9 M ex/s;
  // 64 / 32 lose: longer tiles stretch the lane into the next forward)
  constexpr int64_t kLbTiles = 128;
  int64_t ntiles = std::min<int64_t>(kLbTiles, std::max<int64_t>(1, nnz / 4096));
  int64_t rt = std::min<int64_t>(kLbMaxRows, std::max<int64_t>(1, (B + ntiles - 1) / ntiles));
  ntiles = (B + rt - 1) / rt;
  DFX_TRY(ws.keys0.ensure(nnz * 8));
  DFX_TRY(ws.keys1.ensure(nnz * 8));
  DFX_TRY(ws.vals0.ensure(nnz * 8));
  DFX_TRY(ws.vals1.ensure(nnz * 8));
  DFX_TRY(ws.lbq.ensure(nnz * 8));
  DFX_TRY(ws.lbcnt.ensure(sizeof(uint32_t) * ((size_t)ntiles * nbk + 4 * (nbk + 1))));
  DFX_TRY(ws.lbsplit.ensure(lb_split_bytes()));  // the hot-key map persists across batches
  LbArgs a{};
  a.B = B; a.nnz = nnz; a.offset = offset; a.index = index; a.max_index = max_index;
  a.keys_ready = o.keys_ready ? 1 : 0;
  a.value = valued ? o.value : nullptr;
  a.rt = rt; a.ntiles = ntiles; a.wbits = wbits;
  a.nt = (c->nt_mask & kNtLane) ? 1 : 0;
  a.tilecnt = ws.lbcnt.as<uint32_t>();
  a.totals = a.tilecnt + (size_t)ntiles * nbk;
  a.bstart = a.totals + nbk + 1;
  a.bheads = a.bstart + nbk + 1;
  a.brank = a.bheads + nbk + 1;
  a.kbuf = ws.keys0.as<uint64_t>();
  a.kscr = ws.keys1.as<uint64_t>();
  a.sbuf = ws.vals0.as<uint64_t>();
  // valued data: each position's row written in input order, the row and value gathered by
  // position at the outputs (lb_gather=1), or {value, row} carried beside each item (0)
  const bool gather = valued && c->lb_gather;
  a.rowof = gather ? ws.vals0.as<uint2>() : nullptr;
  a.sscr = ws.vals1.as<uint64_t>();
  a.qbuf = ws.lbq.as<uint32_t>();
  a.qscr = a.qbuf + nnz;
  a.ds = L.ds;
  a.uniq = o.uniq; a.segstart = o.segstart; a.occ_row = o.occ_row;
  a.occ_x = valued ? o.occ_x : nullptr;
  a.hint = ws.lb_hint;
  a.diag = (c->lb_diag & ~(16 | 32 | 64 | 128 | 256 | 512)) | c->lb_skip;
  {
    constexpr size_t kNb = (size_t)1 << kLbMaxBits;
    char* q = ws.lbsplit.as<char>();
    a.hl_key = reinterpret_cast<uint64_t*>(q);
    a.hm_key = a.hl_key + kLbHotMax;
    a.bfk = a.hm_key + kLbHotMax;
    a.blk = a.bfk + kNb;
    a.hl_len = reinterpret_cast<uint32_t*>(a.blk + kNb);
    a.hm_p = a.hl_len + kLbHotMax;
    a.hm_w = a.hm_p + kLbHotMax + 1;
    a.hm_ic = a.hm_w + kLbHotMax;
    a.bcont = a.hm_ic + kNb / 2 + 1;
  }
  a.hm_lds = hm_lds;
  a.wbits_hot = wbits_hot;
  a.hot_th = (uint32_t)std::max<int64_t>(
      kWave, std::min<int64_t>(nnz / ((int64_t)1 << wbits_key) / 2, kLbCap));
  const size_t sp_bytes = a.hm_lds ? lb_hot_lds(nbk) : 0;
  hipLaunchKernelGGL(k_lb_init, dim3(1), dim3(1), 0, L.stream, L.ds);
#define DFX_LB_HIST(NT)                                                                     \
  if (a.hm_lds) {                                                                           \
    lb_lds_attr((const void*)k_lb_hist<NT, true>);                                          \
    hipLaunchKernelGGL((k_lb_hist<NT, true>), dim3((unsigned)ntiles), dim3(NT),             \
                       nbk * sizeof(uint32_t) + sp_bytes, L.stream, a);                     \
  } else {                                                                                  \
    hipLaunchKernelGGL((k_lb_hist<NT, false>), dim3((unsigned)ntiles), dim3(NT),            \
                       nbk * sizeof(uint32_t), L.stream, a);                                \
  }
  // lb_hnt (0: auto): 512-thread blocks for valued batches, whose scatter also writes the
  // {row, value} pairs (C2 +5.6 %), 1024 for binary ones (C3: 1024 best)
  const int hnt = c->lb_hnt ? c->lb_hnt : (valued ? 512 : 1024);
  if (hnt == 256) { DFX_LB_HIST(256) }
  else if (hnt == 512) { DFX_LB_HIST(512) }
  else { DFX_LB_HIST(1024) }
#undef DFX_LB_HIST
  hipLaunchKernelGGL(k_lb_colscan, dim3((nbk + kWave - 1) / kWave), dim3(kLbScanWaves * kWave), 0,
                     L.stream, a);
  const size_t scatter_lds =
      ((nbk + 1) & ~1u) * sizeof(uint32_t) + (rt + 1) * sizeof(uint64_t) + sp_bytes;
#define DFX_LB_SCAT(NT)                                                                    \
  lb_lds_attr((const void*)k_lb_scatter<true, NT, false>);                                 \
  lb_lds_attr((const void*)k_lb_scatter<false, NT, false>);                                \
  lb_lds_attr((const void*)k_lb_scatter<false, NT, true>);                                 \
  if (valued)                                                                              \
    hipLaunchKernelGGL((k_lb_scatter<true, NT, false>), dim3((unsigned)ntiles), dim3(NT),   \
                       scatter_lds, L.stream, a);                                          \
  else if (a.hm_lds)                                                                       \
    hipLaunchKernelGGL((k_lb_scatter<false, NT, true>), dim3((unsigned)ntiles), dim3(NT),   \
                       scatter_lds, L.stream, a);                                          \
  else                                                                                     \
    hipLaunchKernelGGL((k_lb_scatter<false, NT, false>), dim3((unsigned)ntiles), dim3(NT),  \
                       scatter_lds, L.stream, a);
  if (c->lb_skip & 16) {}  // (measurement only)
  else if (hnt == 256) { DFX_LB_SCAT(256) }
  else if (hnt == 512) { DFX_LB_SCAT(512) }
  else { DFX_LB_SCAT(1024) }
#undef DFX_LB_SCAT
  // the LDS form of the per-bucket sort follows the last batch's item form (a batch whose items
  // do not pack while the launch expected packed ones sorts through global memory: correct)
  const bool q_lds = hint[2] == 2u;
  const dim3 bg(nbk), bb(kLbNT);
  const bool carry = valued && !gather;  // side payloads through the sort
  if (carry)
    hipLaunchKernelGGL(k_lb_big<true>, dim3(kLbBigBlocks), bb, 0, L.stream, a, q_lds ? 1 : 0);
  else
    hipLaunchKernelGGL(k_lb_big<false>, dim3(kLbBigBlocks), bb, 0, L.stream, a, q_lds ? 1 : 0);
  const dim3 wb(kWave);  // one wave per bucket
  if (c->lb_skip & 32) {}  // (measurement only)
  else if (carry) {
    if (q_lds) hipLaunchKernelGGL((k_lb_wbucket<true, true>), bg, wb, 0, L.stream, a);
    else hipLaunchKernelGGL((k_lb_wbucket<false, true>), bg, wb, 0, L.stream, a);
  } else {
    if (q_lds) hipLaunchKernelGGL((k_lb_wbucket<true, false>), bg, wb, 0, L.stream, a);
    else hipLaunchKernelGGL((k_lb_wbucket<false, false>), bg, wb, 0, L.stream, a);
  }
  // (lb_gather=2, the fused step) the backward reads {row, value} by position itself
  const bool defer = gather && c->lb_gather == 2 && o.rowof_out != nullptr;
  if (o.rowof_out) *o.rowof_out = defer ? a.rowof : nullptr;
  if (gather && !defer && nnz > 0)
    hipLaunchKernelGGL(k_lb_gather, dim3((unsigned)((nnz + kLbNT - 1) / kLbNT)), bb, 0, L.stream,
                       a);
  hipLaunchKernelGGL(k_lb_bscan, dim3(1), dim3(kLbScanNT), 0, L.stream, a);
  if (!(c->lb_skip & 64)) hipLaunchKernelGGL(k_lb_out, bg, bb, 0, L.stream, a);
  if (!valued && a.uniq && a.segstart) {  // the next batch's hot-key map
    hipLaunchKernelGGL(k_lb_hotlist, dim3(kLbHotGrid), bb, 0, L.stream, a);
    hipLaunchKernelGGL(k_lb_hotmap, dim3(1), dim3(kLbHotMax), 0, L.stream, a);
  }
  DFX_HIP(hipGetLastError());
  *used = true;
  return DFX_OK;
}

}  // namespace dfx
