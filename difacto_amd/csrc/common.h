// Device helpers shared by the gfx950 kernels: wave64 scans, key scrambling, the device
// hash table view, glibc rand_r restated as an LCG with jump-ahead.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfx {

constexpr int kWave = 64;

// Loads / stores with the streaming (non-temporal) cache policy when nt is set: traffic that
// is touched once per step (the Localizer's sort passes, the model table's random lines) need
// not displace what is re-read within the step from the Infinity Cache / L2 (the [XV*p | p]
// rows the backward reads once per occurrence).  Context kwarg nt (a mask, store.hip).
typedef float dfx_f4v __attribute__((ext_vector_type(4)));
typedef float dfx_f2v __attribute__((ext_vector_type(2)));
__device__ inline float4 ld4(const float* p, bool nt) {
  if (nt) {
    const dfx_f4v v = __builtin_nontemporal_load(reinterpret_cast<const dfx_f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return *reinterpret_cast<const float4*>(p);
}
__device__ inline float2 ld2(const float* p, bool nt) {
  if (nt) {
    const dfx_f2v v = __builtin_nontemporal_load(reinterpret_cast<const dfx_f2v*>(p));
    return make_float2(v.x, v.y);
  }
  return *reinterpret_cast<const float2*>(p);
}
__device__ inline void st4(float* p, float4 v, bool nt) {
  if (nt) {
    const dfx_f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<dfx_f4v*>(p));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
template <typename T>
__device__ inline T ldnt(const T* p, bool nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T>
__device__ inline void stnt(T* p, T v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// the context kwarg nt's bits
constexpr int kNtLane = 1, kNtBwdTable = 2, kNtFwdTable = 4, kNtBwdOcc = 8;
constexpr uint64_t kEmptyKey = ~0ull;  // never produced by the Localizer
// the slot of a key whose insert failed (table full, or the reserved key ~0): every consumer
// skips it — no update ever lands in another key's entry
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// include/difacto/base.h:39-51 — nibble reversal (involution).
__host__ __device__ inline uint64_t reverse_bytes(uint64_t x) {
  x = x << 32 | x >> 32;
  x = (x & 0x0000FFFF0000FFFFull) << 16 | (x & 0xFFFF0000FFFF0000ull) >> 16;
  x = (x & 0x00FF00FF00FF00FFull) << 8 | (x & 0xFF00FF00FF00FF00ull) >> 8;
  x = (x & 0x0F0F0F0F0F0F0F0Full) << 4 | (x & 0xF0F0F0F0F0F0F0F0ull) >> 4;
  return x;
}

__device__ inline int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ inline uint64_t lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// inclusive scan over the 64 lanes of a wave
__device__ inline uint32_t wave_incl_scan(uint32_t v) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    uint32_t t = __shfl_up(v, off, kWave);
    if (l >= off) v += t;
  }
  return v;
}

// exclusive scan over a block of NT threads; lds needs NT/64 + 1 words.
template <int NT>
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
  constexpr int NW = NT / kWave;
  const int w = threadIdx.x / kWave;
  uint32_t inc = wave_incl_scan(v);
  if (lane_id() == kWave - 1) lds[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int i = 0; i < NW; ++i) { uint32_t t = lds[i]; lds[i] = run; run += t; }
    lds[NW] = run;
  }
  __syncthreads();
  uint32_t r = lds[w] + inc - v;
  if (total) *total = lds[NW];
  __syncthreads();
  return r;
}

// ---- glibc rand_r (stdlib/rand_r.c): three LCG steps per call ------------------------
constexpr uint32_t kLcgA = 1103515245u, kLcgC = 12345u;

// (A, C) such that stepping the LCG m times maps s -> A*s + C (mod 2^32).
__host__ __device__ inline void lcg_jump(uint64_t m, uint32_t* A, uint32_t* C) {
  uint32_t ra = 1, rc = 0, ca = kLcgA, cc = kLcgC;
  while (m) {
    if (m & 1) { ra = ca * ra; rc = ca * rc + cc; }
    cc = ca * cc + cc;
    ca = ca * ca;
    m >>= 1;
  }
  *A = ra; *C = rc;
}

__host__ __device__ inline uint32_t lcg_advance(uint32_t s, uint64_t steps) {
  uint32_t A, C;
  lcg_jump(steps, &A, &C);
  return A * s + C;
}

__host__ __device__ inline int rand_r_dev(uint32_t* seed) {
  uint32_t next = *seed;
  int result;
  next = next * kLcgA + kLcgC;
  result = (int)((next >> 16) % 2048u);
  next = next * kLcgA + kLcgC;
  result = (int)(((uint32_t)result << 10) ^ ((next >> 16) % 1024u));
  next = next * kLcgA + kLcgC;
  result = (int)(((uint32_t)result << 10) ^ ((next >> 16) % 1024u));
  *seed = next;
  return result;
}

// InitV's draw (sgd_updater.cc:148): (float)(((float)r / (float)RAND_MAX - 0.5) * scale)
__host__ __device__ inline float initv_value(int r, float scale) {
  float q = (float)r / 2147483648.0f;  // (real_t)RAND_MAX == 2^31 in float
  return (float)(((double)q - 0.5) * (double)scale);
}

// InitV's rows a coordinate per thread: row i of a block's list starts at LCG state st[i]
// (3·d·rank steps past the seed) and its coordinate j is the rand_r draw 3·j steps further,
// (A[j], C[j]) = lcg_jump(3·j) — the values one thread walking the row would draw.  vrow
// 0xFFFFFFFF: skipped (pool full).  Callers: store.hip k_initv / k_initv_onepass, dist.hip
// k_dist_initv_sum.
constexpr int kIvMaxD = 256;  // up to this V_dim; wider rows are drawn a row per thread
template <int NT, class RowV, class RowC>
__device__ inline void initv_draw_list(uint32_t n, const uint32_t* st, const uint32_t* vrow,
                                       int d, float scale, const uint32_t* A, const uint32_t* C,
                                       RowV row_v, RowC row_c) {
  const uint32_t npairs = n * (uint32_t)d;
  for (uint32_t q = threadIdx.x; q < npairs; q += NT) {
    const uint32_t i = q / (uint32_t)d, j = q - i * (uint32_t)d;
    const uint32_t vr = vrow[i];
    if (vr == 0xFFFFFFFFu) continue;
    uint32_t s = A[j] * st[i] + C[j];
    row_v(vr)[j] = initv_value(rand_r_dev(&s), scale);
    row_c(vr)[j] = 0.f;
  }
}

// ---- device hash table (open addressing, linear probing) -----------------------------
// One 32-byte entry per key (SGDEntry, sgd_updater.h:20-34): the probe that finds the key
// brings the FTRL state and the V-pool row in the same cache line.
// {w, vrow} lead so the forward pass reads both with one 8-byte load.
struct __attribute__((aligned(32))) Entry {
  float w;
  int32_t vrow;                 // V pool row, -1 == no V (SGDEntry::V == nullptr)
  float sqrt_g, z;
  float fea_cnt;
  uint32_t pad;
  unsigned long long key;       // kEmptyKey == free slot
};
static_assert(sizeof(Entry) == 32, "Entry must be 32 bytes");

struct Table {
  Entry* ent;       // cap slots of 32 << es bytes, the entry first
  float* V;         // split layout (es == 0): vcap rows of [V(d) | Vaux(d)] — a key's embedding
                    // and its AdaGrad accumulators share one 2*d*4-byte row (one 128-byte line
                    // at d = 16); fat slots (es > 0): cap rows of Vaux(d), row = slot
  uint64_t mask;    // cap - 1
  int logcap;
  int d;
  int64_t vcap;
  int ordered;      // home slot = top bits of the key (see tbl_hash)
  int* probe_flag;  // device word: set when an insert probed past kClusterProbe slots
  // ordered hash of a key-range server: the table holds the keys of one of range_mul equal
  // ranges of the key space (dist.hip, owner(k) = floor(k * N / 2^64)), whose top bits are
  // constant; k * range_mul (mod 2^64) is the key's position inside its range, monotone in k
  uint64_t range_mul;
  // slot stride: 32 << es bytes.  es = 0: the split layout (32-byte entries, V rows in the pool,
  // vrow = pool row).  es = 1 / 2 (fat slots, 64 / 128 bytes, 4 <= d <= 24): the slot holds the
  // entry and then the key's V, so the forward's lookup and its V read are one line; Vaux
  // stays in the pool, one d-float row per slot; a key's vrow is its own slot (InitV sets it,
  // a rehash moves the row with the slot)
  int es;
};

__host__ __device__ inline Entry* ent_at(const Table& t, int64_t s) { return t.ent + (s << t.es); }

__host__ __device__ inline float* row_V(const Table& t, int64_t vr) {
  return t.es ? reinterpret_cast<float*>(t.ent + (vr << t.es) + 1) : t.V + vr * 2 * (int64_t)t.d;
}
__host__ __device__ inline float* row_C(const Table& t, int64_t vr) {
  return t.es ? t.V + vr * (int64_t)t.d : t.V + vr * 2 * (int64_t)t.d + t.d;
}

// the V row InitV gives a key: the q-th new row of this Update in the split layout (rows are
// allocated in key order), the key's own slot with fat slots
__host__ __device__ inline int64_t initv_row(const Table& t, uint64_t n_vrows, int64_t q,
                                             uint32_t slot) {
  return t.es ? (int64_t)slot : (int64_t)n_vrows + q;
}

// fat slot stride for V_dim d (0: the split layout): the entry and V in 64 or 128 bytes
__host__ __device__ inline int fat_es(int d) {
  if (d < 4 || d % 4 != 0 || 32 + 4 * d > 128) return 0;
  return 32 + 4 * d <= 64 ? 1 : 2;
}

__device__ inline float4 ent_state(const Entry* e) {
  const float4 a = *reinterpret_cast<const float4*>(e);  // w, vrow, sqrt_g, z
  return make_float4(a.x, a.z, a.w, e->fea_cnt);          // {w, sqrt_g, z, fea_cnt}
}
// a gradient update's write-back: {w, vrow, sqrt_g, z} as one 16-byte store (fea_cnt does not
// change in Update(kGradient); vrow is written back as read — InitV sets it later, in order)
__device__ inline void ent_store_hot(Entry* e, float4 s, int vrow, bool nt = false) {
  st4(reinterpret_cast<float*>(e), make_float4(s.x, __int_as_float(vrow), s.y, s.z), nt);
}

// writes back {w, sqrt_g, z, fea_cnt}; vrow is untouched
__device__ inline void ent_set_state(Entry* e, float4 s) {
  e->w = s.x;
  e->sqrt_g = s.y;
  e->z = s.z;
  e->fea_cnt = s.w;
}

// Home slot of a key.  Ordered (the default): the top logcap bits of the key itself.  Keys
// are nibble-reversed feature ids, uniform in their top bits for hashed or dense ids, so
// the table stays collision-light, and the key-sorted walks of the backward and the pull
// touch table lines in address order (sorted random access runs ~1.35x the rate of
// unsorted on MI355X, tools/membench).  When keys cluster in their top bits, an insert
// that probes past kClusterProbe slots raises probe_flag and the store rehashes with the
// multiplicative hash at the next sync point (store.hip: table_unclump).
constexpr int kClusterProbe = 64;
__host__ __device__ inline uint64_t tbl_hash(uint64_t k, const Table& t) {
  return t.ordered ? ((k * t.range_mul) >> (64 - t.logcap))
                   : ((k * 0x9E3779B97F4A7C15ull) >> (64 - t.logcap));
}

__device__ inline int64_t tbl_find(const Table& t, uint64_t k) {
  if (k == kEmptyKey) return -1;  // the reserved key is never stored
  uint64_t h = tbl_hash(k, t);
  for (uint64_t probe = 0; probe <= t.mask; ++probe) {
    uint64_t kk = ent_at(t, h)->key;
    if (kk == k) return (int64_t)h;
    if (kk == kEmptyKey) return -1;
    h = (h + 1) & t.mask;
  }
  return -1;
}

// find-or-insert; -1 when the table is full, -2 for the reserved key kEmptyKey (it marks free
// slots, so it cannot be stored: the raw-key store calls reject it, the Localizer never makes
// it).  Concurrent inserts of one key are safe (the CAS loser finds the winner's slot).
// Fresh slots already hold zero state and vrow -1 (the table is never compacted), which is
// what `model_[key]` default-constructs (sgd_updater.h:20-34).
__device__ inline int64_t tbl_insert(const Table& t, uint64_t k, bool* inserted) {
  *inserted = false;
  if (k == kEmptyKey) return -2;
  uint64_t h = tbl_hash(k, t);
  for (uint64_t probe = 0; probe <= t.mask; ++probe) {
    uint64_t kk = ent_at(t, h)->key;
    if (kk == k) return (int64_t)h;
    if (kk == kEmptyKey) {
      unsigned long long old = atomicCAS(&ent_at(t, h)->key, (unsigned long long)kEmptyKey,
                                         (unsigned long long)k);
      if (old == kEmptyKey) {
        *inserted = true;
        if (probe > (uint64_t)kClusterProbe && t.probe_flag) atomicOr(t.probe_flag, 1);
        return (int64_t)h;
      }
      if (old == k) return (int64_t)h;
    }
    h = (h + 1) & t.mask;
  }
  return -1;
}

// device-side error word bits (checked at dfx_sync)
enum : int {
  kErrTableFull = 1,
  kErrPoolFull = 2,
  kErrLens = 4,
  kErrNoV = 8,
  kErrSort = 16,
  kErrBadKey = 32,
};

// the error bit of a failed tbl_insert
__device__ inline int insert_error(int64_t s) { return s == -2 ? kErrBadKey : kErrTableFull; }

struct Params {
  float l1, l2, V_l2, lr, lr_beta, V_lr, V_lr_beta, V_init_scale;
  int V_dim, V_threshold;
  int l1_shrk;
};

// SGDUpdater::UpdateW (sgd_updater.cc:105-131), exact float expression order.
// Returns +1 / -1 / 0 for the new_w statistic; *transition is set on a 0 -> nonzero move.
__device__ inline int ftrl_update(const Params& P, float gw, float4* e, bool* transition) {
  float sg = e->y;
  float w = e->x;
  gw += w * P.l2;
  float nsg = sqrtf(sg * sg + gw * gw);
  e->y = nsg;
  e->z -= gw - (nsg - sg) / P.lr * w;
  float z = e->z;
  float l1 = P.l1;
  if (z <= l1 && z >= -l1) {
    e->x = 0;
  } else {
    float eta = (P.lr_beta + nsg) / P.lr;
    e->x = (z > 0 ? z - l1 : z + l1) / eta;
  }
  *transition = false;
  if (w == 0 && e->x != 0) { *transition = true; return 1; }
  if (w != 0 && e->x == 0) return -1;
  return 0;
}

// SGDUpdater::UpdateV (sgd_updater.cc:133-142) for one coordinate.
__device__ inline void adagrad_update(const Params& P, float gV, float* v, float* cg) {
  float g = gV + P.V_l2 * (*v);
  float c = *cg;
  float nc = sqrtf(c * c + g * g);
  *cg = nc;
  float eta = P.V_lr / (nc + P.V_lr_beta);
  *v -= eta * g;
}

__host__ __device__ inline int next_pow2_lanes(int d) {
  int g = 1;
  while (g < d && g < 64) g <<= 1;
  return g;
}

}  // namespace dfx
