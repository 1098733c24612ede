// The device model store: SGDUpdater (src/sgd/sgd_updater.{h,cc}) behind the Store
// push/pull boundary (include/difacto/store.h:44-75), on one GPU.
//
// Layout in HBM (sized for 288 GB):
//   ent   Entry[cap]    32-byte records {w, sqrt_g, z, fea_cnt | key | vrow}: SGDEntry
//                       (sgd_updater.h:20-34) + its key, open addressing with a
//                       multiplicative hash of the (already nibble-reversed) key and linear
//                       probing, cap = pow2 >= 2*max_keys.  A probe's cache line carries the
//                       key's whole scalar state.
//   V     f32[vcap*2d]  rows of [V(d) | Vaux(d)] (embedding + AdaGrad accumulators in one
//                       row: one 128-byte line per key at V_dim 16), allocated by InitV
// InitV (sgd_updater.cc:144-152) draws glibc rand_r in key order; on the GPU every key that
// needs V gets its exclusive-scan rank r among this push's InitV keys and jumps the LCG by
// 3*V_dim*r steps, which reproduces the reference's sequential draws exactly.
#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <sstream>
#include <vector>

#include <chrono>

#include "lookback.h"

namespace dfx {

constexpr int kStNT = 256;

__device__ inline void block_count_add(int v, unsigned long long* dst) {
  __shared__ int red[kStNT / kWave];
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < kStNT / kWave; ++i) s += red[i];
    if (s) atomicAdd(dst, (unsigned long long)(long long)s);
  }
  __syncthreads();
}

__device__ inline int64_t count_of(int64_t n_host, const DevState* ds) {
  return n_host >= 0 ? n_host : (int64_t)ds->u_count;
}

// ---- InitV --------------------------------------------------------------------------------
// excl: exclusive scan of the per-key InitV flags; *total: their sum; slot: table slot of
// each flagged key.
__global__ __launch_bounds__(kStNT) void k_initv(int64_t n_host, const uint32_t* excl,
                                                 const uint32_t* total, const uint32_t* slot,
                                                 Table T, float scale, DevState* ds,
                                                 const DevState* nds, const uint32_t* gate) {
  if (gate && *gate == 0u) return;
  const int64_t n = count_of(n_host, nds);
  const int d = T.d;
  if (d > kIvMaxD) {  // (wide V: a row per thread)
    // strided over a grid capped like a gated scan's (run_initv)
    for (int64_t u = (int64_t)blockIdx.x * kStNT + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * kStNT) {
      const uint32_t e = excl[u];
      const uint32_t nx = (u + 1 < n) ? excl[u + 1] : *total;
      if (nx == e) continue;
      uint32_t s = lcg_advance(ds->seed, 3ull * (uint64_t)d * e);
      const int64_t vr = initv_row(T, ds->n_vrows, e, slot[u]);
      if (vr >= T.vcap) {
        atomicOr(&ds->err, kErrPoolFull);
        continue;
      }
      float* V = row_V(T, vr);
      float* C = row_C(T, vr);
      for (int k = 0; k < d; ++k) {
        V[k] = initv_value(rand_r_dev(&s), scale);
        C[k] = 0.f;
      }
      ent_at(T, slot[u])->vrow = (int32_t)vr;
    }
    return;
  }
  // per kStNT keys: the flagged ones listed (a block scan), then drawn a coordinate per thread
  __shared__ uint32_t s_st[kStNT], s_vr[kStNT], s_A[kIvMaxD], s_C[kIvMaxD];
  __shared__ uint32_t lds[kStNT / kWave + 1];
  for (int j = threadIdx.x; j < d; j += kStNT) lcg_jump(3ull * (uint64_t)j, &s_A[j], &s_C[j]);
  for (int64_t b0 = (int64_t)blockIdx.x * kStNT; b0 < n; b0 += (int64_t)gridDim.x * kStNT) {
    const int64_t u = b0 + threadIdx.x;
    uint32_t e = 0;
    bool f = false;
    if (u < n) {
      e = excl[u];
      f = ((u + 1 < n) ? excl[u + 1] : *total) != e;
    }
    uint32_t cnt;
    const uint32_t at = block_excl_scan<kStNT>(f ? 1u : 0u, lds, &cnt);
    if (f) {
      const int64_t vr = initv_row(T, ds->n_vrows, e, slot[u]);
      s_st[at] = lcg_advance(ds->seed, 3ull * (uint64_t)d * e);
      if (vr >= T.vcap) {
        atomicOr(&ds->err, kErrPoolFull);
        s_vr[at] = 0xFFFFFFFFu;
      } else {
        s_vr[at] = (uint32_t)vr;
        ent_at(T, slot[u])->vrow = (int32_t)vr;
      }
    }
    __syncthreads();
    initv_draw_list<kStNT>(cnt, s_st, s_vr, d, scale, s_A, s_C,
                           [&](uint32_t r) { return row_V(T, r); },
                           [&](uint32_t r) { return row_C(T, r); });
    __syncthreads();
  }
}

__global__ void k_initv_finalize(const uint32_t* total, int d, int64_t vcap, DevState* ds) {
  const uint32_t n = *total;
  ds->seed = lcg_advance(ds->seed, 3ull * (uint64_t)d * n);
  unsigned long long nv = ds->n_vrows + n;
  ds->n_vrows = nv > (unsigned long long)vcap ? (unsigned long long)vcap : nv;
}

// The fused step's InitV in ONE launch (it replaced the scan's three launches + k_initv: in the
// steady state, where no key needs V, all four only found the device gate closed).  Block b
// counts tile b's kIvTile flags, publishes the count and finds its prefix by the block-wide
// decoupled look-back over the lower tiles' tagged words (lookback.h), then draws its keys' V
// exactly as k_initv.
// The last tile writes the total; with fin.ds set the step's last work follows in this launch
// (step_finalize_body: the seed and n_vrows advanced by the total, the progress, the capacity
// guard's counts) — by block 0 when the gate is closed, else by the last block to finish, one
// launch less per step (round 6).
// 8192-key tiles (a thread's 32 flags as one bit mask), the requested keys listed kIvList at a
// time: 4096-key tiles took 850 tickets at C3, ~9 us of serialised atomics.
constexpr int kIvItems = 32, kIvTile = kStNT * kIvItems, kIvList = 4096;

static_assert(kStNT == kFinNT, "the fused InitV's blocks run the step's finalize");

__device__ void initv_onepass_body(const uint32_t* flags, uint32_t* total, const uint32_t* slot,
                                   const Table& T, float scale, DevState* ds, const DevState* nds,
                                   unsigned long long* status, int64_t n, uint32_t need);

__global__ __launch_bounds__(kStNT) void k_initv_onepass(const uint32_t* flags, uint32_t* total,
                                                         const uint32_t* slot, Table T,
                                                         float scale, DevState* ds,
                                                         const DevState* nds,
                                                         const uint32_t* gate,
                                                         unsigned long long* status, FinArgs fin) {
  __shared__ double s_red[kFinNT / kWave];
  __shared__ bool s_last;
  const int64_t n = (int64_t)nds->u_count;
  const uint32_t need = (uint32_t)((n + kIvTile - 1) / kIvTile);
  if (*gate == 0u || need == 0) {  // nothing to draw: block 0 finalizes
    if (blockIdx.x != 0) return;
    if (threadIdx.x == 0)
      __hip_atomic_store(total, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (fin.ds) {
      __syncthreads();
      step_finalize_body<kFinNT>(fin, s_red);
    }
    return;
  }
  if (blockIdx.x >= need) return;
  initv_onepass_body(flags, total, slot, T, scale, ds, nds, status, n, need);
  if (!fin.ds) return;
  // every block that took a tile counts itself done; the last one finalizes the step (its
  // draws read ds->seed / n_vrows, which the finalize advances).  No fence: the finalize reads
  // nothing this launch wrote but the total (an agent-scope store and load), and a device-scope
  // fence per block writes its XCD's L2 back — here full of the backward's dirty model lines
  // (measured: with the fences C3 lost 2.7 % in every step that drew a V row)
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&ds->iv_done, 1u) == need - 1;
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) __hip_atomic_store(&ds->iv_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  step_finalize_body<kFinNT>(fin, s_red);
}

__device__ void initv_onepass_body(const uint32_t* flags, uint32_t* total, const uint32_t* slot,
                                   const Table& T, float scale, DevState* ds, const DevState* nds,
                                   unsigned long long* status, int64_t n, uint32_t need) {
  __shared__ uint32_t lds[kStNT / kWave + 1];
  __shared__ uint32_t s_lb[3 * kStNT / kWave];
  // tile by ticket, in the order blocks start: a block only waits on running ones.  Block index
  // order is not start order across XCDs, and the AUC lane's look-back sort can run beside this
  // kernel, so tile = block index could wait on a block that cannot be placed.  The
  // block that draws the last ticket zeroes the counter for the next launch (k_step_finalize
  // zeroes it too).  Only as many blocks as the batch has tiles draw one: the grid is sized for
  // the nnz bound, and each ticket is a returning atomic on one word, ~11 ns apiece serialised
  // (DESIGN.md (d)); the blocks past the count leave at once, and the tickets still go to running
  // blocks in start order.
  __shared__ uint32_t s_tile;
  if (threadIdx.x == 0) {
    s_tile = atomicAdd(&ds->iv_ticket, 1u);
    if (s_tile == need - 1)
      __hip_atomic_store(&ds->iv_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t base = tile * kIvTile;
  const uint32_t tag = ds->iv_epoch & 0x3FFFFFFFu;
  // this thread's kIvItems consecutive flags (0 / 1) as bits
  const int64_t i0 = base + (int64_t)threadIdx.x * kIvItems;
  uint32_t mask = 0;
  if (i0 + kIvItems <= n && ((uintptr_t)flags & 15u) == 0) {
    const uint4* f4 = reinterpret_cast<const uint4*>(flags + i0);
#pragma unroll
    for (int q = 0; q < kIvItems / 4; ++q) {
      const uint4 v = f4[q];
      mask |= ((v.x ? 1u : 0u) | (v.y ? 2u : 0u) | (v.z ? 4u : 0u) | (v.w ? 8u : 0u)) << (4 * q);
    }
  } else {
#pragma unroll 4
    for (int k = 0; k < kIvItems; ++k)
      if (i0 + k < n && flags[i0 + k]) mask |= 1u << k;
  }
  const uint32_t cnt = (uint32_t)__popc(mask);
  uint32_t tot;
  const uint32_t ex = block_excl_scan<kStNT>(cnt, lds, &tot);
  const uint32_t pre = block_lookback<kStNT>(status, tile, tag, tot, &ds->err, s_lb);
  if (threadIdx.x == 0 && base + kIvTile >= n)  // the last tile
    __hip_atomic_store(total, pre + tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tot == 0) return;  // block-uniform
  const int d = T.d;
  if (d > kIvMaxD) {  // (wide V: each thread draws its keys' rows in turn)
    uint32_t e = pre + ex;
    for (uint32_t m = mask; m; m &= m - 1) {
      const int64_t u = i0 + (__ffs(m) - 1);
      uint32_t s = lcg_advance(ds->seed, 3ull * (uint64_t)d * e);
      const int64_t vr = initv_row(T, ds->n_vrows, e, slot[u]);
      ++e;
      if (vr >= T.vcap) {
        atomicOr(&ds->err, kErrPoolFull);
        continue;
      }
      float* V = row_V(T, vr);
      float* C = row_C(T, vr);
      for (int q = 0; q < d; ++q) {
        V[q] = initv_value(rand_r_dev(&s), scale);
        C[q] = 0.f;
      }
      ent_at(T, slot[u])->vrow = (int32_t)vr;
    }
    return;
  }
  // the block's requested keys, kIvList at a time, each with its V row and the LCG state at its
  // first draw (3·d·rank steps past the seed, sgd_updater.cc:118-121), then every (key,
  // coordinate) drawn by its own thread: coordinate j's state is 3·j steps on (A_j·state + C_j),
  // the same rand_r values as one thread walking the row — a row's d draws were one lane's d · 3
  // dependent LCG steps (C5: ~0.1 ms of the step with ~1.5 k requests per 4096-key tile)
  __shared__ uint32_t s_st[kIvList], s_vr[kIvList];
  __shared__ uint32_t s_A[kIvMaxD], s_C[kIvMaxD];
  for (int j = threadIdx.x; j < d; j += kStNT) lcg_jump(3ull * (uint64_t)j, &s_A[j], &s_C[j]);
  for (uint32_t q0 = 0; q0 < tot; q0 += kIvList) {
    if (ex < q0 + kIvList && ex + cnt > q0) {
      uint32_t idx = ex;
      for (uint32_t m = mask; m; m &= m - 1, ++idx) {
        if (idx < q0) continue;
        if (idx >= q0 + kIvList) break;
        const int64_t u = i0 + (__ffs(m) - 1);
        const uint32_t e = pre + idx;
        const int64_t vr = initv_row(T, ds->n_vrows, e, slot[u]);
        s_st[idx - q0] = lcg_advance(ds->seed, 3ull * (uint64_t)d * e);
        if (vr >= T.vcap) {
          atomicOr(&ds->err, kErrPoolFull);
          s_vr[idx - q0] = 0xFFFFFFFFu;
        } else {
          s_vr[idx - q0] = (uint32_t)vr;
          ent_at(T, slot[u])->vrow = (int32_t)vr;
        }
      }
    }
    __syncthreads();
    initv_draw_list<kStNT>(tot - q0 < (uint32_t)kIvList ? tot - q0 : (uint32_t)kIvList, s_st, s_vr,
                           d, scale, s_A, s_C, [&](uint32_t r) { return row_V(T, r); },
                           [&](uint32_t r) { return row_C(T, r); });
    __syncthreads();
  }
}

// flags[0..n) -> InitV.  flags is scanned in place; total_dev receives the count.
int run_initv(Context* c, int64_t n_host, int64_t n_bound, uint32_t* flags, uint32_t* total_dev,
              const uint32_t* slot, const DevState* nds, const uint32_t* gate, bool finalize,
              const FinArgs* fin) {
  if (c->P.V_dim <= 0 || n_bound <= 0) return DFX_OK;
  if (!nds) nds = c->ds;
  if (gate && n_host < 0 && !finalize) {  // the fused step
    const int64_t ntiles = (n_bound + kIvTile - 1) / kIvTile;
    Workspace& ws = c->ws;
    void* before = ws.ivstat.p;
    DFX_TRY(ws.ivstat.ensure((size_t)ntiles * 8));
    if (ws.ivstat.p != before)  // fresh words read as unpublished (tag 0, flag 0)
      DFX_HIP(hipMemsetAsync(ws.ivstat.p, 0, ws.ivstat.bytes, c->stream));
    hipLaunchKernelGGL(k_initv_onepass, dim3((unsigned)ntiles), dim3(kStNT), 0, c->stream, flags,
                       total_dev, slot, c->T, c->P.V_init_scale, c->ds, nds, gate,
                       ws.ivstat.as<unsigned long long>(), fin ? *fin : FinArgs{});
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  DFX_TRY(scan_u32(c, flags, n_bound, total_dev, n_host >= 0 ? nullptr : &nds->u_count, gate));
  const int64_t nb = (n_bound + kStNT - 1) / kStNT;
  hipLaunchKernelGGL(k_initv, dim3((unsigned)(gate && nb > 1024 ? 1024 : nb)), dim3(kStNT), 0,
                     c->stream,
                     n_host, flags, total_dev, slot, c->T, c->P.V_init_scale, c->ds, nds, gate);
  if (finalize)
    hipLaunchKernelGGL(k_initv_finalize, dim3(1), dim3(1), 0, c->stream, total_dev, c->P.V_dim,
                       c->T.vcap, c->ds);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// ---- Update(kFeaCount) (sgd_updater.cc:64-75) ---------------------------------------------
__device__ inline uint32_t feacnt_apply(const Table& T, const Params& P, int64_t s, float c) {
  Entry* e = ent_at(T, s);
  float4 st = ent_state(e);
  st.w += c;  // fea_cnt
  ent_set_state(e, st);
  return (P.V_dim > 0 && e->vrow < 0 && st.x != 0.f && st.w > (float)P.V_threshold) ? 1u : 0u;
}

// standalone: keys + float counts (find-or-insert)
__global__ __launch_bounds__(kStNT) void k_push_cnt(int64_t n, const uint64_t* keys,
                                                    const float* cnt, Table T, Params P,
                                                    uint32_t* slot, uint32_t* flags,
                                                    DevState* ds) {
  const int64_t u = (int64_t)blockIdx.x * kStNT + threadIdx.x;
  int ins = 0;
  if (u < n) {
    bool inserted;
    int64_t s = tbl_insert(T, keys[u], &inserted);
    ins = inserted;
    uint32_t f = 0;
    if (s < 0) {
      atomicOr(&ds->err, insert_error(s));
    } else {
      f = feacnt_apply(T, P, s, cnt[u]);
      slot[u] = (uint32_t)s;
    }
    flags[u] = f;
  }
  block_count_add(ins, &ds->n_keys);
}

// fused: one segment per unique key, already resolved to a slot; count = segment length
__global__ __launch_bounds__(kStNT) void k_push_cnt_seg(const uint32_t* segstart,
                                                        const uint32_t* segslot, Table T,
                                                        Params P, uint32_t* flags,
                                                        const DevState* ds) {
  const int64_t u = (int64_t)blockIdx.x * kStNT + threadIdx.x;
  if (u >= (int64_t)ds->u_count) return;
  const float c = (float)(segstart[u + 1] - segstart[u]);
  const uint32_t s = segslot[u];
  flags[u] = s == kNoSlot ? 0u : feacnt_apply(T, P, s, c);
}

int push_cnt_seg_run(Context* c, int64_t n_bound, const uint32_t* segstart,
                     const uint32_t* segslot, uint32_t* flags, uint32_t* total_dev,
                     const DevState* nds) {
  if (n_bound <= 0) return DFX_OK;
  hipLaunchKernelGGL(k_push_cnt_seg, dim3((n_bound + kStNT - 1) / kStNT), dim3(kStNT), 0,
                     c->stream, segstart, segslot, c->T, c->P, flags, nds);
  DFX_HIP(hipGetLastError());
  return run_initv(c, -1, n_bound, flags, total_dev, segslot, nds);
}

int push_cnt_seg_flags(Context* c, const Lane& L, int64_t n_bound, const uint32_t* segstart,
                       const uint32_t* segslot, uint32_t* flags, const DevState* nds) {
  if (n_bound <= 0) return DFX_OK;
  hipLaunchKernelGGL(k_push_cnt_seg, dim3((n_bound + kStNT - 1) / kStNT), dim3(kStNT), 0,
                     L.stream, segstart, segslot, c->T, c->P, flags, nds);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// ---- standalone Get: interleaved [w | V] + lens ---------------------------------------------
// SGDUpdater::Get (sgd_updater.cc:34-58): V only if present and not (l1_shrk && w == 0).
// Missing keys read as w = 0 without V; Get's insertion of empty entries is not observable.
__global__ __launch_bounds__(kStNT) void k_pull_lens(int64_t n, const uint64_t* keys, Table T,
                                                     Params P, int32_t* slot_out,
                                                     uint32_t* len_out, DevState* ds) {
  const int64_t i = (int64_t)blockIdx.x * kStNT + threadIdx.x;
  if (i >= n) return;
  if (keys[i] == kEmptyKey) atomicOr(&ds->err, kErrBadKey);  // reported at the next sync
  int64_t s = tbl_find(T, keys[i]);
  int vr = -1;
  float w = 0.f;
  if (s >= 0) { w = ent_at(T, s)->w; vr = ent_at(T, s)->vrow; }
  bool live = vr >= 0 && !(P.l1_shrk && w == 0.f);
  slot_out[i] = (int32_t)s;
  len_out[i] = live ? (uint32_t)(T.d + 1) : 1u;
}

__global__ __launch_bounds__(kStNT) void k_pull_write(int64_t n, Table T, Params P,
                                                      const int32_t* slot_in,
                                                      const uint32_t* off, float* vals,
                                                      int32_t* lens) {
  const int64_t i = (int64_t)blockIdx.x * kStNT + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot_in[i];
  const uint32_t o = off[i];
  const float w = s >= 0 ? ent_at(T, s)->w : 0.f;
  const int vr = s >= 0 ? ent_at(T, s)->vrow : -1;
  const bool live = vr >= 0 && !(P.l1_shrk && w == 0.f);
  vals[o] = w;
  const int d = T.d;
  if (live) {
    const float* V = row_V(T, vr);
    for (int k = 0; k < d; ++k) vals[o + 1 + k] = V[k];
  }
  if (lens) lens[i] = live ? d + 1 : 1;
}

// ---- standalone Update(kGradient) (sgd_updater.cc:76-98) -----------------------------------
__global__ __launch_bounds__(kStNT) void k_push_grad(int64_t n, const uint64_t* keys,
                                                     const float* vals, const int32_t* lens,
                                                     const uint32_t* off, Table T, Params P,
                                                     uint32_t* slot, uint32_t* flags,
                                                     DevState* ds) {
  const int64_t i = (int64_t)blockIdx.x * kStNT + threadIdx.x;
  int ins = 0, dnew = 0;
  if (i < n) {
    bool inserted;
    int64_t s = tbl_insert(T, keys[i], &inserted);
    ins = inserted;
    uint32_t f = 0;
    if (s < 0) {
      atomicOr(&ds->err, insert_error(s));
    } else {
      const int d = T.d;
      const uint32_t o = lens ? off[i] : (uint32_t)i;
      Entry* en = ent_at(T, s);
      float4 e = ent_state(en);
      bool tr;
      dnew = ftrl_update(P, vals[o], &e, &tr);
      ent_set_state(en, e);
      const int vr = en->vrow;
      if (lens && lens[i] > 1) {
        if (lens[i] != d + 1) {
          atomicOr(&ds->err, kErrLens);
        } else if (vr < 0) {
          atomicOr(&ds->err, kErrNoV);
        } else {
          float* V = row_V(T, vr);
          float* C = row_C(T, vr);
          for (int k = 0; k < d; ++k) adagrad_update(P, vals[o + 1 + k], V + k, C + k);
        }
      }
      // InitV when w leaves 0 and the feature is frequent enough (sgd_updater.cc:118-121)
      if (tr && d > 0 && vr < 0 && e.w > (float)P.V_threshold) f = 1;
      slot[i] = (uint32_t)s;
    }
    flags[i] = f;
  }
  block_count_add(ins, &ds->n_keys);
  block_count_add(dnew, (unsigned long long*)&ds->new_w);
}

__global__ void k_check_total(const uint32_t* total, int64_t n_vals, DevState* ds) {
  if ((int64_t)*total != n_vals) atomicOr(&ds->err, kErrLens);
}

__global__ void k_lens_u32(int64_t n, const int32_t* lens, uint32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (uint32_t)lens[i];
}

// ---- table allocation / growth ------------------------------------------------------------
__global__ void k_tbl_init(Table T, int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  Entry e;
  e.w = e.sqrt_g = e.z = e.fea_cnt = 0.f;
  e.key = kEmptyKey;
  e.vrow = -1;
  e.pad = 0;
  *ent_at(T, i) = e;
}

// re-insert every key of table O into T; with fat slots a key's V and Vaux rows move with it
// (its vrow is its slot).  map (optional): map[old slot] = its new slot
__global__ void k_rehash(Table O, int64_t ocap, Table T, DevState* ds, uint32_t* map) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ocap) return;
  Entry e = *ent_at(O, i);
  if (e.key == kEmptyKey) {
    if (map) map[i] = kNoSlot;
    return;
  }
  bool ins;
  int64_t s = tbl_insert(T, e.key, &ins);
  if (map) map[i] = s < 0 ? kNoSlot : (uint32_t)s;
  if (s < 0) { atomicOr(&ds->err, kErrTableFull); return; }
  if (T.es && e.vrow >= 0) {
    const float* V0 = row_V(O, e.vrow);
    const float* C0 = row_C(O, e.vrow);
    float* V1 = row_V(T, s);
    float* C1 = row_C(T, s);
    for (int k = 0; k < T.d; ++k) {
      V1[k] = V0[k];
      C1[k] = C0[k];
    }
    e.vrow = (int32_t)s;
  }
  *ent_at(T, s) = e;
}

// slots (and, with fat slots, the Vaux pool: one row per slot) for capacity cap
static int table_alloc_entries(Table* T, int64_t cap, hipStream_t st) {
  DFX_HIP(hipMalloc(&T->ent, cap * (sizeof(Entry) << T->es)));
  if (T->es) {
    DFX_HIP(hipMalloc(&T->V, cap * (int64_t)T->d * sizeof(float)));
    T->vcap = cap;
  }
  hipLaunchKernelGGL(k_tbl_init, dim3((cap + 255) / 256), dim3(256), 0, st, *T, cap);
  DFX_HIP(hipGetLastError());
  int lg = 0;
  while ((1ll << lg) < cap) ++lg;
  T->logcap = lg;
  T->mask = (uint64_t)cap - 1;
  return DFX_OK;
}

// a live key-range server step's segment slots, moved to the rebuilt table
__global__ void k_remap_segslots(uint32_t* segslot, const uint32_t* nseg, int64_t bound,
                                 const uint32_t* map) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= bound || u >= (int64_t)*nseg) return;
  const uint32_t s = segslot[u];
  if (s != kNoSlot) segslot[u] = map[s];
}

// Rebuild the table as NT (new hash parameters and/or capacity): every entry of the old
// table is re-inserted.  The old table is freed only once every entry landed; on a failure
// (a full new table) the old one stays and the error is returned.  A key-range server's step
// slots that hold table positions across calls (dfx_dist_owner_begin to its push / InitV: a
// pipelined schedule's other step) get their positions moved with the keys.
static int table_rebuild(Context* c, Table NT, int64_t new_cap) {
  Table& T = c->T;
  DFX_TRY(table_alloc_entries(&NT, new_cap, c->stream));
  int err0 = 0, err1 = 0;
  DFX_HIP(hipMemcpyAsync(&err0, &c->ds->err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  bool remap = false;
  for (int s = 0; s < kSlots; ++s)
    remap = remap || (c->dist_live[s] && !c->dist_segs_pending[s] && c->dist_R[s] > 0);
  uint32_t* map = nullptr;
  if (remap) DFX_HIP(hipMalloc(&map, (size_t)c->cap * sizeof(uint32_t)));
  hipLaunchKernelGGL(k_rehash, dim3((c->cap + 255) / 256), dim3(256), 0, c->stream, T,
                     c->cap, NT, c->ds, map);
  DFX_HIP(hipGetLastError());
  DFX_HIP(hipMemcpyAsync(&err1, &c->ds->err, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  if ((err1 & ~err0) & kErrTableFull) {
    (void)hipFree(NT.ent);
    if (NT.es) (void)hipFree(NT.V);
    if (map) (void)hipFree(map);
    DFX_HIP(hipMemcpy(&c->ds->err, &err0, sizeof(int), hipMemcpyHostToDevice));
    set_error("table rebuild: the new table cannot hold every key; the old table is kept");
    return DFX_ERR_CAPACITY;
  }
  for (int s = 0; s < kSlots && map; ++s) {
    const int64_t R = c->dist_R[s];
    if (!c->dist_live[s] || c->dist_segs_pending[s] || R <= 0) continue;
    hipLaunchKernelGGL(k_remap_segslots, dim3((unsigned)((R + 255) / 256)), dim3(256), 0,
                       c->stream, c->ows[s].osegslot.as<uint32_t>(), &c->ods[s]->totals[1], R,
                       map);
    DFX_HIP(hipGetLastError());
  }
  if (map) {
    DFX_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(map);
  }
  (void)hipFree(T.ent);
  if (T.es) (void)hipFree(T.V);
  T = NT;
  c->cap = new_cap;
  return DFX_OK;
}

int table_unclump(Context* c) {
  Table& T = c->T;
  if (!T.ent) return DFX_OK;
  int flag = 0;
  DFX_HIP(hipMemcpyAsync(&flag, &c->ds->probe_flag, sizeof(int), hipMemcpyDeviceToHost,
                         c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  if (!flag) return DFX_OK;
  DFX_HIP(hipMemsetAsync(&c->ds->probe_flag, 0, sizeof(int), c->stream));
  if (!T.ordered) return DFX_OK;
  // the keys cluster in their top bits: rebuild with the multiplicative hash (same capacity)
  Table NT = T;
  NT.ordered = 0;
  return table_rebuild(c, NT, c->cap);
}

// A key-range server's table (dist.hip): the ordered hash over the position of a key inside
// the server's range (Table::range_mul = the number of ranges).  The plain ordered hash would
// send all of one server's keys, which share their top bits, into 1/N of the table — probe
// chains the length of the whole key set.  Rebuilds the table once when the range count
// changes (same capacity); a table on the multiplicative hash needs nothing.
int table_set_ranges(Context* c, int nranks) {
  Table& T = c->T;
  const uint64_t mul = (uint64_t)(nranks > 0 ? nranks : 1);
  if (!T.ent || T.range_mul == mul) return DFX_OK;
  if (!T.ordered) {
    T.range_mul = mul;
    return DFX_OK;
  }
  Table NT = T;
  NT.range_mul = mul;
  return table_rebuild(c, NT, c->cap);
}

int table_alloc(Context* c, int64_t n_keys, int64_t n_vrows) {
  if (n_keys < 64) n_keys = 64;
  int64_t cap = 1;
  while (cap < 2 * n_keys) cap <<= 1;
  Table& T = c->T;
  T.d = c->P.V_dim;
  T.es = c->slot_es;
  DFX_TRY(table_alloc_entries(&T, cap, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  c->cap = cap;
  if (T.es) return DFX_OK;  // the Vaux pool came with the slots
  T.vcap = T.d > 0 ? (n_vrows > 0 ? n_vrows : 1) : 0;
  if (T.d > 0) DFX_HIP(hipMalloc(&T.V, T.vcap * 2 * T.d * sizeof(float)));
  return DFX_OK;
}

void table_release(Context* c) {
  Table& T = c->T;
  if (T.ent) (void)hipFree(T.ent);
  if (T.V) (void)hipFree(T.V);
  T = Table{};
}

struct HostCounters {
  unsigned long long n_keys, n_vrows;
  unsigned seed;
  long long new_w;
};

static int read_counters(Context* c, HostCounters* h) {
  DevState s;
  DFX_HIP(hipMemcpyAsync(&s, c->ds, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  h->n_keys = s.n_keys;
  h->n_vrows = s.n_vrows;
  h->seed = s.seed;
  h->new_w = s.new_w;
  return DFX_OK;
}

int store_reserve(Context* c, int64_t n_keys, int64_t n_vrows) {
  DFX_HIP(hipStreamSynchronize(c->stream));
  Table& T = c->T;
  DFX_TRY(table_unclump(c));
  if (2 * n_keys > c->cap) {
    int64_t cap = c->cap;
    while (cap < 2 * n_keys) cap <<= 1;
    DFX_TRY(table_rebuild(c, T, cap));
  }
  if (T.d > 0 && !T.es && n_vrows > T.vcap) {  // fat slots: V grows with the slots
    HostCounters h;
    DFX_TRY(read_counters(c, &h));
    float* nV;
    DFX_HIP(hipMalloc(&nV, n_vrows * 2 * T.d * sizeof(float)));
    if (h.n_vrows) {
      DFX_HIP(hipMemcpy(nV, T.V, h.n_vrows * 2 * T.d * sizeof(float), hipMemcpyDeviceToDevice));
    }
    (void)hipFree(T.V);
    T.V = nV;
    T.vcap = n_vrows;
  }
  return DFX_OK;
}

// ---- automatic growth ---------------------------------------------------------------------
// consume the oldest recorded counts (wait: block for them; else only when complete)
static int cap_pop_oldest(Context* c, bool wait, bool* popped) {
  CapGuard& g = c->capg;
  *popped = false;
  if (g.count == 0) return DFX_OK;
  const int i = (g.head - g.count + kCapRing) % kCapRing;
  if (wait) {
    DFX_HIP(hipEventSynchronize(g.ev[i]));
  } else {
    const hipError_t q = hipEventQuery(g.ev[i]);
    if (q == hipErrorNotReady) return DFX_OK;
    DFX_HIP(q);
  }
  g.known_keys = (int64_t)g.host[2 * i];
  g.known_vrows = (int64_t)g.host[2 * i + 1];
  g.known_enq = g.enq_at[i];
  --g.count;
  *popped = true;
  return DFX_OK;
}

// the ring entry the next recorded counts go to: the step's last kernel may write them there
// itself (k_step_finalize: one launch less than a copy), then cap_record_commit
int cap_record_slot(Context* c, unsigned long long** slot) {
  *slot = nullptr;
  if (!c->autogrow) return DFX_OK;
  CapGuard& g = c->capg;
  if (!g.host) {
    DFX_HIP(hipHostMalloc(reinterpret_cast<void**>(&g.host), 2 * kCapRing * 8,
                          hipHostMallocDefault));
    for (auto& e : g.ev) DFX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  bool popped;
  if (g.count == kCapRing) DFX_TRY(cap_pop_oldest(c, true, &popped));
  *slot = g.host + 2 * g.head;
  return DFX_OK;
}

// the counts of the slot cap_record_slot returned are written by work already on the stream
int cap_record_commit(Context* c, hipEvent_t* recorded) {
  if (recorded) *recorded = nullptr;
  if (!c->autogrow) return DFX_OK;
  CapGuard& g = c->capg;
  const int i = g.head;
  DFX_HIP(hipEventRecord(g.ev[i], c->stream));
  if (recorded) *recorded = g.ev[i];  // (re-recorded kCapRing steps later)
  g.enq_at[i] = g.enq_total;
  g.head = (g.head + 1) % kCapRing;
  ++g.count;
  return DFX_OK;
}

int cap_record(Context* c) {
  unsigned long long* slot = nullptr;
  DFX_TRY(cap_record_slot(c, &slot));
  if (!slot) return DFX_OK;
  static_assert(offsetof(DevState, n_vrows) == offsetof(DevState, n_keys) + 8, "layout");
  DFX_HIP(hipMemcpyAsync(slot, &c->ds->n_keys, 16, hipMemcpyDeviceToHost, c->stream));
  return cap_record_commit(c);
}

void cap_release(Context* c) {
  CapGuard& g = c->capg;
  for (auto& e : g.ev)
    if (e) (void)hipEventDestroy(e);
  if (g.host) (void)hipHostFree(g.host);
  g = CapGuard{};
}

// table capacity >= 2 * need_keys, V pool >= need_vrows (doubling at least, unless exact)
static int grow_to(Context* c, int64_t need_keys, int64_t need_vrows, bool exact = false) {
  const Table& T = c->T;
  const bool gk = 2 * need_keys > c->cap;
  const bool gv = T.d > 0 && need_vrows > T.vcap;
  if (!gk && !gv) return DFX_OK;
  return store_reserve(c, gk ? need_keys : 0,
                       gv ? (exact ? need_vrows : std::max<int64_t>(2 * T.vcap, need_vrows)) : 0);
}

int cap_check(Context* c, int64_t add) {
  if (!c->autogrow || !c->T.ent) return DFX_OK;
  CapGuard& g = c->capg;
  bool popped = true;
  while (popped) DFX_TRY(cap_pop_oldest(c, false, &popped));
  const bool has_v = c->T.d > 0;
  // Waiting on an older step's counts only pays while the table has room for kCapRunAhead
  // steps of worst-case inserts beyond them: below that, each step would wait for the one
  // before it to finish, and the Localizer lane of step t+1 could no longer run beside step t
  // (C2: 2^20 keys, 4M occurrences a batch, 0.73 -> 0.45 ms).  Then grow once at a sync point.
  constexpr int64_t kCapRunAhead = 3;
  for (;;) {
    const int64_t pend = g.enq_total - g.known_enq + add;
    const bool keys_ok = 10 * (g.known_keys + pend) <= 9 * c->cap;
    const bool vrows_ok = !has_v || g.known_vrows + pend <= c->T.vcap;
    if (keys_ok && vrows_ok) break;
    const auto t0 = std::chrono::steady_clock::now();
    const bool room_ahead = 10 * (g.known_keys + kCapRunAhead * add) <= 9 * c->cap &&
                            (!has_v || g.known_vrows + kCapRunAhead * add <= c->T.vcap);
    if (g.count > 0 && room_ahead) {  // an older step's counts may show room: wait for it
      DFX_TRY(cap_pop_oldest(c, true, &popped));
      c->host_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      c->host_waits += 1;
      continue;
    }
    // exact counts at a sync point; grow so that kCapRunAhead such steps fit below 0.9 load
    DFX_HIP(hipStreamSynchronize(c->stream));
    c->host_wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    c->host_waits += 1;
    HostCounters h;
    DFX_TRY(read_counters(c, &h));
    while (g.count > 0) DFX_TRY(cap_pop_oldest(c, false, &popped));  // all complete now
    g.known_keys = (int64_t)h.n_keys;
    g.known_vrows = (int64_t)h.n_vrows;
    g.known_enq = g.enq_total;
    const int64_t need = g.known_keys + kCapRunAhead * add;
    const int64_t need_cap_keys = (10 * need + 8) / 9;  // 0.9 load with that many in flight
    const int64_t need_keys = std::max<int64_t>(need_cap_keys / 2 + 1,
                                                2 * g.known_keys > c->cap ? g.known_keys : 0);
    if (grow_to(c, need_keys, has_v ? g.known_vrows + kCapRunAhead * add : 0) != DFX_OK) {
      // the V pool's run-ahead is priced at one V row per occurrence (the worst case; lazy V
      // draws far fewer): when that much does not fit, grow it by one step's worst case only,
      // exactly — the guard above then waits on older steps' counts instead of running ahead
      (void)hipGetLastError();
      DFX_TRY(grow_to(c, need_keys, has_v ? g.known_vrows + add : 0, true));
    }
    break;
  }
  g.enq_total += add;
  return DFX_OK;
}

int store_maybe_grow(Context* c) {
  if (!c->T.ent) return DFX_OK;
  HostCounters h;
  DFX_TRY(read_counters(c, &h));
  if (c->autogrow && 2 * (int64_t)h.n_keys > c->cap)
    DFX_TRY(grow_to(c, (int64_t)h.n_keys, 0));
  // the stream is idle: every recorded count is complete, and the exact ones are at hand
  CapGuard& g = c->capg;
  g.count = 0;
  g.known_keys = (int64_t)h.n_keys;
  g.known_vrows = (int64_t)h.n_vrows;
  g.known_enq = g.enq_total;
  return DFX_OK;
}

// load: host-parsed entries uploaded and inserted (SGDEntry::LoadEntry keeps fea_cnt, and
// keeps sqrt_g/z when the file has no aux data)
// vr: the entry's V row in the split layout (uploaded to the pool beforehand), or with fat
// slots its row of VV ([V | Vaux] per loaded V row, vr - vbase), copied into the slot here
__global__ void k_load(int64_t n, const uint64_t* keys, const float4* st, const int32_t* vr,
                       int has_aux, Table T, DevState* ds, const float* VV, int64_t vbase) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int ins = 0;
  if (i < n) {
    bool inserted;
    int64_t s = tbl_insert(T, keys[i], &inserted);
    ins = inserted;
    if (s < 0) {
      atomicOr(&ds->err, insert_error(s));
    } else {
      Entry* en = ent_at(T, s);
      float4 e = ent_state(en);
      e.x = st[i].x;
      if (has_aux) { e.y = st[i].y; e.z = st[i].z; }
      ent_set_state(en, e);
      if (vr[i] >= 0 && T.es) {
        const float* src = VV + (vr[i] - vbase) * 2 * (int64_t)T.d;
        float* V = row_V(T, s);
        float* C = row_C(T, s);
        for (int k = 0; k < T.d; ++k) {
          V[k] = src[k];
          C[k] = src[T.d + k];
        }
        en->vrow = (int32_t)s;
      } else if (vr[i] >= 0) {
        en->vrow = vr[i];
      }
    }
  }
  block_count_add(ins, &ds->n_keys);
}

__global__ void k_penalty(Table T, int64_t cap, Params P, double* acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double objv = 0, nnz = 0;
  if (i < cap && ent_at(T, i)->key != kEmptyKey) {
    const float w = ent_at(T, i)->w;
    if (w != 0.f) nnz += 1;
    objv += P.l1 * fabs(w) + .5 * P.l2 * w * w;
    const int vr = ent_at(T, i)->vrow;
    if (vr >= 0) {
      nnz += T.d;
      const float* V = row_V(T, vr);
      for (int k = 0; k < T.d; ++k) objv += .5 * P.l2 * V[k] * V[k];  // (sic) l2, :21
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    objv += __shfl_xor(objv, off, kWave);
    nnz += __shfl_xor(nnz, off, kWave);
  }
  if (lane_id() == 0 && (objv != 0 || nnz != 0)) {
    atomicAdd(&acc[0], objv);
    atomicAdd(&acc[1], nnz);
  }
}

// probe distance of every occupied slot from its key's home slot (linear probing)
__global__ void k_probe_stats(Table T, int64_t cap, unsigned long long* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long dist = 0, occ = 0, mx = 0;
  if (i < cap && ent_at(T, i)->key != kEmptyKey) {
    const uint64_t h = tbl_hash(ent_at(T, i)->key, T);
    dist = ((uint64_t)i - h) & T.mask;
    occ = 1;
    mx = dist;
  }
  for (int off = 32; off > 0; off >>= 1) {
    dist += __shfl_xor(dist, off, kWave);
    occ += __shfl_xor(occ, off, kWave);
    const unsigned long long o = __shfl_xor(mx, off, kWave);
    mx = o > mx ? o : mx;
  }
  if (lane_id() == 0 && occ) {
    atomicAdd(&out[0], dist);
    atomicAdd(&out[1], occ);
    atomicMax(&out[2], mx);
  }
}

// Every stored entry with its V and Vaux rows (null without V), in slot order, for save /
// dump.  Fat slots stream the table in chunks of kHostChunk slots (a key's V and Vaux rows are
// its slot's, so a chunk carries them); the split layout copies the entries and the used V pool
// rows once (V rows are in allocation order, not slot order).
constexpr int64_t kHostChunk = 1 << 20;

template <typename F>
static int for_each_entry(Context* c, F fn) {
  const Table& T = c->T;
  const int d = T.d;
  HostCounters hc;
  DFX_TRY(read_counters(c, &hc));
  if (T.es) {
    std::vector<Entry> raw((size_t)std::min<int64_t>(c->cap, kHostChunk) << T.es);
    std::vector<float> aux((size_t)std::min<int64_t>(c->cap, kHostChunk) * d);
    for (int64_t i0 = 0; i0 < c->cap; i0 += kHostChunk) {
      const int64_t n = std::min<int64_t>(kHostChunk, c->cap - i0);
      DFX_HIP(hipMemcpy(raw.data(), ent_at(T, i0), ((size_t)n << T.es) * sizeof(Entry),
                        hipMemcpyDeviceToHost));
      if (d > 0)
        DFX_HIP(hipMemcpy(aux.data(), T.V + i0 * d, (size_t)n * d * 4, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < n; ++i) {
        const Entry& e = raw[(size_t)i << T.es];
        if (e.key == kEmptyKey) continue;
        const bool v = e.vrow >= 0;
        fn(e, v ? reinterpret_cast<const float*>(&raw[(size_t)i << T.es] + 1) : nullptr,
           v ? aux.data() + (size_t)i * d : nullptr);
      }
    }
    return DFX_OK;
  }
  std::vector<Entry> ent((size_t)c->cap);
  std::vector<float> VV((size_t)hc.n_vrows * 2 * d);  // [V(d) | Vaux(d)] per V row
  DFX_HIP(hipMemcpy(ent.data(), T.ent, c->cap * sizeof(Entry), hipMemcpyDeviceToHost));
  if (!VV.empty()) DFX_HIP(hipMemcpy(VV.data(), T.V, VV.size() * 4, hipMemcpyDeviceToHost));
  for (const Entry& e : ent) {
    if (e.key == kEmptyKey) continue;
    const bool v = e.vrow >= 0;
    fn(e, v ? VV.data() + (size_t)e.vrow * 2 * d : nullptr,
       v ? VV.data() + (size_t)e.vrow * 2 * d + d : nullptr);
  }
  return DFX_OK;
}

}  // namespace dfx

using namespace dfx;

extern "C" {

int dfx_store_pull(dfx_ctx* ctx, const uint64_t* keys, int64_t n, float* vals, int32_t* lens,
                   int64_t* n_vals) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  const int d = c->P.V_dim;
  DFX_CHECK_ARG(n >= 0, "pull: negative n");
  DFX_CHECK_ARG(d == 0 || lens || n == 0, "pull: lens required when V_dim > 0");
  if (n == 0) {
    if (n_vals) *n_vals = 0;
    return DFX_OK;
  }
  DFX_CHECK_ARG(keys && vals, "pull: null buffer");
  Workspace& ws = c->ws;
  DFX_TRY(ws.flags.ensure((n + 1) * 4));
  DFX_TRY(ws.slot.ensure((n + 1) * 4));
  DFX_TRY(ws.cnt.ensure(16));
  uint32_t* off = ws.flags.as<uint32_t>();
  int32_t* sl = ws.slot.as<int32_t>();
  uint32_t* total = ws.cnt.as<uint32_t>();
  dim3 grid((n + kStNT - 1) / kStNT);
  hipLaunchKernelGGL(k_pull_lens, grid, dim3(kStNT), 0, c->stream, n, keys, c->T, c->P, sl, off,
                     c->ds);
  DFX_TRY(scan_u32(c, off, n, total));
  hipLaunchKernelGGL(k_pull_write, grid, dim3(kStNT), 0, c->stream, n, c->T, c->P, sl, off, vals,
                     d > 0 ? lens : nullptr);
  DFX_HIP(hipGetLastError());
  if (n_vals) {
    uint32_t t = 0;
    DFX_HIP(hipMemcpyAsync(&t, total, 4, hipMemcpyDeviceToHost, c->stream));
    DFX_HIP(hipStreamSynchronize(c->stream));
    *n_vals = t;
  }
  return DFX_OK;
}

static int store_push(Context* c, const uint64_t* keys, int64_t n, int type, const float* vals,
                      int64_t n_vals, const int32_t* lens);

int dfx_store_push(dfx_ctx* ctx, const uint64_t* keys, int64_t n, int type, const float* vals,
                   int64_t n_vals, const int32_t* lens) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(n >= 0, "push: negative n");
  if (n == 0) return DFX_OK;
  DFX_CHECK_ARG(keys && vals, "push: null buffer");
  DFX_TRY(cap_check(c, n));
  DFX_TRY(store_push(c, keys, n, type, vals, n_vals, lens));
  return cap_record(c);
}

static int store_push(Context* c, const uint64_t* keys, int64_t n, int type, const float* vals,
                      int64_t n_vals, const int32_t* lens) {
  Workspace& ws = c->ws;
  DFX_TRY(ws.flags.ensure((n + 1) * 4));
  DFX_TRY(ws.slot.ensure((n + 1) * 4));
  DFX_TRY(ws.cnt.ensure(16));
  uint32_t* flags = ws.flags.as<uint32_t>();
  uint32_t* slot = ws.slot.as<uint32_t>();
  uint32_t* total = ws.cnt.as<uint32_t>();
  if (type == DFX_FEA_COUNT) {
    if (n_vals != n) {
      set_error("CHECK_EQ(fea_ids.size(), values.size()) failed (sgd_updater.cc:65)");
      return DFX_ERR_CHECK;
    }
    hipLaunchKernelGGL(k_push_cnt, dim3((n + kStNT - 1) / kStNT), dim3(kStNT), 0, c->stream, n,
                       keys, vals, c->T, c->P, slot, flags, c->ds);
    DFX_HIP(hipGetLastError());
    return run_initv(c, n, n, flags, total, slot);
  }
  if (type != DFX_GRADIENT) {
    set_error("UNKNOWN value_type (sgd_updater.cc:100)");
    return DFX_ERR_CHECK;
  }
  uint32_t* off = nullptr;
  if (lens) {
    DFX_TRY(ws.rowtmp.ensure((n + 1) * 4));
    off = ws.rowtmp.as<uint32_t>();
    hipLaunchKernelGGL(k_lens_u32, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, lens, off);
    DFX_TRY(scan_u32(c, off, n, total));
    hipLaunchKernelGGL(k_check_total, dim3(1), dim3(1), 0, c->stream, total, n_vals, c->ds);
  } else if (n_vals != n) {
    set_error("CHECK_EQ(values.size(), size) failed (sgd_updater.cc:79)");
    return DFX_ERR_CHECK;
  }
  hipLaunchKernelGGL(k_push_grad, dim3((n + kStNT - 1) / kStNT), dim3(kStNT), 0, c->stream, n,
                     keys, vals, lens, off, c->T, c->P, slot, flags, c->ds);
  DFX_HIP(hipGetLastError());
  return run_initv(c, n, n, flags, total, slot);
}

int dfx_store_reserve(dfx_ctx* ctx, int64_t n_keys, int64_t n_vrows) {
  DFX_CHECK_ARG(ctx, "null ctx");
  return store_reserve(&ctx->c, n_keys, n_vrows);
}

int dfx_store_stats(dfx_ctx* ctx, int64_t* n_keys, int64_t* n_vrows, double* new_w,
                    uint32_t* seed) {
  DFX_CHECK_ARG(ctx, "null ctx");
  HostCounters h;
  DFX_TRY(read_counters(&ctx->c, &h));
  if (n_keys) *n_keys = (int64_t)h.n_keys;
  if (n_vrows) *n_vrows = (int64_t)h.n_vrows;
  if (new_w) *new_w = (double)h.new_w;
  if (seed) *seed = h.seed;
  return dfx_sync(ctx);
}

// table health: the mean and the longest distance of a stored key from its home slot, and the
// capacity (slots) — the ordered hash keeps both small at load factor <= 0.5
int dfx_store_probe_stats(dfx_ctx* ctx, double* mean_probe, int64_t* max_probe,
                          int64_t* capacity) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  DFX_TRY(c->ws.dscratch.ensure(64));
  unsigned long long* acc = c->ws.dscratch.as<unsigned long long>();
  DFX_HIP(hipMemsetAsync(acc, 0, 3 * 8, c->stream));
  hipLaunchKernelGGL(k_probe_stats, dim3((unsigned)((c->cap + 255) / 256)), dim3(256), 0,
                     c->stream, c->T, c->cap, acc);
  unsigned long long h[3];
  DFX_HIP(hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  if (mean_probe) *mean_probe = h[1] ? (double)h[0] / (double)h[1] : 0.0;
  if (max_probe) *max_probe = (int64_t)h[2];
  if (capacity) *capacity = c->cap;
  return DFX_OK;
}

int dfx_store_evaluate(dfx_ctx* ctx, double* penalty, int64_t* nnz) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  DFX_TRY(c->ws.dscratch.ensure(64));
  double* acc = c->ws.dscratch.as<double>();
  DFX_HIP(hipMemsetAsync(acc, 0, 2 * sizeof(double), c->stream));
  hipLaunchKernelGGL(k_penalty, dim3((c->cap + 255) / 256), dim3(256), 0, c->stream, c->T, c->cap,
                     c->P, acc);
  double h[2];
  DFX_HIP(hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  if (penalty) *penalty = h[0];
  if (nnz) *nnz = (int64_t)h[1];
  return DFX_OK;
}

int dfx_store_entry(dfx_ctx* ctx, uint64_t key, float* state, float* V, int* has_v, int* found) {
  DFX_CHECK_ARG(ctx && state && has_v && found, "null argument");
  Context* c = &ctx->c;
  const Table& T = c->T;
  DFX_HIP(hipStreamSynchronize(c->stream));
  // host-side probe of the same hash sequence (test hook; not a hot path)
  uint64_t h = tbl_hash(key, T);
  *found = 0;
  for (uint64_t probe = 0; probe <= T.mask; ++probe) {
    Entry e;
    DFX_HIP(hipMemcpy(&e, ent_at(T, h), sizeof(Entry), hipMemcpyDeviceToHost));
    if (e.key == kEmptyKey) return DFX_OK;
    if (e.key == key) {
      state[0] = e.w; state[1] = e.sqrt_g; state[2] = e.z; state[3] = e.fea_cnt;
      *has_v = e.vrow >= 0;
      if (e.vrow >= 0 && V) {
        DFX_HIP(hipMemcpy(V, row_V(T, e.vrow), T.d * 4, hipMemcpyDeviceToHost));
        DFX_HIP(hipMemcpy(V + T.d, row_C(T, e.vrow), T.d * 4,
                          hipMemcpyDeviceToHost));
      }
      *found = 1;
      return DFX_OK;
    }
    h = (h + 1) & T.mask;
  }
  return DFX_OK;
}

// SGDUpdater::Save (sgd_updater.h:84-106, SGDEntry::SaveEntry :35-48)
int dfx_store_save(dfx_ctx* ctx, const char* path, int save_aux) {
  DFX_CHECK_ARG(ctx && path, "null argument");
  Context* c = &ctx->c;
  const int d = c->T.d;
  FILE* f = fopen(path, "wb");
  if (!f) { set_error(std::string("cannot open ") + path); return DFX_ERR_IO; }
  bool aux = save_aux != 0;
  fwrite(&aux, sizeof(bool), 1, f);
  const int rc = for_each_entry(c, [&](const Entry& e, const float* V, const float* C) {
    const int size = V ? 1 + d : 1;
    if (e.w == 0.f && size == 1) return;  // SGDEntry::empty()
    const uint64_t key = e.key;
    fwrite(&key, 8, 1, f);
    fwrite(&size, sizeof(int), 1, f);
    fwrite(&e.w, 4, 1, f);
    if (aux) { fwrite(&e.sqrt_g, 4, 1, f); fwrite(&e.z, 4, 1, f); }
    if (size == 1) return;
    fwrite(V, 4, d, f);
    if (aux) fwrite(C, 4, d, f);
  });
  if (rc != DFX_OK) {
    fclose(f);
    return rc;
  }
  fclose(f);
  return DFX_OK;
}

// SGDUpdater::Load (sgd_updater.h:84-96, SGDEntry::LoadEntry :50-68)
int dfx_store_load(dfx_ctx* ctx, const char* path) {
  return dfx_store_load_part(ctx, path, 0, 1);
}

// the keys of `path` that rank `rank` of `nranks` owns under the sharded store's rule
// owner(k) = floor(k * nranks / 2^64) (dist.hip): a model saved by N servers loads into M
int dfx_store_load_part(dfx_ctx* ctx, const char* path, int rank, int nranks) {
  DFX_CHECK_ARG(ctx && path, "null argument");
  DFX_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "store_load_part: bad rank");
  Context* c = &ctx->c;
  DFX_TRY(table_set_ranges(c, nranks));  // this server keeps the keys of range `rank`
  Table& T = c->T;
  FILE* f = fopen(path, "rb");
  if (!f) { set_error(std::string("cannot open ") + path); return DFX_ERR_IO; }
  bool aux;
  if (fread(&aux, sizeof(bool), 1, f) != 1) { fclose(f); return DFX_OK; }
  HostCounters hc;
  DFX_TRY(read_counters(c, &hc));
  std::vector<uint64_t> keys;
  std::vector<float4> st;
  std::vector<int32_t> vr;
  std::vector<float> VV;  // rows of [V(d) | Vaux(d)]
  uint64_t key;
  int64_t vnext = (int64_t)hc.n_vrows;
  while (fread(&key, 8, 1, f) == 1) {
    int size;
    float4 e = make_float4(0, 0, 0, 0);
    if (fread(&size, sizeof(int), 1, f) != 1 || fread(&e.x, 4, 1, f) != 1) {
      fclose(f); set_error("truncated model file"); return DFX_ERR_IO;
    }
    if (aux && (fread(&e.y, 4, 1, f) != 1 || fread(&e.z, 4, 1, f) != 1)) {
      fclose(f); set_error("truncated model file"); return DFX_ERR_IO;
    }
    int32_t row = -1;
    if (size > 1) {
      if (size != T.d + 1) { fclose(f); set_error("model V_dim mismatch"); return DFX_ERR_CHECK; }
      size_t base = VV.size();
      VV.resize(base + 2 * T.d, 0.f);
      if (fread(VV.data() + base, 4, T.d, f) != (size_t)T.d) {
        fclose(f); set_error("truncated model file"); return DFX_ERR_IO;
      }
      if (aux && fread(VV.data() + base + T.d, 4, T.d, f) != (size_t)T.d) {
        fclose(f); set_error("truncated model file"); return DFX_ERR_IO;
      }
      row = (int32_t)vnext++;
    }
    if (key == kEmptyKey) {
      fclose(f);
      set_error("model file holds key 0xffffffffffffffff, reserved as the empty-slot marker");
      return DFX_ERR_ARG;
    }
    if ((int)(((unsigned __int128)key * (unsigned)nranks) >> 64) != rank) {
      if (row >= 0) {  // not ours: drop its V row again
        VV.resize(VV.size() - 2 * T.d);
        --vnext;
      }
      continue;
    }
    keys.push_back(key);
    st.push_back(e);
    vr.push_back(row);
  }
  fclose(f);
  const int64_t n = (int64_t)keys.size();
  DFX_TRY(store_reserve(c, (int64_t)hc.n_keys + n, vnext));
  if (n == 0) return DFX_OK;
  uint64_t* dk;
  float4* dst;
  int32_t* dvr;
  float* dVV = nullptr;
  DFX_HIP(hipMalloc(&dk, n * 8));
  DFX_HIP(hipMalloc(&dst, n * sizeof(float4)));
  DFX_HIP(hipMalloc(&dvr, n * 4));
  DFX_HIP(hipMemcpy(dk, keys.data(), n * 8, hipMemcpyHostToDevice));
  DFX_HIP(hipMemcpy(dst, st.data(), n * sizeof(float4), hipMemcpyHostToDevice));
  DFX_HIP(hipMemcpy(dvr, vr.data(), n * 4, hipMemcpyHostToDevice));
  if (!VV.empty() && T.es) {  // fat slots: k_load copies each row into its key's slot
    DFX_HIP(hipMalloc(&dVV, VV.size() * 4));
    DFX_HIP(hipMemcpy(dVV, VV.data(), VV.size() * 4, hipMemcpyHostToDevice));
  } else if (!VV.empty()) {
    DFX_HIP(hipMemcpy(row_V(T, hc.n_vrows), VV.data(), VV.size() * 4, hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(k_load, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, dk, dst, dvr,
                     aux ? 1 : 0, T, c->ds, dVV, (int64_t)hc.n_vrows);
  DFX_HIP(hipStreamSynchronize(c->stream));
  if (dVV) (void)hipFree(dVV);
  unsigned long long nv = (unsigned long long)vnext;
  DFX_HIP(hipMemcpy(&c->ds->n_vrows, &nv, 8, hipMemcpyHostToDevice));
  // new_w = model_.size() (sgd_updater.h:91)
  DevState s;
  DFX_HIP(hipMemcpy(&s, c->ds, sizeof(s), hipMemcpyDeviceToHost));
  long long nw = (long long)s.n_keys;
  DFX_HIP(hipMemcpy(&c->ds->new_w, &nw, 8, hipMemcpyHostToDevice));
  (void)hipFree(dk);
  (void)hipFree(dst);
  (void)hipFree(dvr);
  return dfx_sync(ctx);
}

// SGDUpdater::Dump (sgd_updater.h:108-139): text, one entry per line
int dfx_store_dump(dfx_ctx* ctx, const char* path, int dump_aux, int need_reverse) {
  DFX_CHECK_ARG(ctx && path, "null argument");
  Context* c = &ctx->c;
  const int d = c->T.d;
  std::ofstream os(path);
  if (!os) { set_error(std::string("cannot open ") + path); return DFX_ERR_IO; }
  return for_each_entry(c, [&](const Entry& e, const float* V, const float* C) {
    const int size = V ? 1 + d : 1;
    if (e.w == 0.f && size == 1) return;
    os << (need_reverse ? reverse_bytes(e.key) : (uint64_t)e.key);
    os << '\t' << size << '\t' << e.w;
    if (dump_aux) os << '\t' << e.sqrt_g << '\t' << e.z;
    if (size > 1) {
      for (int k = 0; k < d; ++k) os << '\t' << V[k];
      if (dump_aux)
        for (int k = 0; k < d; ++k) os << '\t' << C[k];
    }
    os << '\n';
  });
}

}  // extern "C"
