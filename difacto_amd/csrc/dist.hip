// Key-range-sharded multi-GPU store: the device phases of one synchronous data-parallel step.
//
// The reference's distributed store (src/store/kvstore_dist.h) shards the model over ps-lite
// servers by key range; a worker ZPushes / ZPulls its sorted keys (:90-108) and each server
// answers a pull with updater_->Get (:167-175) and applies every push as one
// updater_->Update call (:158-165), each server holding its own SGDUpdater (own rand_r seed,
// own new_w).  Here every GPU is both a worker (its own minibatch) and the server of one
// contiguous range of the nibble-reversed (hence uniform) key space:
//   owner(k) = floor(k * N / 2^64).
// The reference's sync_mode is a TODO (kvstore_dist.h:137-147); this is its bulk-synchronous
// (max_delay 0) schedule, made deterministic by applying pushes in worker-rank order:
//
//   worker  dist_localize     Localizer::Compact of its batch; sorted keys split by owner
//   --- alltoallv keys (+ occurrence counts in epoch 0) ---
//   owner   dist_owner_begin  merge the ranks' sorted key runs (stable: rank order within a key),
//                             find-or-insert their table slots; with counts, the ranks'
//                             Update(kFeaCount) pushes in rank order, then their InitV draws
//   owner   dist_owner_pull   SGDUpdater::Get per received key: record [V(d) | w | live | 0 0]
//   --- alltoallv records back ---
//   worker  dist_fwd_bwd      FMLoss Predict/Evaluate/AUC on its batch, CalcGrad into per-key
//                             gradient records [gV(d) | gw | 0 | 0 | 0]
//   --- alltoallv gradient records to the owners ---
//   owner   dist_owner_push   the ranks' Update(kGradient) pushes in rank order: per key,
//                             FTRL (+ AdaGrad if V was pulled) once per pushing rank; InitV
//                             draws in (rank, key) order, the order one server would meet them
//
// Every per-key result therefore equals what N reference servers produce when worker r's push
// reaches them r-th, with every pull of the step answered before any push.
#include <algorithm>
#include <cstdlib>

#include "fm_args.h"

namespace dfx {

constexpr int kDNT = 256;
constexpr int kMaxRanks = kMaxDistRanks;

// launchers shared with fm.hip / metric.hip
int launch_fwd_records(const FwdArgs& a, hipStream_t st, int* nblk);
int launch_bwd_positions(const BwdArgs& a, int64_t nseg_bound, hipStream_t st);
void sum_parts(Context* c, const double* part, int64_t n, double* out, bool accumulate);

__host__ __device__ inline int rec_floats(int d) { return d + 4; }

__device__ inline uint32_t owner_of(uint64_t k, uint32_t n) {
  return (uint32_t)__umul64hi(k, (uint64_t)n);
}

// offsets of each source rank's keys in the owner's receive buffer (kernel argument)
struct RankOffs {
  int n;
  int64_t off[kMaxRanks + 1];
};

__device__ inline int rank_of(const RankOffs& ro, int64_t i) {
  int lo = 0, hi = ro.n;  // off[lo] <= i < off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (ro.off[mid] <= i) lo = mid; else hi = mid;
  }
  return lo;
}

// ---- worker: split sorted unique keys by owner --------------------------------------------
// out[r] = first rank u of the sorted unique keys with owner(uniq[u]) >= r (r <= nranks, so
// out[nranks] = U), out[kMaxRanks + 1] = U
__global__ void k_owner_splits(const uint64_t* uniq, const DevState* lds, uint32_t nranks,
                               unsigned long long* out) {
  const uint32_t U = lds->u_count;
  const uint32_t r = threadIdx.x;
  if (r <= nranks) {
    uint32_t lo = 0, hi = U;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (owner_of(uniq[mid], nranks) < r) lo = mid + 1; else hi = mid;
    }
    out[r] = lo;
  }
  if (r == 0) out[kMaxRanks + 1] = U;
}

__global__ void k_dist_worker_finalize(DevState* ds, int64_t B) {
  ds->prog[0] += (double)B;  // sgd::Progress of this worker (sgd_learner.cc:213-229)
  ds->prog[1] += ds->scratch[3];  // the AUC lane adds prog[2] itself
}

// ---- owner: received keys -> unique segments (sort.hip merge_runs: stable tile merges)

__global__ void k_dist_heads(const uint64_t* K, int64_t R, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R) return;
  flags[i] = (i == 0 || K[i] != K[i - 1]) ? 1u : 0u;
}

// segstart[seg], segslot[seg] (find-or-insert), seg_of[received index], sorted_idx[sorted
// position] = received index (P == NULL: identity).  *total = number of unique keys.
__global__ __launch_bounds__(kDNT) void k_dist_segs(const uint64_t* K, const uint32_t* P,
                                                    int64_t R, DevState* ds,
                                                    const uint32_t* excl, const uint32_t* total,
                                                    Table T, uint32_t* segstart,
                                                    uint32_t* segslot, uint32_t* seg_of,
                                                    uint32_t* sorted_idx) {
  const int64_t i = (int64_t)blockIdx.x * kDNT + threadIdx.x;
  int ins = 0;
  if (i < R) {
    const bool head = (i == 0 || K[i] != K[i - 1]);
    const uint32_t seg = head ? excl[i] : excl[i] - 1u;  // excl[i] = heads before i
    const uint32_t src = P ? P[i] : (uint32_t)i;
    sorted_idx[i] = src;
    seg_of[src] = seg;
    if (head) {
      segstart[seg] = (uint32_t)i;
      bool inserted;
      int64_t s = tbl_insert(T, K[i], &inserted);
      if (s < 0) atomicOr(&ds->err, insert_error(s));
      ins = inserted;
      segslot[seg] = s < 0 ? kNoSlot : (uint32_t)s;
    }
    if (i == R - 1) segstart[*total] = (uint32_t)R;
  }
  for (int off = 32; off > 0; off >>= 1) ins += __shfl_xor(ins, off, kWave);
  if (lane_id() == 0 && ins) atomicAdd(&ds->n_keys, (unsigned long long)ins);
}

// k_dist_segs and SGDUpdater::Get (sgd_updater.cc:34-58) in one pass, for a step with no
// count push between the owner's find-or-insert and its pull: a group of G lanes per received
// key.  Lane 0 keeps the segment books and finds-or-inserts the key (a repeat of a key sent by
// several ranks finds the slot its head inserted: tbl_insert is safe against concurrent
// inserts of one key); the group then writes the key's pull record [V(d) | w | live | 0 0] at
// the key's received index.  d % 4 == 0.
template <int G>
__global__ __launch_bounds__(kDNT) void k_dist_segs_pull(
    const uint64_t* __restrict__ K, const uint32_t* __restrict__ P, int64_t R, DevState* ds,
    const uint32_t* __restrict__ excl, const uint32_t* total, Table T, Params Pp,
    uint32_t* segstart, uint32_t* segslot, uint32_t* sorted_idx, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * (kDNT / G) + threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int leader = (lane_id() / G) * G;
  int ins = 0;
  uint32_t slot = 0, src = 0;
  int2 wr = make_int2(0, -1);
  int found = 0;  // the key sat at its home slot: wr already holds its {w, vrow}
  if (i < R && l == 0) {
    const uint64_t k = K[i];
    const bool head = (i == 0 || k != K[i - 1]);
    const uint32_t seg = head ? excl[i] : excl[i] - 1u;
    src = P ? P[i] : (uint32_t)i;
    sorted_idx[i] = src;
    // the home entry's {w, vrow} and key in one trip (w / vrow of a slot are not written in
    // this kernel, and a fresh slot already holds the zero state)
    const uint64_t hh = tbl_hash(k, T);
    wr = *reinterpret_cast<const int2*>(ent_at(T, hh));
    bool inserted = false;
    int64_t s = (int64_t)hh;
    if (ent_at(T, hh)->key == k) {
      found = 1;
    } else {
      s = tbl_insert(T, k, &inserted);
    }
    if (s < 0) atomicOr(&ds->err, insert_error(s));
    slot = s < 0 ? kNoSlot : (uint32_t)s;
    ins = inserted;  // whichever of the key's items won the insert
    if (head) {
      segstart[seg] = (uint32_t)i;
      segslot[seg] = slot;
    }
    if (i == R - 1) segstart[*total] = (uint32_t)R;
  }
  slot = (uint32_t)__shfl((int)slot, leader, kWave);
  src = (uint32_t)__shfl((int)src, leader, kWave);
  found = __shfl(found, leader, kWave);
  wr.x = __shfl(wr.x, leader, kWave);
  wr.y = __shfl(wr.y, leader, kWave);
  if (i < R) {
    const int d = T.d, nc = d >> 2;
    if (!found)  // {w, vrow}; a key that could not be inserted reads as absent
      wr = slot == kNoSlot ? make_int2(0, -1) : *reinterpret_cast<const int2*>(ent_at(T, slot));
    const float w = __int_as_float(wr.x);
    const int vr = wr.y;
    const bool live = vr >= 0 && !(Pp.l1_shrk && w == 0.f);
    float4* o = reinterpret_cast<float4*>(out + (int64_t)src * rec_floats(d));
    const float4* V = reinterpret_cast<const float4*>(live ? row_V(T, vr) : T.V);
    for (int c = l; c < nc; c += G) o[c] = live ? V[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (l == 0) o[nc] = make_float4(w, live ? 1.f : 0.f, 0.f, 0.f);
  }
  for (int off = 32; off > 0; off >>= 1) ins += __shfl_xor(ins, off, kWave);
  if (lane_id() == 0 && ins) atomicAdd(&ds->n_keys, (unsigned long long)ins);
}

// The ranks' Update(kFeaCount) pushes in rank order (sgd_updater.cc:64-75), per owned key:
// fea_cnt += count; InitV once V is absent, w != 0 and fea_cnt > V_threshold.  frank[u] = the
// pushing rank whose Update draws the key's InitV.
__global__ void k_dist_feacnt(const uint32_t* segstart, const uint32_t* segslot,
                              const uint32_t* sorted_idx, const float* recv_cnt, RankOffs ro,
                              Table T, Params P, const uint32_t* nuniq, uint32_t* flags,
                              uint32_t* frank, uint32_t* fcount) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (int64_t)*nuniq) return;
  if (segslot[u] == kNoSlot) {  // not inserted (the error word says why): no update
    flags[u] = 0;
    frank[u] = 0;
    return;
  }
  Entry* e = ent_at(T, segslot[u]);
  float4 st = ent_state(e);  // {w, sqrt_g, z, fea_cnt}
  bool has_v = e->vrow >= 0;
  uint32_t f = 0, fr = 0;
  for (uint32_t i = segstart[u]; i < segstart[u + 1]; ++i) {
    const uint32_t src = sorted_idx[i];
    st.w += recv_cnt[src];
    if (P.V_dim > 0 && !has_v && st.x != 0.f && st.w > (float)P.V_threshold) {
      has_v = true;
      f = 1;
      fr = (uint32_t)rank_of(ro, src);
    }
  }
  e->fea_cnt = st.w;
  flags[u] = f;
  frank[u] = fr;
  if (f) atomicAdd(fcount, 1u);  // gates the InitV pass
}

// The ranks' Update(kGradient) pushes in rank order (sgd_updater.cc:76-100): per pushing rank,
// UpdateW (FTRL) and, when the rank pulled V (lens > 1: the record's live slot), UpdateV
// (AdaGrad).  A V pulled by any rank exists at push time (V rows are never freed).
__global__ void k_dist_push(const uint32_t* segstart, const uint32_t* segslot,
                            const uint32_t* sorted_idx, const float* g, RankOffs ro, Table T,
                            Params P, const uint32_t* nuniq, uint32_t* flags, uint32_t* frank,
                            DevState* ds, uint32_t* fcount) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int dnew = 0, nf = 0;
  if (u < (int64_t)*nuniq && segslot[u] == kNoSlot) {  // not inserted: no update
    flags[u] = 0;
    frank[u] = 0;
  } else if (u < (int64_t)*nuniq) {
    const int d = T.d;
    const int64_t S = rec_floats(d);
    Entry* en = ent_at(T, segslot[u]);
    float4 e = ent_state(en);
    const int vr = en->vrow;
    bool has_v = vr >= 0;
    float* V = has_v ? row_V(T, vr) : nullptr;
    float* C = has_v ? row_C(T, vr) : nullptr;
    uint32_t f = 0, fr = 0;
    for (uint32_t i = segstart[u]; i < segstart[u + 1]; ++i) {
      const uint32_t src = sorted_idx[i];
      const float* gr = g + (int64_t)src * S;
      bool tr;
      dnew += ftrl_update(P, gr[d], &e, &tr);
      if (tr && d > 0 && !has_v && e.w > (float)P.V_threshold) {  // :118-121
        has_v = true;
        f = 1;
        fr = (uint32_t)rank_of(ro, src);
      }
      if (d > 0 && gr[d + 1] != 0.f && V)
        for (int k = 0; k < d; ++k) adagrad_update(P, gr[k], V + k, C + k);
    }
    ent_set_state(en, e);
    flags[u] = f;
    frank[u] = fr;
    nf = (int)f;
  }
  for (int off = 32; off > 0; off >>= 1) {
    dnew += __shfl_xor(dnew, off, kWave);
    nf += __shfl_xor(nf, off, kWave);
  }
  if (lane_id() == 0 && dnew)
    atomicAdd((unsigned long long*)&ds->new_w, (unsigned long long)(long long)dnew);
  if (lane_id() == 0 && nf) atomicAdd(fcount, (uint32_t)nf);
}

// flagged keys (key order) -> (rank, key) order: rank keys, segment payloads (the sort that
// follows reads the first *ftotal of them).  Strided over a capped grid.
__global__ void k_dist_initv_list(const uint32_t* flags_excl, const uint32_t* ftotal,
                                  const uint32_t* frank, const uint32_t* nuniq, int64_t bound,
                                  uint32_t* rk, uint32_t* rv) {
  const uint32_t F = *ftotal;
  if (F == 0) return;  // no InitV this step (the steady state)
  const int64_t n = std::min<int64_t>(*nuniq, bound);
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n;
       u += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t e = flags_excl[u];
    const uint32_t nx = (u + 1 < n) ? flags_excl[u + 1] : F;
    if (nx != e) {
      rk[e] = frank[u];
      rv[e] = (uint32_t)u;
    }
  }
}

// InitV (sgd_updater.cc:144-152) of the q-th draw: seed jumped 3*d*q steps, pool row n_vrows+q
__global__ void k_dist_initv(const uint32_t* rv0, const uint32_t* rv1, const uint32_t* ftotal,
                             const uint32_t* segslot, Table T, float scale, DevState* ds,
                             const unsigned int* sortmeta) {
  const int64_t F = (int64_t)*ftotal;
  const uint32_t* rv = sortmeta[31] ? rv1 : rv0;
  const int d = T.d;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < F;
       q += (int64_t)gridDim.x * blockDim.x) {
    uint32_t s = lcg_advance(ds->seed, 3ull * (uint64_t)d * (uint64_t)q);
    const int64_t vr = initv_row(T, ds->n_vrows, q, segslot[rv[q]]);
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
    ent_at(T, segslot[rv[q]])->vrow = (int32_t)vr;
  }
}

__global__ void k_dist_initv_finalize(const uint32_t* ftotal, int d, int64_t vcap,
                                      DevState* ds, uint32_t* fcount) {
  const uint32_t F = *ftotal;
  *fcount = 0u;  // the flag count of the next Update of this slot
  ds->seed = lcg_advance(ds->seed, 3ull * (uint64_t)d * F);
  const unsigned long long nv = ds->n_vrows + F;
  ds->n_vrows = nv > (unsigned long long)vcap ? (unsigned long long)vcap : nv;
}

// SGDUpdater::Get (sgd_updater.cc:34-58) per received key, in received order
__global__ void k_dist_pull(int64_t R, const uint32_t* seg_of, const uint32_t* segslot,
                            Table T, Params P, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R) return;
  const int d = T.d;
  const uint32_t sl = segslot[seg_of[i]];
  const float w = sl == kNoSlot ? 0.f : ent_at(T, sl)->w;
  const int vr = sl == kNoSlot ? -1 : ent_at(T, sl)->vrow;
  const bool live = vr >= 0 && !(P.l1_shrk && w == 0.f);
  float* o = out + i * rec_floats(d);
  const float* V = live ? row_V(T, vr) : nullptr;
  for (int k = 0; k < d; ++k) o[k] = live ? V[k] : 0.f;
  o[d] = w;
  o[d + 1] = live ? 1.f : 0.f;
  o[d + 2] = 0.f;
  o[d + 3] = 0.f;
}

// d % 4 == 0: a group of G lanes per key, float4 chunks of V / Vaux / records
template <int G>
__global__ __launch_bounds__(kDNT) void k_dist_pull_vec(int64_t R, const uint32_t* seg_of,
                                                        const uint32_t* segslot, Table T,
                                                        Params P, float* out) {
  const int64_t i = (int64_t)blockIdx.x * (kDNT / G) + threadIdx.x / G;
  const int l = threadIdx.x % G;
  if (i >= R) return;
  const int d = T.d, nc = d >> 2;
  const uint32_t sl = segslot[seg_of[i]];
  const int2 wr = sl == kNoSlot ? make_int2(0, -1)
                                : *reinterpret_cast<const int2*>(ent_at(T, sl));  // {w, vrow}
  const float w = __int_as_float(wr.x);
  const int vr = wr.y;
  const bool live = vr >= 0 && !(P.l1_shrk && w == 0.f);
  float4* o = reinterpret_cast<float4*>(out + i * (int64_t)rec_floats(d));
  const float4* V = reinterpret_cast<const float4*>(live ? row_V(T, vr) : T.V);
  for (int c = l; c < nc; c += G) o[c] = live ? V[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  if (l == 0) o[nc] = make_float4(w, live ? 1.f : 0.f, 0.f, 0.f);
}

// The loads run in three dependency levels, each level's loads issued together: the key's
// segment bounds and slot; its table entry and its first pushing rank's record index; then
// its V / Vaux chunk and that record's gradient chunk and {gw, pulled}.  A key pushed by more
// than one rank (N > 1) reads its later records in the rank loop.
template <int G>
__global__ __launch_bounds__(kDNT) void k_dist_push_vec(const uint32_t* __restrict__ segstart,
                                                        const uint32_t* __restrict__ segslot,
                                                        const uint32_t* __restrict__ sorted_idx,
                                                        const float* __restrict__ g, RankOffs ro,
                                                        Table T, Params P, const uint32_t* nuniq,
                                                        uint32_t* flags, uint32_t* frank,
                                                        DevState* ds, uint32_t* fcount) {
  const int64_t u = (int64_t)blockIdx.x * (kDNT / G) + threadIdx.x / G;
  const int l = threadIdx.x % G;
  int dnew = 0, nf = 0;
  const uint32_t sl = u < (int64_t)*nuniq ? segslot[u] : kNoSlot;
  if (u < (int64_t)*nuniq && sl == kNoSlot) {  // not inserted: no update
    if (l == 0) {
      flags[u] = 0;
      frank[u] = 0;
    }
  } else if (u < (int64_t)*nuniq) {
    const int d = T.d, nc = d >> 2;
    const int64_t S = rec_floats(d);
    // level 1
    const uint32_t s0 = segstart[u], s1 = segstart[u + 1];
    // level 2
    Entry* en = ent_at(T, sl);
    const float4 h = *reinterpret_cast<const float4*>(en);  // w, vrow, sqrt_g, z
    const float fc = en->fea_cnt;
    const uint32_t src0 = sorted_idx[s0];
    // level 3
    const int vr = __float_as_int(h.y);
    const float* g0 = g + (int64_t)src0 * S;
    const float2 gwp0 = *reinterpret_cast<const float2*>(g0 + d);  // {gw, pulled}
    float4* V4 = reinterpret_cast<float4*>(row_V(T, vr >= 0 ? vr : 0));
    float4* C4 = reinterpret_cast<float4*>(row_C(T, vr >= 0 ? vr : 0));
    const bool mine = vr >= 0 && l < nc;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = mine ? V4[l] : z4, cg = mine ? C4[l] : z4;
    const float4 gv0 = mine ? reinterpret_cast<const float4*>(g0)[l] : z4;
    // UpdateW per pushing rank (sgd_updater.cc:76-100, 105-131); every lane of the group runs
    // the same sequence
    float4 e = make_float4(h.x, h.z, h.w, fc);  // {w, sqrt_g, z, fea_cnt}
    bool has_v = vr >= 0;
    uint32_t f = 0, fr = 0;
    for (uint32_t i = s0; i < s1; ++i) {
      const uint32_t src = i == s0 ? src0 : sorted_idx[i];
      const float gw = i == s0 ? gwp0.x : g[(int64_t)src * S + d];
      bool tr;
      const int dw = ftrl_update(P, gw, &e, &tr);
      if (l == 0) dnew += dw;
      if (tr && d > 0 && !has_v && e.w > (float)P.V_threshold) {  // :118-121
        has_v = true;
        f = 1;
        fr = (uint32_t)rank_of(ro, src);
      }
    }
    if (l == 0) {
      ent_set_state(en, e);
      flags[u] = f;
      frank[u] = fr;
      nf = (int)f;
    }
    // UpdateV per pushing rank that pulled V (each coordinate independent)
    if (vr >= 0) {
      for (int c = l; c < nc; c += G) {
        if (c != l) {
          v = V4[c];
          cg = C4[c];
        }
        for (uint32_t i = s0; i < s1; ++i) {
          float4 gv;
          if (i == s0 && c == l) {
            if (gwp0.y == 0.f) continue;
            gv = gv0;
          } else {
            const float* gr = g + (int64_t)sorted_idx[i] * S;
            if (gr[d + 1] == 0.f) continue;
            gv = reinterpret_cast<const float4*>(gr)[c];
          }
          adagrad_update(P, gv.x, &v.x, &cg.x);
          adagrad_update(P, gv.y, &v.y, &cg.y);
          adagrad_update(P, gv.z, &v.z, &cg.z);
          adagrad_update(P, gv.w, &v.w, &cg.w);
        }
        V4[c] = v;
        C4[c] = cg;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    dnew += __shfl_xor(dnew, off, kWave);
    nf += __shfl_xor(nf, off, kWave);
  }
  if (lane_id() == 0 && dnew)
    atomicAdd((unsigned long long*)&ds->new_w, (unsigned long long)(long long)dnew);
  if (lane_id() == 0 && nf) atomicAdd(fcount, (uint32_t)nf);
}

// ---- aggregated push (push_agg=sum) -----------------------------------
// One step over N workers is one reference step over the concatenation of their batches: a
// key's gradient is the sum of the workers' gradient records (in rank order), applied by ONE
// Update (sgd_updater.cc:76-142) — UpdateW, and UpdateV when V was pulled (every worker of the
// step pulled the same state, so the records agree on `live`).  InitV requests are flagged in
// key order; their draws are ranked over all owners (k_dist_initv_sum), so the rand_r stream is
// the single reference updater's.
template <int G>
__global__ __launch_bounds__(kDNT) void k_dist_push_sum_vec(
    const uint32_t* __restrict__ segstart, const uint32_t* __restrict__ segslot,
    const uint32_t* __restrict__ sorted_idx, const float* __restrict__ g, Table T, Params P,
    const uint32_t* nuniq, uint32_t* flags, DevState* ds, uint32_t* fcount) {
  const int64_t u = (int64_t)blockIdx.x * (kDNT / G) + threadIdx.x / G;
  const int l = threadIdx.x % G;
  int dnew = 0, nf = 0;
  const uint32_t sl = u < (int64_t)*nuniq ? segslot[u] : kNoSlot;
  if (u < (int64_t)*nuniq && sl == kNoSlot) {  // not inserted: no update
    if (l == 0) flags[u] = 0;
  } else if (u < (int64_t)*nuniq) {
    const int d = T.d, nc = d >> 2;
    const int64_t S = rec_floats(d);
    const uint32_t s0 = segstart[u], s1 = segstart[u + 1];
    Entry* en = ent_at(T, sl);
    const float4 h = *reinterpret_cast<const float4*>(en);  // w, vrow, sqrt_g, z
    const float fc = en->fea_cnt;
    const uint32_t src0 = sorted_idx[s0];
    const float* g0 = g + (int64_t)src0 * S;
    const float2 gwp0 = *reinterpret_cast<const float2*>(g0 + d);  // {gw, pulled}
    const int vr = __float_as_int(h.y);
    float4* V4 = reinterpret_cast<float4*>(row_V(T, vr >= 0 ? vr : 0));
    float4* C4 = reinterpret_cast<float4*>(row_C(T, vr >= 0 ? vr : 0));
    const bool upd_v = vr >= 0 && gwp0.y != 0.f;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = upd_v && l < nc ? V4[l] : z4, cg = upd_v && l < nc ? C4[l] : z4;
    float4 gv = upd_v && l < nc ? reinterpret_cast<const float4*>(g0)[l] : z4;
    float gw = gwp0.x;
    for (uint32_t i = s0 + 1; i < s1; ++i) gw += g[(int64_t)sorted_idx[i] * S + d];
    float4 e = make_float4(h.x, h.z, h.w, fc);  // {w, sqrt_g, z, fea_cnt}
    bool tr;
    const int dw = ftrl_update(P, gw, &e, &tr);
    if (l == 0) {
      ent_set_state(en, e);
      dnew = dw;
      // InitV on a 0 -> nonzero transition (sgd_updater.cc:118-121); e.w is fea_cnt
      const bool need = tr && d > 0 && vr < 0 && e.w > (float)P.V_threshold;
      flags[u] = need ? 1u : 0u;
      nf = need ? 1 : 0;
    }
    if (upd_v) {
      for (int c = l; c < nc; c += G) {
        if (c != l) {
          v = V4[c];
          cg = C4[c];
          gv = reinterpret_cast<const float4*>(g0)[c];
        }
        for (uint32_t i = s0 + 1; i < s1; ++i) {
          const float4 q = reinterpret_cast<const float4*>(g + (int64_t)sorted_idx[i] * S)[c];
          gv.x += q.x; gv.y += q.y; gv.z += q.z; gv.w += q.w;
        }
        adagrad_update(P, gv.x, &v.x, &cg.x);
        adagrad_update(P, gv.y, &v.y, &cg.y);
        adagrad_update(P, gv.z, &v.z, &cg.z);
        adagrad_update(P, gv.w, &v.w, &cg.w);
        V4[c] = v;
        C4[c] = cg;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    dnew += __shfl_xor(dnew, off, kWave);
    nf += __shfl_xor(nf, off, kWave);
  }
  if (lane_id() == 0 && dnew)
    atomicAdd((unsigned long long*)&ds->new_w, (unsigned long long)(long long)dnew);
  if (lane_id() == 0 && nf) atomicAdd(fcount, (uint32_t)nf);
}

// the same for any V_dim (one lane per key)
__global__ void k_dist_push_sum(const uint32_t* segstart, const uint32_t* segslot,
                                const uint32_t* sorted_idx, const float* g, Table T, Params P,
                                const uint32_t* nuniq, uint32_t* flags, DevState* ds,
                                uint32_t* fcount) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int dnew = 0, nf = 0;
  if (u < (int64_t)*nuniq && segslot[u] == kNoSlot) {
    flags[u] = 0;
  } else if (u < (int64_t)*nuniq) {
    const int d = T.d;
    const int64_t S = rec_floats(d);
    Entry* en = ent_at(T, segslot[u]);
    float4 e = ent_state(en);
    const int vr = en->vrow;
    const uint32_t s0 = segstart[u], s1 = segstart[u + 1];
    const float* g0 = g + (int64_t)sorted_idx[s0] * S;
    float gw = g0[d];
    for (uint32_t i = s0 + 1; i < s1; ++i) gw += g[(int64_t)sorted_idx[i] * S + d];
    bool tr;
    dnew = ftrl_update(P, gw, &e, &tr);
    ent_set_state(en, e);
    if (vr >= 0 && g0[d + 1] != 0.f) {
      float* V = row_V(T, vr);
      float* C = row_C(T, vr);
      for (int k = 0; k < d; ++k) {
        float gk = g0[k];
        for (uint32_t i = s0 + 1; i < s1; ++i) gk += g[(int64_t)sorted_idx[i] * S + k];
        adagrad_update(P, gk, V + k, C + k);
      }
    }
    const bool need = tr && d > 0 && vr < 0 && e.w > (float)P.V_threshold;
    flags[u] = need ? 1u : 0u;
    nf = need ? 1 : 0;
  }
  for (int off = 32; off > 0; off >>= 1) {
    dnew += __shfl_xor(dnew, off, kWave);
    nf += __shfl_xor(nf, off, kWave);
  }
  if (lane_id() == 0 && dnew)
    atomicAdd((unsigned long long*)&ds->new_w, (unsigned long long)(long long)dnew);
  if (lane_id() == 0 && nf) atomicAdd(fcount, (uint32_t)nf);
}

__global__ void k_dist_initv_count(const uint32_t* ftotal, int64_t* out) {
  *out = (int64_t)*ftotal;
}

// InitV draws of this owner's flagged keys (key order), ranked after every lower owner's
// draws of this step: the q-th of them jumps the shared seed by 3*d*(sum_{h<rank} F_h + q)
__global__ __launch_bounds__(kDNT) void k_dist_initv_sum(const uint32_t* excl,
                                                         const uint32_t* ftotal,
                                                         const uint32_t* nuniq, int64_t bound,
                                                         const uint32_t* segslot,
                                                         const int64_t* Fall, int rank, Table T,
                                                         float scale, const DevState* ds) {
  const uint32_t F = *ftotal;
  if (F == 0) return;
  int64_t off = 0;
  for (int h = 0; h < rank; ++h) off += Fall[h];
  const int64_t n = std::min<int64_t>(*nuniq, bound);
  const int d = T.d;
  if (d > kIvMaxD) {  // (wide V: a row per thread)
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
      const uint32_t e = excl[u];
      const uint32_t nx = (u + 1 < n) ? excl[u + 1] : F;
      if (nx == e) continue;
      uint32_t s = lcg_advance(ds->seed, 3ull * (uint64_t)d * (uint64_t)(off + e));
      const int64_t vr = initv_row(T, ds->n_vrows, e, segslot[u]);
      if (vr >= T.vcap) continue;  // kErrPoolFull is set by the finalize
      float* V = row_V(T, vr);
      float* C = row_C(T, vr);
      for (int k = 0; k < d; ++k) {
        V[k] = initv_value(rand_r_dev(&s), scale);
        C[k] = 0.f;
      }
      ent_at(T, segslot[u])->vrow = (int32_t)vr;
    }
    return;
  }
  // per kDNT keys: the flagged ones listed (a block scan), then drawn a coordinate per thread
  __shared__ uint32_t s_st[kDNT], s_vr[kDNT], s_A[kIvMaxD], s_C[kIvMaxD];
  __shared__ uint32_t lds[kDNT / kWave + 1];
  for (int j = threadIdx.x; j < d; j += kDNT) lcg_jump(3ull * (uint64_t)j, &s_A[j], &s_C[j]);
  for (int64_t b0 = (int64_t)blockIdx.x * kDNT; b0 < n; b0 += (int64_t)gridDim.x * kDNT) {
    const int64_t u = b0 + threadIdx.x;
    uint32_t e = 0;
    bool f = false;
    if (u < n) {
      e = excl[u];
      f = ((u + 1 < n) ? excl[u + 1] : F) != e;
    }
    uint32_t cnt;
    const uint32_t at = block_excl_scan<kDNT>(f ? 1u : 0u, lds, &cnt);
    if (f) {
      const int64_t vr = initv_row(T, ds->n_vrows, e, segslot[u]);
      s_st[at] = lcg_advance(ds->seed, 3ull * (uint64_t)d * (uint64_t)(off + e));
      if (vr >= T.vcap) {
        s_vr[at] = 0xFFFFFFFFu;  // kErrPoolFull is set by the finalize
      } else {
        s_vr[at] = (uint32_t)vr;
        ent_at(T, segslot[u])->vrow = (int32_t)vr;
      }
    }
    __syncthreads();
    initv_draw_list<kDNT>(cnt, s_st, s_vr, d, scale, s_A, s_C,
                          [&](uint32_t r) { return row_V(T, r); },
                          [&](uint32_t r) { return row_C(T, r); });
    __syncthreads();
  }
}

__global__ void k_dist_initv_sum_finalize(const uint32_t* ftotal, const int64_t* Fall,
                                          int nranks, int d, int64_t vcap, DevState* ds,
                                          uint32_t* fcount) {
  int64_t tot = 0;
  for (int h = 0; h < nranks; ++h) tot += Fall[h];
  const uint32_t F = *ftotal;
  *fcount = 0u;
  ds->seed = lcg_advance(ds->seed, 3ull * (uint64_t)d * (uint64_t)tot);
  const unsigned long long nv = ds->n_vrows + F;
  if (nv > (unsigned long long)vcap) atomicOr(&ds->err, kErrPoolFull);
  ds->n_vrows = nv > (unsigned long long)vcap ? (unsigned long long)vcap : nv;
}

// ---- the split owner's ranked InitV in two launches (round 6; was a three-launch scan, a count
// kernel, the draws and a finalize: six launches on the critical path of every step, even in
// the steady state where the backward flagged nothing and every launch exits at once).
//   count: per tile of kIvrTile flags its count (ts[tile]); the last block (a ticket per block)
//          sums them into this owner's F — the request count the owners all-gather
//   draw:  per tile its exclusive prefix from ts, per chunk of kIvrNT flags a block scan, then the
//          listed keys drawn a coordinate per thread at their rank over all owners (off + e);
//          the last block advances the shared seed by every owner's draws and the V pool by F
// The draws equal k_dist_initv_sum's (the same rank per key, the same rand_r jump); the tiles'
// counts cross blocks through agent-scope atomics, as the look-back words do (lookback.h)
constexpr int kIvrTile = 4096, kIvrNT = 256, kIvrGrid = 256;

__device__ inline int64_t ivr_n(const uint32_t* nuniq, int64_t bound) {
  const int64_t n = (int64_t)*nuniq;
  return n < bound ? n : bound;
}

// the block's last-block ticket: true in every thread of the block that took the last ticket.
// No fence: what crosses blocks goes through agent-scope atomics (a device-scope fence per
// block would write back its XCD's L2, store.hip k_initv_onepass)
__device__ inline bool ivr_last_block(unsigned* ticket, bool* s_last) {
  __syncthreads();
  if (threadIdx.x == 0) *s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  return *s_last;
}

__global__ __launch_bounds__(kIvrNT) void k_initv_rank_count(const uint32_t* flags, int64_t bound,
                                                             const uint32_t* nuniq,
                                                             const uint32_t* gate, uint32_t* ts,
                                                             uint32_t* ftotal, int64_t* count_out,
                                                             unsigned* ticket) {
  __shared__ uint32_t lds[kIvrNT / kWave + 1];
  __shared__ bool s_last;
  if (gate && *gate == 0u) {  // no key flagged this step (the steady state): F = 0
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *ftotal = 0u;
      *count_out = 0;
    }
    return;
  }
  const int64_t n = ivr_n(nuniq, bound);
  const int64_t ntiles = (n + kIvrTile - 1) / kIvrTile;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t b0 = tile * kIvrTile;
    uint32_t f = 0;
    for (int i = threadIdx.x; i < kIvrTile; i += kIvrNT) {
      const int64_t u = b0 + i;
      f += (u < n && flags[u]) ? 1u : 0u;
    }
    uint32_t tot;
    (void)block_excl_scan<kIvrNT>(f, lds, &tot);
    if (threadIdx.x == 0)
      __hip_atomic_store(ts + tile, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!ivr_last_block(ticket, &s_last)) return;
  uint32_t f = 0;
  for (int64_t i = threadIdx.x; i < ntiles; i += kIvrNT)
    f += __hip_atomic_load(ts + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t F;
  (void)block_excl_scan<kIvrNT>(f, lds, &F);
  if (threadIdx.x == 0) {
    *ftotal = F;
    *count_out = (int64_t)F;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(kIvrNT) void k_initv_rank_draw(
    const uint32_t* flags, int64_t bound, const uint32_t* nuniq, const uint32_t* ftotal,
    const uint32_t* ts, const uint32_t* segslot, const int64_t* Fall, int rank, int nranks,
    Table T, float scale, DevState* ds, int64_t vcap, uint32_t* fcount, unsigned* ticket,
    unsigned long long* cap_host) {
  __shared__ uint32_t lds[kIvrNT / kWave + 1];
  __shared__ uint32_t s_st[kIvrNT], s_vr[kIvrNT], s_A[kIvMaxD], s_C[kIvMaxD];
  __shared__ bool s_last;
  int64_t tot = 0, off = 0;
  for (int h = 0; h < nranks; ++h) {
    tot += Fall[h];
    if (h < rank) off += Fall[h];
  }
  if (tot == 0) {  // no owner draws: nothing advances (the gate's reset only)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *fcount = 0u;
      if (cap_host) {  // the capacity guard's counts (pinned host words)
        cap_host[0] = ds->n_keys;
        cap_host[1] = ds->n_vrows;
      }
    }
    return;
  }
  const uint32_t F = *ftotal;
  const int d = T.d;
  if (F > 0) {
    for (int j = threadIdx.x; j < d && j < kIvMaxD; j += kIvrNT)
      lcg_jump(3ull * (uint64_t)j, &s_A[j], &s_C[j]);
    const int64_t n = ivr_n(nuniq, bound);
    const int64_t ntiles = (n + kIvrTile - 1) / kIvrTile;
    const uint32_t seed = ds->seed;
    const uint64_t nv0 = ds->n_vrows;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      uint32_t pre = 0;  // the tile's exclusive prefix: the counts of the tiles before it
      for (int64_t i = threadIdx.x; i < tile; i += kIvrNT)
        pre += __hip_atomic_load(ts + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t base;
      (void)block_excl_scan<kIvrNT>(pre, lds, &base);
      if (__hip_atomic_load(ts + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) continue;
      const int64_t b0 = tile * kIvrTile;
      for (int c0 = 0; c0 < kIvrTile; c0 += kIvrNT) {
        const int64_t u = b0 + c0 + threadIdx.x;
        const bool f = u < n && flags[u] != 0u;
        uint32_t cnt;
        const uint32_t at = block_excl_scan<kIvrNT>(f ? 1u : 0u, lds, &cnt);
        if (f) {
          const uint32_t e = base + at;
          uint32_t st = lcg_advance(seed, 3ull * (uint64_t)d * (uint64_t)(off + e));
          const int64_t vr = initv_row(T, nv0, e, segslot[u]);
          if (vr >= T.vcap) {
            s_vr[at] = 0xFFFFFFFFu;  // kErrPoolFull: set by the last block
          } else {
            s_vr[at] = (uint32_t)vr;
            ent_at(T, segslot[u])->vrow = (int32_t)vr;
            if (d > kIvMaxD) {  // (wide V: the row by its own thread)
              float* V = row_V(T, vr);
              float* C = row_C(T, vr);
              for (int k = 0; k < d; ++k) {
                V[k] = initv_value(rand_r_dev(&st), scale);
                C[k] = 0.f;
              }
            }
          }
          s_st[at] = st;
        }
        __syncthreads();
        if (d <= kIvMaxD)
          initv_draw_list<kIvrNT>(cnt, s_st, s_vr, d, scale, s_A, s_C,
                                  [&](uint32_t r) { return row_V(T, r); },
                                  [&](uint32_t r) { return row_C(T, r); });
        base += cnt;
        __syncthreads();
      }
    }
  }
  // the last block: every owner's draws advance the shared seed, this owner's F the pool
  if (!ivr_last_block(ticket, &s_last) || threadIdx.x != 0) return;
  __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *fcount = 0u;
  ds->seed = lcg_advance(ds->seed, 3ull * (uint64_t)d * (uint64_t)tot);
  const unsigned long long nv = ds->n_vrows + F;
  if (nv > (unsigned long long)vcap) atomicOr(&ds->err, kErrPoolFull);
  ds->n_vrows = nv > (unsigned long long)vcap ? (unsigned long long)vcap : nv;
  if (cap_host) {
    cap_host[0] = ds->n_keys;
    cap_host[1] = ds->n_vrows;
  }
}

int initv_rank_count(const Lane& L, uint32_t* flags, int64_t bound, const uint32_t* nuniq,
                     uint32_t* ftotal, const uint32_t* gate, int64_t* count_dev) {
  const int64_t ntiles = std::max<int64_t>(1, (bound + kIvrTile - 1) / kIvrTile);
  DFX_TRY(L.ws->tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  const dim3 g((unsigned)std::min<int64_t>(ntiles, kIvrGrid));
  hipLaunchKernelGGL(k_initv_rank_count, g, dim3(kIvrNT), 0, L.stream, flags, bound, nuniq, gate,
                     L.ws->tiles.as<uint32_t>(), ftotal, count_dev, &L.ds->ivr_ticket[0]);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int initv_rank_draw(Context* c, const Lane& L, const uint32_t* flags, const uint32_t* ftotal,
                    const uint32_t* nuniq, int64_t bound, const uint32_t* segslot,
                    const int64_t* counts_all, int rank, int nranks, uint32_t* fcount,
                    unsigned long long* cap_host) {
  const int64_t ntiles = std::max<int64_t>(1, (bound + kIvrTile - 1) / kIvrTile);
  DFX_TRY(L.ws->tiles.ensure(sizeof(uint32_t) * (ntiles + 1)));
  const dim3 g((unsigned)std::min<int64_t>(ntiles, kIvrGrid));
  hipLaunchKernelGGL(k_initv_rank_draw, g, dim3(kIvrNT), 0, L.stream, flags, bound, nuniq, ftotal,
                     L.ws->tiles.as<uint32_t>(), segslot, counts_all, rank, nranks, c->T,
                     c->P.V_init_scale, c->ds, c->T.vcap, fcount, &L.ds->ivr_ticket[1], cap_host);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// ---- union-indexed collectives (the north_star's literal reduce-scatter / all-gather) -------
// The union of every worker's keys, sorted: union[excl[i]] = K[i] at run heads; upos[src] =
// the union position of the item the merge took from source index src
__global__ void k_union_write(const uint64_t* K, const uint32_t* P, const uint32_t* excl,
                              int64_t R, uint64_t* uni, uint32_t* upos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R) return;
  const bool head = i == 0 || K[i] != K[i - 1];
  const uint32_t u = head ? excl[i] : excl[i] - 1u;
  if (head) uni[u] = K[i];
  upos[P ? P[i] : (uint32_t)i] = u;
}

// out[r] = first union position owned by rank >= r (r <= nranks)
__global__ void k_union_bounds(const uint64_t* uni, const uint32_t* n_uni, uint32_t nranks,
                               int64_t* out) {
  const uint32_t r = threadIdx.x;
  if (r > nranks) return;
  uint32_t lo = 0, hi = *n_uni;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (owner_of(uni[mid], nranks) < r) lo = mid + 1; else hi = mid;
  }
  out[r] = lo;
}

struct Bounds {
  int n;
  int64_t b[kMaxRanks + 1];
};

// a worker's key i <-> row (owner g) * M + (union position - bounds[g]) of a union-indexed,
// owner-chunked buffer.  to_union: scatter src (the worker's rows) into dst (union rows);
// else gather dst (the worker's rows) from src (union rows)
__global__ void k_union_rows(const uint64_t* keys, const uint32_t* upos, int64_t U, Bounds bd,
                             int64_t M, int width, int to_union, const float* src, float* dst) {
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x / 4) + threadIdx.x / 4;
  const int l = threadIdx.x % 4;
  if (i >= U) return;
  const uint32_t g = owner_of(keys[i], (uint32_t)bd.n);
  const int64_t row = (int64_t)g * M + ((int64_t)upos[i] - bd.b[g]);
  const float* a = to_union ? src + i * width : src + row * width;
  float* b = to_union ? dst + row * width : dst + i * width;
  for (int k = l; k < width; k += 4) b[k] = a[k];
}

static int vec_group(int d) {
  if (d <= 0 || d % 4 != 0) return 0;
  int g = 1;
  while (g < d / 4 && g < 64) g <<= 1;
  return g;
}

#define DFX_DIST_GROUPS(X) X(1) X(2) X(4) X(8) X(16) X(32) X(64)

// the owner lane of a step slot: the main stream with the slot's owner buffers and state
static Lane owner_lane(Context* c, int slot) {
  return Lane{c->stream, &c->ows[slot], c->ods[slot], &c->ds->err};
}

// InitV of the flagged keys in (pushing rank, key) order, all on the device
static int owner_initv(Context* c, int slot, int nranks) {
  const Lane OL = owner_lane(c, slot);
  Workspace& ws = *OL.ws;
  const int64_t R = c->dist_R[slot];
  uint32_t* flags = ws.oflags.as<uint32_t>();
  uint32_t* nuniq = &OL.ds->totals[1];
  uint32_t* ftotal = &OL.ds->totals[2];
  uint32_t* fcount = &OL.ds->totals[3];
  // gated on the device by the flag count: the scan, the sort and the draws exit at once
  // when no key asked for V (the steady state)
  DFX_TRY(scan_u32(OL, flags, R, ftotal, nuniq, fcount));
  uint32_t* rk0 = ws.vals0.as<uint32_t>();
  uint32_t* rv0 = ws.vals1.as<uint32_t>();
  uint32_t* rk1 = reinterpret_cast<uint32_t*>(ws.keys0.as<uint64_t>());
  uint32_t* rv1 = reinterpret_cast<uint32_t*>(ws.keys1.as<uint64_t>());
  const dim3 grid((R + kDNT - 1) / kDNT);
  const dim3 igrid((unsigned)std::min<int64_t>((R + kDNT - 1) / kDNT, 1024));
  hipLaunchKernelGGL(k_dist_initv_list, igrid, dim3(kDNT), 0, OL.stream, flags, ftotal,
                     ws.ofrank.as<uint32_t>(), nuniq, R, rk0, rv0);
  int bits = 0;
  while ((1 << bits) < nranks) ++bits;
  // stable by rank, over the *ftotal flagged keys
  DFX_TRY(radix_sort_pairs<uint32_t>(OL, rk0, rv0, rk1, rv1, R, 0, bits > 0 ? 8 : 0, nullptr,
                                     OL.ds->sortmeta, ftotal));
  hipLaunchKernelGGL(k_dist_initv, igrid, dim3(kDNT), 0, OL.stream, rv0, rv1, ftotal,
                     ws.osegslot.as<uint32_t>(), c->T, c->P.V_init_scale, c->ds,
                     OL.ds->sortmeta);
  hipLaunchKernelGGL(k_dist_initv_finalize, dim3(1), dim3(1), 0, OL.stream, ftotal, c->P.V_dim,
                     c->T.vcap, c->ds, fcount);
  return DFX_OK;
}

// the owner's segments of a slot (find-or-insert of every received key), when still pending
static void owner_segs(Context* c, int slot) {
  if (!c->dist_segs_pending[slot]) return;
  c->dist_segs_pending[slot] = false;
  const Lane OL = owner_lane(c, slot);
  Workspace& ws = *OL.ws;
  const int64_t R = c->dist_R[slot];
  hipLaunchKernelGGL(k_dist_segs, dim3((R + kDNT - 1) / kDNT), dim3(kDNT), 0, OL.stream,
                     c->dist_K[slot], c->dist_P[slot], R, c->ds, ws.oflags.as<uint32_t>(),
                     &OL.ds->totals[1], c->T, ws.osegstart.as<uint32_t>(),
                     ws.osegslot.as<uint32_t>(), ws.oseg_of.as<uint32_t>(),
                     ws.osorted.as<uint32_t>());
}

static RankOffs rank_offs(const Context* c, int slot) {
  RankOffs ro{};
  ro.n = (int)c->dist_offs[slot].size() - 1;
  for (int r = 0; r <= ro.n; ++r) ro.off[r] = c->dist_offs[slot][r];
  return ro;
}

}  // namespace dfx

using namespace dfx;

extern "C" {

int dfx_dist_record_floats(dfx_ctx* ctx) { return ctx ? rec_floats(ctx->c.P.V_dim) : -1; }

#define DFX_CHECK_SLOT(slot) DFX_CHECK_ARG((slot) >= 0 && (slot) < kSlots, "dist: slot must be 0 .. 3")

// Localizer lane: Compact of the batch into the slot's buffers, then the owner splits, copied
// to pinned memory; dfx_dist_localize_wait joins it on the host
int dfx_dist_localize(dfx_ctx* ctx, const dfx_batch* b, uint64_t max_index, int nranks,
                      int slot, uint64_t* keys_out, float* cnt_out) {
  DFX_CHECK_ARG(ctx && b, "null argument");
  DFX_CHECK_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxRanks, "dist: 1 <= nranks <= 64");
  DFX_CHECK_ARG(b->size >= 0 && b->nnz >= 0, "dist_localize: negative sizes");
  DFX_CHECK_ARG(b->size == 0 || b->offset, "dist_localize: null offset");
  DFX_CHECK_ARG(b->nnz == 0 || (b->index && keys_out), "dist_localize: null buffer");
  Context* c = &ctx->c;
  DFX_TRY(pipeline_init(c));
  const int64_t B = b->size, nnz = b->nnz;
  DFX_TRY(ws_reserve(c, B, nnz));
  Workspace& bw = c->bws[slot];
  DFX_TRY(loc_reserve(bw, nnz, c->loc_stream));
  DFX_TRY(bw.ofrank.ensure((kMaxRanks + 2) * 8));
  const Lane LL{c->loc_stream, &bw, c->bds[slot], &c->ds->err};
  // the batch is ready on the caller's (input) stream; the slot's buffers are free once the
  // main stream passed the dfx_dist_fwd_bwd that read them
  DFX_HIP(hipEventRecord(c->ev_in, c->has_in_stream ? c->in_stream : c->stream));
  DFX_HIP(hipStreamWaitEvent(c->loc_stream, c->ev_in, 0));
  DFX_HIP(hipStreamWaitEvent(c->loc_stream, c->ev_free[slot], 0));
  LocOut o;
  o.uniq = keys_out;
  o.cnt = cnt_out;
  o.col = bw.col.as<uint32_t>();
  o.segstart = bw.segstart.as<uint32_t>();
  o.value = b->value;
  o.occ_row = bw.occ_row.as<uint32_t>();
  o.occ_x = b->value ? bw.occ_x.as<float>() : nullptr;
  DFX_TRY(localize_run(c, LL, B, nnz, b->offset, b->index, max_index, o));
  unsigned long long* splits = bw.ofrank.as<unsigned long long>();
  hipLaunchKernelGGL(k_owner_splits, dim3(1), dim3(kMaxRanks + 1), 0, c->loc_stream,
                     keys_out, c->bds[slot], (uint32_t)nranks, splits);
  DFX_HIP(hipMemcpyAsync(c->dist_host[slot], splits, (kMaxRanks + 2) * 8,
                         hipMemcpyDeviceToHost, c->loc_stream));
  DFX_HIP(hipEventRecord(c->ev_loc[slot], c->loc_stream));
  DFX_HIP(hipGetLastError());
  c->dist_rows[slot] = B;
  c->dist_U[slot] = -1;  // known after dfx_dist_localize_wait
  return DFX_OK;
}

int dfx_dist_localize_wait(dfx_ctx* ctx, int slot, int nranks, int64_t* split_counts,
                           int64_t* n_uniq) {
  DFX_CHECK_ARG(ctx && split_counts && n_uniq, "null argument");
  DFX_CHECK_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxRanks, "dist: 1 <= nranks <= 64");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(c->loc_stream, "dist_localize_wait: no dfx_dist_localize issued");
  DFX_HIP(hipEventSynchronize(c->ev_loc[slot]));
  const unsigned long long* h = c->dist_host[slot];
  for (int r = 0; r < nranks; ++r) split_counts[r] = (int64_t)(h[r + 1] - h[r]);
  *n_uniq = (int64_t)h[kMaxRanks + 1];
  c->dist_U[slot] = *n_uniq;
  return DFX_OK;
}

int dfx_dist_fwd_bwd(dfx_ctx* ctx, int slot, const dfx_batch* b, const float* pulled,
                     int job_type, float* grads_out, float* pred_out) {
  DFX_CHECK_ARG(ctx && b, "null argument");
  DFX_CHECK_SLOT(slot);
  DFX_CHECK_ARG(job_type == DFX_JOB_TRAINING || job_type == DFX_JOB_VALIDATION ||
                    job_type == DFX_JOB_PREDICTION,
                "dist_fwd_bwd: bad job type");
  Context* c = &ctx->c;
  Workspace& ws = c->ws;
  Workspace& bw = c->bws[slot];
  const int d = c->P.V_dim;
  const int64_t B = b->size;
  DFX_CHECK_ARG(c->dist_U[slot] >= 0, "dist_fwd_bwd: dfx_dist_localize_wait first");
  DFX_CHECK_ARG(B == c->dist_rows[slot], "dist_fwd_bwd: batch differs from dist_localize's");
  DFX_CHECK_ARG(B == 0 || b->label, "dist_fwd_bwd: null label");
  const int64_t U = c->dist_U[slot];
  DFX_CHECK_ARG(U == 0 || pulled, "dist_fwd_bwd: null pulled records");
  const bool train = job_type == DFX_JOB_TRAINING && U > 0;
  DFX_CHECK_ARG(!train || grads_out, "dist_fwd_bwd: grads_out required for training");
  const int64_t S = rec_floats(d);
  float* pred = pred_out ? pred_out : ws.pred.as<float>();
  FwdArgs a{};
  a.B = B; a.offs = b->offset; a.col = bw.col.as<uint32_t>(); a.val = b->value; a.W = pulled;
  a.rec_S = (int)S; a.Vbase = pulled; a.zpad = c->zpad; a.d = d; a.label = b->label;
  a.rw = b->weight; a.pred = pred; a.p_out = ws.p.as<float>(); a.XVp = ws.XVp.as<float>();
  a.xs = xvp_stride(c);
  a.loss_part = ws.dscratch.as<double>() + 8;
  // AUC on its own lane beside the backward (as in the fused step): the forward writes the
  // snapshot of (pred, label) once the previous AUC released the lane's buffers
  const Lane AL{c->aux_stream, &c->aws, c->ads, &c->ds->err};
  DFX_TRY(auc_reserve(c->aws, B, c->aux_stream));
  a.auc_key = c->aws.ak0.as<uint32_t>();
  a.auc_lab = c->aws.av0.as<uint32_t>();
  DFX_HIP(hipStreamWaitEvent(c->stream, c->ev_auc, 0));
  int nblk = 0;
  DFX_TRY(launch_fwd_records(a, c->stream, &nblk));
  sum_parts(c, a.loss_part, nblk, &c->ds->scratch[3], false);
  DFX_HIP(hipEventRecord(c->ev_fwd, c->stream));
  DFX_HIP(hipStreamWaitEvent(c->aux_stream, c->ev_fwd, 0));
  DFX_TRY(auc_finish(AL, B, &c->ds->prog[2], true, c->auc_sort));
  DFX_HIP(hipEventRecord(c->ev_auc, c->aux_stream));
  // (snapshot buffer 0's last reader, for a fused step of this context that writes it next)
  DFX_HIP(hipEventRecord(c->ev_auc_p[0], c->aux_stream));
  ++c->auc_seq_p[0];
  hipLaunchKernelGGL(k_dist_worker_finalize, dim3(1), dim3(1), 0, c->stream, c->ds, B);
  if (train) {
    // every gradient record is written whole, the live slot carrying whether this worker
    // pulled V (the lens of its push: the server updates V only then, sgd_updater.cc:89-98)
    BwdArgs g{};
    g.segstart = bw.segstart.as<uint32_t>(); g.ds = c->ds; g.nseg_host = U; g.segcol = nullptr;
    g.occ_row = bw.occ_row.as<uint32_t>();
    g.occ_x = b->value ? bw.occ_x.as<float>() : nullptr;
    g.zpad = c->zpad; g.p = ws.p.as<float>(); g.XVp = ws.XVp.as<float>(); g.d = d;
    g.xs = xvp_stride(c);
    g.rec_S = (int)S; g.W = pulled; g.grad = grads_out;
    DFX_TRY(launch_bwd_positions(g, U, c->stream));
  }
  // the slot's Localizer buffers may be refilled once the main stream is past this point
  DFX_HIP(hipEventRecord(c->ev_free[slot], c->stream));
  c->slot_free[slot] = nullptr;
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_dist_owner_begin(dfx_ctx* ctx, int slot, const uint64_t* recv_keys,
                         const int64_t* recv_offsets, int nranks, const float* recv_cnt) {
  DFX_CHECK_ARG(ctx && recv_offsets, "null argument");
  DFX_CHECK_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxRanks, "dist: 1 <= nranks <= 64");
  Context* c = &ctx->c;
  DFX_TRY(pipeline_init(c));
  DFX_CHECK_ARG(!any_pending(c->dist_initv_pending),
                "dist_owner_begin: finish the pending InitV first (dfx_dist_initv_local / _draw)");
  // this table serves one of nranks key ranges: hash keys by their position in the range
  DFX_TRY(table_set_ranges(c, nranks));
  const Lane OL = owner_lane(c, slot);
  Workspace& ws = *OL.ws;
  DFX_CHECK_ARG(recv_offsets[0] == 0, "dist_owner_begin: recv_offsets[0] must be 0");
  for (int r = 0; r < nranks; ++r)
    DFX_CHECK_ARG(recv_offsets[r + 1] >= recv_offsets[r], "dist_owner_begin: bad offsets");
  const int64_t R = recv_offsets[nranks];
  DFX_CHECK_ARG(R < 0x7FFFFFFFll, "dist_owner_begin: too many keys");
  DFX_CHECK_ARG(R == 0 || recv_keys, "dist_owner_begin: null keys");
  // this begin ends the slot's previous step; it inserts at most R keys and draws at most R V
  // rows: the table grows here first if they might not fit (the reference's model is an
  // unbounded map, sgd_updater.h:178).  Growth rehashes; a pipelined schedule's other step,
  // which holds table positions until its push, gets them moved (table_rebuild)
  c->dist_live[slot] = false;
  DFX_TRY(cap_check(c, R));
  c->dist_live[slot] = true;
  c->dist_pushed[slot] = false;
  c->dist_R[slot] = R;
  c->dist_offs[slot].assign(recv_offsets, recv_offsets + nranks + 1);
  DFX_HIP(hipMemsetAsync(&OL.ds->totals[1], 0, 12, OL.stream));
  if (R == 0) return DFX_OK;
  DFX_TRY(ws.keys0.ensure(R * 8));
  DFX_TRY(ws.keys1.ensure(R * 8));
  DFX_TRY(ws.vals0.ensure(R * 4));
  DFX_TRY(ws.vals1.ensure(R * 4));
  DFX_TRY(ws.oflags.ensure((R + kMaxRanks) * 8));
  DFX_TRY(ws.ofrank.ensure((R + 1) * 4));
  DFX_TRY(ws.osegstart.ensure((R + 1) * 4));
  DFX_TRY(ws.osegslot.ensure((R + 1) * 4));
  DFX_TRY(ws.oseg_of.ensure((R + 1) * 4));
  DFX_TRY(ws.osorted.ensure((R + 1) * 4));
  uint32_t* flags = ws.oflags.as<uint32_t>();
  uint32_t* nuniq = &OL.ds->totals[1];
  const dim3 grid((R + kDNT - 1) / kDNT);
  // stable merge of the N sorted runs (none for one run)
  const uint64_t* K = recv_keys;
  const uint32_t* Pm = nullptr;
  merge_runs(OL, std::vector<int64_t>(recv_offsets, recv_offsets + nranks + 1), &K, &Pm);
  hipLaunchKernelGGL(k_dist_heads, grid, dim3(kDNT), 0, OL.stream, K, R, flags);
  DFX_TRY(scan_u32(OL, flags, R, nuniq));
  c->dist_K[slot] = K;
  c->dist_P[slot] = Pm;
  c->dist_segs_pending[slot] = true;
  // with no count push the segments are built by the pull (k_dist_segs_pull), in one pass
  if (recv_cnt || vec_group(c->P.V_dim) == 0) owner_segs(c, slot);
  if (recv_cnt) {
    hipLaunchKernelGGL(k_dist_feacnt, grid, dim3(kDNT), 0, OL.stream,
                       ws.osegstart.as<uint32_t>(), ws.osegslot.as<uint32_t>(),
                       ws.osorted.as<uint32_t>(), recv_cnt, rank_offs(c, slot), c->T, c->P,
                       nuniq, flags, ws.ofrank.as<uint32_t>(), &OL.ds->totals[3]);
    if (c->P.V_dim > 0) {
      if (c->dist_sum)
        c->dist_initv_pending[slot] = true;  // drawn in global key order (dfx_dist_initv_*)
      else
        DFX_TRY(owner_initv(c, slot, nranks));
    }
  }
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_dist_owner_pull(dfx_ctx* ctx, int slot, float* vals_out) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_CHECK_SLOT(slot);
  Context* c = &ctx->c;
  DFX_CHECK_ARG(!c->dist_initv_pending[slot],
                "dist_owner_pull: the count push's InitV is pending (dfx_dist_initv_local / _draw)");
  const int64_t R = c->dist_R[slot];
  if (R == 0) return DFX_OK;
  DFX_CHECK_ARG(vals_out, "dist_owner_pull: null buffer");
  const Lane OL = owner_lane(c, slot);
  const int G = vec_group(c->P.V_dim);
  if (c->dist_segs_pending[slot] && G > 0) {
    c->dist_segs_pending[slot] = false;
    Workspace& ws = *OL.ws;
#define DFX_SEGS_PULL(GG)                                                                    \
    if (G == GG) {                                                                           \
      const int64_t per = kDNT / GG;                                                         \
      hipLaunchKernelGGL(k_dist_segs_pull<GG>, dim3((R + per - 1) / per), dim3(kDNT), 0,     \
                         OL.stream, c->dist_K[slot], c->dist_P[slot], R, c->ds,              \
                         ws.oflags.as<uint32_t>(), &OL.ds->totals[1], c->T, c->P,            \
                         ws.osegstart.as<uint32_t>(), ws.osegslot.as<uint32_t>(),            \
                         ws.osorted.as<uint32_t>(), vals_out);                               \
    }
    DFX_DIST_GROUPS(DFX_SEGS_PULL)
#undef DFX_SEGS_PULL
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  owner_segs(c, slot);
#define DFX_PULL(GG)                                                                         \
  if (G == GG) {                                                                             \
    const int64_t per = kDNT / GG;                                                           \
    hipLaunchKernelGGL(k_dist_pull_vec<GG>, dim3((R + per - 1) / per), dim3(kDNT), 0,        \
                       OL.stream, R, OL.ws->oseg_of.as<uint32_t>(),                          \
                       OL.ws->osegslot.as<uint32_t>(), c->T, c->P, vals_out);               \
  }
  DFX_DIST_GROUPS(DFX_PULL)
#undef DFX_PULL
  if (G == 0)
    hipLaunchKernelGGL(k_dist_pull, dim3((R + kDNT - 1) / kDNT), dim3(kDNT), 0, OL.stream, R,
                       OL.ws->oseg_of.as<uint32_t>(), OL.ws->osegslot.as<uint32_t>(), c->T,
                       c->P, vals_out);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_dist_owner_push(dfx_ctx* ctx, int slot, const float* recv_grads) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_CHECK_SLOT(slot);
  Context* c = &ctx->c;
  DFX_CHECK_ARG(!any_pending(c->dist_initv_pending),
                "dist_owner_push: finish the pending InitV first (dfx_dist_initv_local / _draw)");
  const int64_t R = c->dist_R[slot];
  if (R == 0 && !c->dist_sum) {
    c->dist_live[slot] = false;
    return DFX_OK;
  }
  DFX_CHECK_ARG(R == 0 || recv_grads, "dist_owner_push: null buffer");
  owner_segs(c, slot);  // a push with no pull before it
  const Lane OL = owner_lane(c, slot);
  Workspace& ws = *OL.ws;
  const int G = vec_group(c->P.V_dim);
  if (c->dist_sum) {
    // one Update per key on the summed gradient; InitV drawn in global key order next
    if (R > 0) {
#define DFX_PUSH_SUM(GG)                                                                     \
      if (G == GG) {                                                                         \
        const int64_t per = kDNT / GG;                                                       \
        hipLaunchKernelGGL(k_dist_push_sum_vec<GG>, dim3((R + per - 1) / per), dim3(kDNT), 0, \
                           OL.stream, ws.osegstart.as<uint32_t>(),                           \
                           ws.osegslot.as<uint32_t>(), ws.osorted.as<uint32_t>(),            \
                           recv_grads, c->T, c->P, &OL.ds->totals[1],                        \
                           ws.oflags.as<uint32_t>(), c->ds, &OL.ds->totals[3]);              \
      }
      DFX_DIST_GROUPS(DFX_PUSH_SUM)
#undef DFX_PUSH_SUM
      if (G == 0)
        hipLaunchKernelGGL(k_dist_push_sum, dim3((R + kDNT - 1) / kDNT), dim3(kDNT), 0,
                           OL.stream, ws.osegstart.as<uint32_t>(), ws.osegslot.as<uint32_t>(),
                           ws.osorted.as<uint32_t>(), recv_grads, c->T, c->P,
                           &OL.ds->totals[1], ws.oflags.as<uint32_t>(), c->ds,
                           &OL.ds->totals[3]);
    }
    // every owner takes part in the InitV ranking, with or without keys this step
    c->dist_pushed[slot] = true;
    if (c->P.V_dim > 0) {
      c->dist_initv_pending[slot] = true;
    } else {
      c->dist_live[slot] = false;  // the step is done with its table positions
      DFX_TRY(cap_record(c));
    }
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  const RankOffs ro = rank_offs(c, slot);
#define DFX_PUSH(GG)                                                                         \
  if (G == GG) {                                                                             \
    const int64_t per = kDNT / GG;                                                           \
    hipLaunchKernelGGL(k_dist_push_vec<GG>, dim3((R + per - 1) / per), dim3(kDNT), 0,        \
                       OL.stream, ws.osegstart.as<uint32_t>(), ws.osegslot.as<uint32_t>(),   \
                       ws.osorted.as<uint32_t>(), recv_grads, ro, c->T, c->P,               \
                       &OL.ds->totals[1], ws.oflags.as<uint32_t>(),                          \
                       ws.ofrank.as<uint32_t>(), c->ds, &OL.ds->totals[3]);                  \
  }
  DFX_DIST_GROUPS(DFX_PUSH)
#undef DFX_PUSH
  if (G == 0)
    hipLaunchKernelGGL(k_dist_push, dim3((R + kDNT - 1) / kDNT), dim3(kDNT), 0, OL.stream,
                       ws.osegstart.as<uint32_t>(), ws.osegslot.as<uint32_t>(),
                       ws.osorted.as<uint32_t>(), recv_grads, ro, c->T, c->P,
                       &OL.ds->totals[1], ws.oflags.as<uint32_t>(), ws.ofrank.as<uint32_t>(),
                       c->ds, &OL.ds->totals[3]);
  if (c->P.V_dim > 0) DFX_TRY(owner_initv(c, slot, (int)c->dist_offs[slot].size() - 1));
  c->dist_live[slot] = false;  // the step is done with its table positions
  DFX_TRY(cap_record(c));
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// push_agg=sum: the InitV requests of the slot's last count push or gradient push, ranked
// over all owners.  initv_local scans this owner's flags (key order) and writes their number
// to count_dev (device int64); the caller all-gathers the owners' counts (rank order) into
// counts_all_dev[nranks] (device) and initv_draw draws this owner's keys after every lower
// owner's, advancing the shared seed by the total (sgd_updater.cc:144-152 in global key order)
int dfx_dist_initv_local(dfx_ctx* ctx, int slot, int64_t* count_dev) {
  DFX_CHECK_ARG(ctx && count_dev, "null argument");
  DFX_CHECK_SLOT(slot);
  Context* c = &ctx->c;
  DFX_CHECK_ARG(c->dist_sum, "dist_initv_local: only with push_agg=sum");
  const Lane OL = owner_lane(c, slot);
  uint32_t* ftotal = &OL.ds->totals[2];
  if (!c->dist_initv_pending[slot] || c->dist_R[slot] == 0) {
    DFX_HIP(hipMemsetAsync(ftotal, 0, sizeof(uint32_t), OL.stream));
  } else {
    DFX_TRY(scan_u32(OL, OL.ws->oflags.as<uint32_t>(), c->dist_R[slot], ftotal,
                     &OL.ds->totals[1], &OL.ds->totals[3]));
  }
  hipLaunchKernelGGL(k_dist_initv_count, dim3(1), dim3(1), 0, OL.stream, ftotal, count_dev);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_dist_initv_draw(dfx_ctx* ctx, int slot, const int64_t* counts_all_dev, int rank,
                        int nranks) {
  DFX_CHECK_ARG(ctx && counts_all_dev, "null argument");
  DFX_CHECK_SLOT(slot);
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxRanks && rank >= 0 && rank < nranks,
                "dist_initv_draw: bad rank");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(c->dist_sum, "dist_initv_draw: only with push_agg=sum");
  const Lane OL = owner_lane(c, slot);
  const int64_t R = c->dist_R[slot];
  uint32_t* ftotal = &OL.ds->totals[2];
  if (c->dist_initv_pending[slot] && R > 0) {
    const dim3 igrid((unsigned)std::min<int64_t>((R + kDNT - 1) / kDNT, 1024));
    hipLaunchKernelGGL(k_dist_initv_sum, igrid, dim3(kDNT), 0, OL.stream,
                       OL.ws->oflags.as<uint32_t>(), ftotal, &OL.ds->totals[1], R,
                       OL.ws->osegslot.as<uint32_t>(), counts_all_dev, rank, c->T,
                       c->P.V_init_scale, c->ds);
  }
  hipLaunchKernelGGL(k_dist_initv_sum_finalize, dim3(1), dim3(1), 0, OL.stream, ftotal,
                     counts_all_dev, nranks, c->P.V_dim, c->T.vcap, c->ds, &OL.ds->totals[3]);
  c->dist_initv_pending[slot] = false;
  if (c->dist_pushed[slot]) c->dist_live[slot] = false;  // the step is done with the table
  DFX_TRY(cap_record(c));
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int dfx_dist_push_agg_sum(dfx_ctx* ctx) { return ctx ? ctx->c.dist_sum : -1; }

// The union of the workers' sorted unique keys (the literal north_star schedule: an all-gather
// of keys, union-indexed all-gather of records and reduce-scatter of gradients).  runs: the
// workers' key lists concatenated in rank order, run_offs[nruns+1] (host) their boundaries.
// union_out (room for run_offs[nruns] keys) receives the sorted union, upos_out[i] the union
// position of runs[i], bounds_out[nranks+1] (host) the union positions where each owner's
// keys begin, *n_union (host) the union size.  Synchronises the context stream.
int dfx_dist_union(dfx_ctx* ctx, const uint64_t* runs, const int64_t* run_offs, int nruns,
                   int nranks, uint64_t* union_out, uint32_t* upos_out, int64_t* bounds_out,
                   int64_t* n_union) {
  DFX_CHECK_ARG(ctx && run_offs && bounds_out && n_union, "null argument");
  DFX_CHECK_ARG(nruns >= 1 && nruns <= kMaxRanks && nranks >= 1 && nranks <= kMaxRanks,
                "dist_union: 1 <= nruns, nranks <= 64");
  Context* c = &ctx->c;
  DFX_TRY(pipeline_init(c));
  const int64_t R = run_offs[nruns];
  DFX_CHECK_ARG(R < 0x7FFFFFFFll, "dist_union: too many keys");
  for (int r = 0; r < nruns; ++r)
    DFX_CHECK_ARG(run_offs[r + 1] >= run_offs[r] && run_offs[0] == 0, "dist_union: bad offsets");
  if (R == 0) {
    *n_union = 0;
    for (int r = 0; r <= nranks; ++r) bounds_out[r] = 0;
    return DFX_OK;
  }
  DFX_CHECK_ARG(runs && union_out && upos_out, "dist_union: null buffer");
  Workspace& ws = c->uws;
  DFX_TRY(ws.keys0.ensure(R * 8));
  DFX_TRY(ws.keys1.ensure(R * 8));
  DFX_TRY(ws.vals0.ensure(R * 4));
  DFX_TRY(ws.vals1.ensure(R * 4));
  DFX_TRY(ws.flags.ensure((R + 1) * 4));
  DFX_TRY(ws.cnt.ensure(8 * (kMaxRanks + 2)));
  const Lane L{c->stream, &ws, c->ds, &c->ds->err};
  const uint64_t* K = runs;
  const uint32_t* P = nullptr;
  merge_runs(L, std::vector<int64_t>(run_offs, run_offs + nruns + 1), &K, &P);
  uint32_t* flags = ws.flags.as<uint32_t>();
  uint32_t* total = ws.cnt.as<uint32_t>();
  const dim3 grid((R + kDNT - 1) / kDNT);
  hipLaunchKernelGGL(k_dist_heads, grid, dim3(kDNT), 0, c->stream, K, R, flags);
  DFX_TRY(scan_u32(L, flags, R, total));
  hipLaunchKernelGGL(k_union_write, grid, dim3(kDNT), 0, c->stream, K, P, flags, R, union_out,
                     upos_out);
  int64_t* bd = reinterpret_cast<int64_t*>(ws.cnt.as<char>() + 8);
  hipLaunchKernelGGL(k_union_bounds, dim3(1), dim3(kMaxRanks + 1), 0, c->stream, union_out,
                     total, (uint32_t)nranks, bd);
  std::vector<int64_t> h(kMaxRanks + 2);
  DFX_HIP(hipMemcpyAsync(h.data(), ws.cnt.as<char>(), 8 * (nranks + 2), hipMemcpyDeviceToHost,
                         c->stream));
  DFX_HIP(hipStreamSynchronize(c->stream));
  *n_union = (int64_t)(uint32_t)(h[0] & 0xFFFFFFFFll);
  for (int r = 0; r <= nranks; ++r) bounds_out[r] = h[1 + r];
  return DFX_OK;
}

// rows of `width` floats between a worker's key order (its sorted unique keys) and a
// union-indexed buffer of nranks owner chunks of M rows (row = owner * M + union position -
// bounds[owner]): to_union = 1 scatters the worker's rows there (the reduce-scatter's input;
// other rows untouched), 0 gathers them back (from the all-gathered records)
int dfx_dist_union_rows(dfx_ctx* ctx, const uint64_t* keys, const uint32_t* upos, int64_t U,
                        const int64_t* bounds, int nranks, int64_t M, int width, int to_union,
                        const float* src, float* dst) {
  DFX_CHECK_ARG(ctx && bounds, "null argument");
  DFX_CHECK_ARG(nranks >= 1 && nranks <= kMaxRanks && width >= 1, "dist_union_rows: bad sizes");
  if (U == 0) return DFX_OK;
  DFX_CHECK_ARG(keys && upos && src && dst, "dist_union_rows: null buffer");
  for (int r = 0; r < nranks; ++r)
    DFX_CHECK_ARG(bounds[r + 1] - bounds[r] <= M, "dist_union_rows: a chunk exceeds M rows");
  Bounds bd{};
  bd.n = nranks;
  for (int r = 0; r <= nranks; ++r) bd.b[r] = bounds[r];
  Context* c = &ctx->c;
  hipLaunchKernelGGL(k_union_rows, dim3((unsigned)((U + 63) / 64)), dim3(256), 0, c->stream,
                     keys, upos, U, bd, M, width, to_union, src, dst);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

}  // extern "C"
