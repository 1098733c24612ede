// FMLoss / LogitLoss forward and backward on gfx950 (src/loss/fm_loss.h:56-203,
// src/loss/logit_loss.h:41-103, src/common/spmv.h, spmm.h).
//
// Forward (k_fm_fwd): a group of G lanes owns one CSR row; lane l owns the contiguous V
// coordinates [l*CPL, l*CPL+CPL).  Every lane walks the row's nnz in order, so X*V and
// (X.*X)*(V.*V) are summed in exactly the reference's (row, nnz) order; the V_dim reduction
// then runs serially over coordinates 0..d-1 through wave shuffles — predictions are
// bit-identical to the reference.  At V_dim 16 a group is 4 lanes x float4, so a wave holds
// 16 rows and every gathered V row is one 64-byte segment read by 4 vector loads.
// The walk is latency-bound (slot -> {w, V row} -> V), so each iteration first issues the
// loads of UNR nnz (clamped, unconditional addresses) and only then accumulates them in
// order.
//
// Backward (k_fm_bwd): Xᵀ products as a sorted-key segmented reduction — no atomics.  A
// group owns one unique key and walks its occurrences in the Localizer's sorted (key, pos)
// order, i.e. ascending (row, nnz): the order of the reference's column-range-partitioned
// TransTimes, so gradients are deterministic and, up to expf, bit-identical.  The key's
// table entry and the first occurrences are loaded first, then V / Vaux and the rows' p and
// XV*p; in the fused step the walk ends in the FTRL/AdaGrad update of the key (no gradient
// round trip through HBM).
#include <cstdlib>

#include "fm_args.h"

namespace dfx {

constexpr int kFmNT = 256;

// kFusedProbe: kFused whose nnz find their keys in the table (FwdArgs::index)
enum FwdMode { kPredict = 0, kGradPrep = 1, kFused = 2, kFusedProbe = 3 };


// Coordinates [l*CPL, l*CPL+CPL) of a length-d row.  VEC: d is a multiple of the vector
// width and the row 16-byte aligned, so a lane's chunk is wholly inside or wholly outside
// the row (outside chunks read chunk 0 and are ignored).
template <int CPL, bool VEC>
__device__ inline void load_coords(const float* row, int l, int d, float (&v)[CPL],
                                   bool nt = false) {
  const int base = l * CPL;
  if constexpr (VEC && CPL % 4 == 0) {
    const int b = base < d ? base : 0;
#pragma unroll
    for (int m = 0; m < CPL / 4; ++m) {
      const float4 f = ld4(row + b + 4 * m, nt);
      v[4 * m] = f.x; v[4 * m + 1] = f.y; v[4 * m + 2] = f.z; v[4 * m + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int cd = base + k;
      v[k] = ldnt(row + (cd < d ? cd : 0), nt);
    }
  }
}

template <int CPL, bool VEC>
__device__ inline void store_coords(float* row, int l, int d, const float (&v)[CPL],
                                    bool nt = false) {
  const int base = l * CPL;
  if (base >= d) return;
  if constexpr (VEC && CPL % 4 == 0) {
#pragma unroll
    for (int m = 0; m < CPL / 4; ++m)
      st4(row + base + 4 * m, make_float4(v[4 * m], v[4 * m + 1], v[4 * m + 2], v[4 * m + 3]),
          nt);
  } else {
#pragma unroll
    for (int k = 0; k < CPL; ++k)
      if (base + k < d) stnt(row + base + k, v[k], nt);
  }
}

template <int G, int CPL, int MODE, bool PACKED, bool VEC>
__global__ __launch_bounds__(kFmNT) void k_fm_fwd(FwdArgs a) {
  constexpr int RPB = kFmNT / G;  // rows per block
  constexpr bool PROBE = MODE == kFusedProbe;
  // probe mode carries keys and home slots per item; at CPL 4, 8 items in flight per lane
  // (+1.4 % of the step over 4, same-box A/B; 16 is slower: forward 0.30 -> 0.375 ms)
  constexpr int UNR = PROBE ? (CPL <= 4 ? 8 : 2) : (CPL <= 4 ? 8 : (CPL <= 8 ? 4 : 2));
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t i = (int64_t)blockIdx.x * RPB + g;
  const int64_t r = fwd_row(a, i);
  const int d = a.d;
  __shared__ double red[kFmNT / kWave];
  double loss = 0;
  if (i < a.B) {
    const uint64_t o0 = a.offs[r], o1 = a.offs[r + 1];
    float acc = (MODE == kPredict) ? a.pred[r] : 0.f;
    float xv[CPL], xxvv[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) { xv[k] = 0.f; xxvv[k] = 0.f; }
    const bool valued = a.val != nullptr;
    for (uint64_t j0 = o0; j0 < o1; j0 += UNR) {
      uint32_t c[UNR];
      float x[UNR];
      int2 wr[UNR];
      uint64_t key[UNR], hs[UNR];
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        const uint64_t jj = (j0 + t < o1) ? j0 + t : o1 - 1;
        if constexpr (PROBE) {
          // the Localizer's key (localize.hip k_loc_transform) and its home slot
          const uint64_t id = a.index[jj];
          const uint64_t m = a.max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % a.max_index;
          key[t] = a.keys_ready ? id : reverse_bytes(m);
          hs[t] = tbl_hash(key[t], a.T);
          c[t] = (uint32_t)jj;
        } else if (PACKED && a.wv) {
          wr[t] = a.wv[jj];
          c[t] = (uint32_t)jj;
        } else {
          c[t] = a.col[jj];
        }
        x[t] = valued ? a.val[jj] : 1.f;
      }
      if constexpr (PROBE) {
        // first probes of all UNR items, then the (rare) longer probe chains
        uint64_t ek[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          const Entry* e = ent_at(a.T, hs[t]);
          wr[t] = *reinterpret_cast<const int2*>(e);
          ek[t] = e->key;
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          uint64_t h = hs[t];
          for (uint64_t probe = 0; ek[t] != key[t] && ek[t] != kEmptyKey && probe < a.T.mask;
               ++probe) {
            h = (h + 1) & a.T.mask;
            const Entry* e = ent_at(a.T, h);
            ek[t] = e->key;
            wr[t] = *reinterpret_cast<const int2*>(e);
          }
          // absent (a training step inserts its new keys in the backward): the empty entry
          // model_[key] default-constructs, w = 0 and no V (sgd_updater.h:20-34)
          if (ek[t] != key[t]) wr[t] = make_int2(0, -1);
        }
      }
      float w[UNR];
      int vp[UNR];
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        if (PACKED) {
          // the key's table entry: {w, vrow} in one 8-byte load (or handed over by the
          // Localizer's probe); V is visible only if present and not (l1_shrk && w == 0)
          // (SGDUpdater::Get, sgd_updater.cc:40-43)
          if (PROBE) {
            // found above
          } else if (a.wv_rank) {
            wr[t] = a.wv_rank[c[t]];
          } else if (!a.wv) {
            wr[t] = *reinterpret_cast<const int2*>(ent_at(a.T, c[t]));
          }
          w[t] = __int_as_float(wr[t].x);
          const int vr = wr[t].y;
          vp[t] = (vr >= 0 && !(a.l1_shrk && w[t] == 0.f)) ? vr : -1;
        } else if (a.rec_S) {
          // the pulled record: w and live follow V
          const int64_t rb = (int64_t)c[t] * a.rec_S;
          w[t] = a.W[rb + d];
          vp[t] = (d > 0 && a.W[rb + d + 1] != 0.f) ? (int)rb : -1;
        } else {
          if (a.wpos) {
            const int q = a.wpos[c[t]];
            w[t] = a.W[q < 0 ? 0 : q];
            if (q < 0) w[t] = 0.f;
          } else {
            w[t] = a.W[c[t]];
          }
          vp[t] = d > 0 ? a.vpos[c[t]] : -1;
        }
      }
      float v[UNR][CPL];
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        // masked items read zeros from one of 256 spread lines (one shared line would be a
        // single-L2-channel hotspot when many keys have no V)
        const float* Vr = vp[t] < 0 ? a.zpad + ((c[t] & 255u) << 4)
                                    : (PACKED ? row_V(a.T, vp[t]) : a.Vbase + vp[t]);
        load_coords<CPL, VEC>(Vr, l, d, v[t]);
      }
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        if (j0 + t >= o1) {  // past the row: a no-op item (w == 0 is skipped, no V)
          w[t] = 0.f;
          vp[t] = -1;
        }
        if (MODE != kGradPrep) {
          // SpMV::Times skips w == 0 (spmv.h:124-125)
          if (w[t] != 0.f) acc = valued ? acc + w[t] * x[t] : acc + w[t];
        }
        if (vp[t] >= 0) {
          const float xx = x[t] * x[t];  // XX_ (fm_loss.h:86-92)
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            const float vk = v[t][k];
            xv[k] = valued ? xv[k] + vk * x[t] : xv[k] + vk;
            if (MODE != kGradPrep) {
              const float vv = vk * vk;  // VV (fm_loss.h:95-101)
              xxvv[k] = valued ? xxvv[k] + vv * xx : xxvv[k] + vv;
            }
          }
        }
      }
    }
    float pr = acc;
    if (PROBE && a.part) {
      // owner-computes split: this owner's share of the row; the worker sums the owners'
      // shares and finishes the row (split.hip k_split_combine)
      const int PS = split_part_floats(d, a.part_n);
      float* pr_row = a.part + r * PS;
      if (a.part_n > 1) {  // [XV | sum w x | sum_l XXVV_l (serial over l) | 0 0]
        float sx = 0.f;
        const int gbase = (threadIdx.x % kWave) - l;
        for (int q = 0; q < G; ++q) {
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            const float tk = __shfl(xxvv[k], gbase + q, kWave);
            if (q * CPL + k < d) sx += tk;
          }
        }
        if (d > 0) store_coords<CPL, VEC>(pr_row, l, d, xv);
        if (l == 0) {
          pr_row[d] = acc;
          pr_row[d + 1] = sx;
          pr_row[d + 2] = pr_row[d + 3] = 0.f;
        }
      } else {
        if (d > 0) {
          store_coords<CPL, VEC>(pr_row, l, d, xv);
          store_coords<CPL, VEC>(pr_row + d, l, d, xxvv);
        }
        if (l == 0) {
          pr_row[2 * d] = acc;
          pr_row[2 * d + 1] = pr_row[2 * d + 2] = pr_row[2 * d + 3] = 0.f;
        }
      }
    } else if (MODE != kGradPrep && d > 0) {
      // s = sum_l (XV_l^2 - XXVV_l), serially over l = 0..d-1 (fm_loss.h:110-113)
      float t[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) t[k] = xv[k] * xv[k] - xxvv[k];
      float s = 0.f;
      const int gbase = (threadIdx.x % kWave) - l;
      for (int q = 0; q < G; ++q) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const float tk = __shfl(t[k], gbase + q, kWave);
          if (q * CPL + k < d) s += tk;
        }
      }
      double y = (double)acc + .5 * (double)s;  // float += double (fm_loss.h:114)
      pr = (float)y;
      pr = pr > 20.f ? 20.f : (pr < -20.f ? -20.f : pr);  // clip (fm_loss.h:118)
    }
    if (PROBE && a.part) {
      // written above
    } else if (MODE == kPredict) {
      if (l == 0) a.pred[r] = pr;
    } else {
      const float predv = (MODE == kGradPrep) ? a.pred_in[r] : pr;
      const float p = logit_p(a.label[r], predv, a.rw, r);
      const int64_t xs = a.xs > d ? a.xs : d;
      if (l == 0) {
        a.p_out[r] = p;
        if (xs > d) a.XVp[r * xs + d] = p;
        if (MODE == kFused || PROBE) {
          a.pred[r] = pr;
          double yy = a.label[r] > 0 ? 1.0 : -1.0;
          loss = log(1.0 + exp(-yy * (double)pr));  // Loss::Evaluate (loss.h:57-66)
          if (a.auc_key) {  // the AUC lane's snapshot: orderable key of pred, label > 0
            uint32_t u = __float_as_uint(pr + 0.0f);  // -0 == +0, as operator< sees them
            a.auc_key[r] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            a.auc_lab[r] = a.label[r] > 0 ? 1u : 0u;
          }
        }
      }
      if (d > 0) {
        float o[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) o[k] = xv[k] * p;  // XV_ *= p (fm_loss.h:196-199)
        store_coords<CPL, VEC>(a.XVp + r * xs, l, d, o);
      }
    }
  }
  if ((MODE == kFused || PROBE) && !a.part) {
    for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off, kWave);
    if (lane_id() == 0) red[threadIdx.x / kWave] = loss;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0;
      for (int i = 0; i < kFmNT / kWave; ++i) s += red[i];
      a.loss_part[blockIdx.x] = s;
    }
  }
}

// One row's outputs once its sums are complete (G lanes, CPL coordinates per lane): the split's
// partial, or FMLoss::Predict's finish — s = sum_l (XV_l^2 - XXVV_l) serially over l, the
// clip — then CalcGrad's p, XV_ * p, Evaluate's logloss and the AUC lane's snapshot.
// Loss::Evaluate's term of one row (loss.h:57-66), in double.  Not inlined: a caller that loops
// over rows would otherwise hold exp's and log's double constants in VGPRs across its loop.
__device__ __noinline__ double row_logloss(float label, float pr) {
  const double yy = label > 0 ? 1.0 : -1.0;
  return log(1.0 + exp(-yy * (double)pr));
}

template <int G, int CPL, int DK = 0>
__device__ __forceinline__ void fwd_row_out(const FwdArgs& a, int64_t r, int l, int gbase,
                                            float acc, const float (&xv)[CPL],
                                            const float (&xxvv)[CPL], double* loss) {
  const int d = DK > 0 ? DK : a.d;  // DK: V_dim known to the caller
  if (a.part) {
    // owner-computes split: this owner's share of the row (split.hip k_split_combine)
    float* pr_row = a.part + r * split_part_floats(d, a.part_n);
    if (a.part_n > 1) {  // [XV | sum w x | sum_l XXVV_l (serial over l) | 0 0]
      float sx = 0.f;
      for (int q = 0; q < G; ++q) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const float tk = __shfl(xxvv[k], gbase + q, kWave);
          if (q * CPL + k < d) sx += tk;
        }
      }
#pragma unroll
      for (int m = 0; m < CPL / 4; ++m)
        if (l * CPL + 4 * m < d)
          *reinterpret_cast<float4*>(pr_row + l * CPL + 4 * m) =
              make_float4(xv[4 * m], xv[4 * m + 1], xv[4 * m + 2], xv[4 * m + 3]);
      if (l == 0) {
        pr_row[d] = acc;
        pr_row[d + 1] = sx;
        pr_row[d + 2] = pr_row[d + 3] = 0.f;
      }
    } else {
#pragma unroll
      for (int m = 0; m < CPL / 4; ++m) {
        if (l * CPL + 4 * m < d) {
          *reinterpret_cast<float4*>(pr_row + l * CPL + 4 * m) =
              make_float4(xv[4 * m], xv[4 * m + 1], xv[4 * m + 2], xv[4 * m + 3]);
          *reinterpret_cast<float4*>(pr_row + d + l * CPL + 4 * m) =
              make_float4(xxvv[4 * m], xxvv[4 * m + 1], xxvv[4 * m + 2], xxvv[4 * m + 3]);
        }
      }
      if (l == 0) {
        pr_row[2 * d] = acc;
        pr_row[2 * d + 1] = pr_row[2 * d + 2] = pr_row[2 * d + 3] = 0.f;
      }
    }
  }
  float pr = acc;
  if (d > 0 && !a.part) {
    // s = sum_l (XV_l^2 - XXVV_l), serially over l = 0..d-1 (fm_loss.h:110-113)
    float t4[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) t4[k] = xv[k] * xv[k] - xxvv[k];
    float s = 0.f;
    for (int q = 0; q < G; ++q) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const float tk = __shfl(t4[k], gbase + q, kWave);
        if (q * CPL + k < d) s += tk;
      }
    }
    double y = (double)acc + .5 * (double)s;  // float += double (fm_loss.h:114)
    pr = (float)y;
    pr = pr > 20.f ? 20.f : (pr < -20.f ? -20.f : pr);  // clip (fm_loss.h:118)
  }
  const float p = a.part ? 0.f : logit_p(a.label[r], pr, a.rw, r);
  const int64_t xs = a.xs > d ? a.xs : d;
  if (a.part) {
    // the partial is all this kernel writes
  } else if (l == 0) {
    a.p_out[r] = p;
    if (xs > d) a.XVp[r * xs + d] = p;
    a.pred[r] = pr;
    *loss += row_logloss(a.label[r], pr);  // Loss::Evaluate (loss.h:57-66)
    if (a.auc_key) {  // the AUC lane's snapshot: orderable key of pred, label > 0
      uint32_t u = __float_as_uint(pr + 0.0f);  // -0 == +0, as operator< sees them
      a.auc_key[r] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
      a.auc_lab[r] = a.label[r] > 0 ? 1u : 0u;
    }
  }
#pragma unroll
  for (int m = 0; m < CPL / 4; ++m)  // XV_ *= p (fm_loss.h:196-199)
    if (d > 0 && l * CPL + 4 * m < d && !a.part)
      *reinterpret_cast<float4*>(a.XVp + r * xs + l * CPL + 4 * m) =
          make_float4(xv[4 * m] * p, xv[4 * m + 1] * p, xv[4 * m + 2] * p, xv[4 * m + 3] * p);
}

// Probe-mode forward with the lookups spread over the row's lanes (CPL = 4: float4 per lane,
// G lanes per row).  The row is walked in chunks of 32 nnz: first every lane of the group finds
// the entries of its 32/G of them (id -> key -> home slot -> {w, vrow, key}), all loads issued
// together; then the chunk's {w, V row} are handed round the group with lane shuffles and the
// V rows loaded 8 nnz at a time, accumulated in nnz order.  Per 32 nnz that is one trip for the
// ids, one for the entries and pipelined V trips — where the UNR loop of k_fm_fwd paid three
// dependent trips per 8 nnz.  Sums run in exactly the same (row, nnz) order, so predictions
// are bit-identical to k_fm_fwd's (and the reference's).
//
// CPL = 8 (kwarg fwd_cpl, V_dim a multiple of 8, not FAT): two float4 of V per lane, half the
// lanes per row; each coordinate's sums are still one lane's in nnz order and s is summed over
// l = 0..d-1 in order, so predictions are bit-identical to CPL = 4.
template <int G, int CPL = 4>
__device__ __forceinline__ void fwd_probe_body(const FwdArgs& a) {
  static_assert(CPL == 4 || CPL == 8, "one or two float4 per lane");
  constexpr int RPB = kFmNT / G;  // rows per block
  constexpr int CH = 32;          // nnz per chunk
  constexpr int MA = CH / G;      // lookups per lane per chunk
  constexpr int VB = CPL == 4 ? 8 : 4;  // V rows in flight per batch
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int gbase = (threadIdx.x % kWave) - l;
  const int d = a.d;
  __shared__ double red[kFmNT / kWave];
  double loss = 0;
  const int64_t ri = (int64_t)blockIdx.x * RPB + g;  // one row per group
  if (ri < a.B) {
    const int64_t r = fwd_row(a, ri);
    const uint64_t o0 = a.offs[r], o1 = a.offs[r + 1];
    float acc = 0.f;
    float xv[CPL], xxvv[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) { xv[k] = 0.f; xxvv[k] = 0.f; }
    const bool valued = a.val != nullptr;
    for (uint64_t j0 = o0; j0 < o1; j0 += CH) {
      // ---- the chunk's lookups, MA per lane: nnz j0 + l + G*m
      uint64_t key[MA], hs[MA];
      float xm[MA];
#pragma unroll
      for (int m = 0; m < MA; ++m) {
        const uint64_t j = j0 + l + (uint64_t)G * m;
        const uint64_t jj = j < o1 ? j : o1 - 1;
        const uint64_t id = a.index[jj];
        const uint64_t mm = a.max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % a.max_index;
        key[m] = a.keys_ready ? id : reverse_bytes(mm);
        hs[m] = tbl_hash(key[m], a.T);
        xm[m] = valued ? a.val[jj] : 1.f;
      }
      int2 wr[MA];
      uint64_t ek[MA];
#pragma unroll
      for (int m = 0; m < MA; ++m) {
        const Entry* e = ent_at(a.T, hs[m]);
        wr[m] = *reinterpret_cast<const int2*>(e);
        ek[m] = e->key;
      }
      float wm[MA];
      int vm[MA];
#pragma unroll
      for (int m = 0; m < MA; ++m) {
        uint64_t h = ek[m] != key[m] ? tbl_hash(key[m], a.T) : 0ull;  // (hs[m] not kept live)
        for (uint64_t probe = 0; ek[m] != key[m] && ek[m] != kEmptyKey && probe < a.T.mask;
             ++probe) {  // the (rare) longer probe chains
          h = (h + 1) & a.T.mask;
          const Entry* e = ent_at(a.T, h);
          ek[m] = e->key;
          wr[m] = *reinterpret_cast<const int2*>(e);
        }
        // absent (inserted by this training step's backward): the empty entry, w = 0, no V
        if (ek[m] != key[m] || j0 + l + (uint64_t)G * m >= o1) wr[m] = make_int2(0, -1);
        wm[m] = __int_as_float(wr[m].x);
        const int vr = wr[m].y;
        // V is visible only if present and not (l1_shrk && w == 0) (sgd_updater.cc:40-43)
        vm[m] = (vr >= 0 && !(a.l1_shrk && wm[m] == 0.f)) ? vr : -1;
      }
      // ---- V rows 8 nnz at a time, accumulated in nnz order
      const int nin = (int)((o1 - j0) < (uint64_t)CH ? (o1 - j0) : (uint64_t)CH);
      if (d == 0) {  // LR: the chunk's w x in nnz order (SpMV::Times skips w == 0, spmv.h:124-125)
#pragma unroll
        for (int t = 0; t < CH; ++t) {
          const float w = __shfl(wm[t / G], gbase + t % G, kWave);
          const float x = valued ? __shfl(xm[t / G], gbase + t % G, kWave) : 1.f;
          if (t < nin && w != 0.f) acc = valued ? acc + w * x : acc + w;
        }
        continue;
      }
#pragma unroll
      for (int b = 0; b < CH / VB; ++b) {
        if (b * VB >= nin) break;
        float w[VB], x[VB];
        int vp[VB];
        float v[VB][CPL];
#pragma unroll
        for (int t = 0; t < VB; ++t) {
          const int tt = b * VB + t;  // the chunk's nnz tt sits with lane tt % G, slot tt / G
          w[t] = __shfl(wm[tt / G], gbase + tt % G, kWave);
          vp[t] = __shfl(vm[tt / G], gbase + tt % G, kWave);
          x[t] = valued ? __shfl(xm[tt / G], gbase + tt % G, kWave) : 1.f;
        }
#pragma unroll
        for (int t = 0; t < VB; ++t) {
          const float* Vr = vp[t] < 0 ? a.zpad + (((uint32_t)t & 255u) << 4) : row_V(a.T, vp[t]);
          const int base = l * CPL < d ? l * CPL : 0;
#pragma unroll
          for (int m = 0; m < CPL / 4; ++m) {
            const float4 f = *reinterpret_cast<const float4*>(Vr + base + 4 * m);
            v[t][4 * m] = f.x; v[t][4 * m + 1] = f.y; v[t][4 * m + 2] = f.z; v[t][4 * m + 3] = f.w;
          }
        }
#pragma unroll
        for (int t = 0; t < VB; ++t) {
          if (b * VB + t >= nin) break;
          // SpMV::Times skips w == 0 (spmv.h:124-125)
          if (w[t] != 0.f) acc = valued ? acc + w[t] * x[t] : acc + w[t];
          if (vp[t] >= 0) {
            const float xx = x[t] * x[t];  // XX_ (fm_loss.h:86-92)
            const float (&vk)[CPL] = v[t];
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
              xv[k] = valued ? xv[k] + vk[k] * x[t] : xv[k] + vk[k];
              const float vv = vk[k] * vk[k];  // VV (fm_loss.h:95-101)
              xxvv[k] = valued ? xxvv[k] + vv * xx : xxvv[k] + vv;
            }
          }
        }
      }
    }
    fwd_row_out<G, CPL>(a, r, l, gbase, acc, xv, xxvv, &loss);
  }
  if (a.part) return;  // block-uniform: no loss partial in split mode
  for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int i = 0; i < kFmNT / kWave; ++i) s += red[i];
    a.loss_part[blockIdx.x] = s;
  }
}

// two float4 per lane at V_dim 128 (G = 16, CPL = 8): 4 blocks per CU asked for, 128 VGPRs at
// 4 waves / SIMD instead of 143 at 3 (a few spilled).  Same box: C5 forward 0.336 -> 0.268 ms,
// 116.0 -> 118.6 M ex/s; at V_dim 64 (G = 8) the bound cut the forward 0.41 -> 0.37 ms but the
// backward, beside more of the Localizer lane, rose 1.06 -> 1.11 (C4 shard 65.6 -> 64.2): not there
template <int G, int CPL>
__global__ __launch_bounds__(kFmNT, (CPL == 8 && G >= 16) ? 4 : 1) void k_fm_fwd_probe(FwdArgs a) {
  fwd_probe_body<G, CPL>(a);
}

// ---- the fat-slot forward (k_fm_fwd_walk; V_dim 8 or 16) --------------------------------------
// One group of G = d / 4 lanes per row (lane l: V coordinates 4l..4l+3, a float4), the groups looping
// over rows on a resident grid.  A row's ids are staged in LDS kWkIds at a time (one coalesced
// trip); each trip then issues kWkNB home-slot reads at once — even / odd lanes the entry's halves
// ({w, vrow} / key), lane l its float4 of V, one 128-byte line per nnz — checks the keys (a key
// away from home walks its probe chain) and adds the trip in nnz order: FMLoss::Predict's sums
// in the reference's order (fm_loss.h:67-119), so predictions are bit-identical to the oracle.
// The minimal form of round 4's k_fm_fwd_fat (no next-row prefetch, no runtime value switch):
// 120 -> ~110 us alone at C3 (tools/membench/fwdreal, cold caches; the random-read floor of
// its 3.9 M slot lines is 85 us, tools/membench/fwdbench flat).
constexpr int kWkNB = 8;
constexpr int kWkIds = (40 / kWkNB) * kWkNB;

template <int G, bool VALUED, int MINB = 4>  // MINB blocks per CU: 4 keeps 4 waves per SIMD
__global__ __launch_bounds__(kFmNT, MINB) void k_fm_fwd_walk(FwdArgs a) {
  static_assert(G == 2 || G == 4, "fat slots: d = 4 G, even / odd lanes the entry's halves");
  constexpr int RPB = kFmNT / G;
  __shared__ uint64_t s_id[RPB][kWkIds];
  __shared__ float s_x[VALUED ? RPB : 1][VALUED ? kWkIds : 1];
  __shared__ double red[kFmNT / kWave];
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int gbase = (threadIdx.x % kWave) - l;
  const bool ntf = (a.nt & kNtFwdTable) != 0;
  double loss = 0;
  const int64_t rstride = (int64_t)gridDim.x * RPB;
  for (int64_t ri = (int64_t)blockIdx.x * RPB + g; ri < a.B; ri += rstride) {
    const int64_t r = fwd_row(a, ri);
    const uint64_t o0 = a.offs[r], o1 = a.offs[r + 1];
    float acc = 0.f;
    float xv[4], xxvv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { xv[k] = 0.f; xxvv[k] = 0.f; }
    uint64_t c_end = o0;  // the staged ids end here
    for (uint64_t j0 = o0; j0 < o1; j0 += kWkNB) {
      if (j0 >= c_end) {  // the row's next kWkIds ids, one trip (group-uniform)
        __builtin_amdgcn_wave_barrier();  // the last chunk's reads are done
#pragma unroll
        for (int m = 0; m < (kWkIds + G - 1) / G; ++m) {
          const uint64_t j = j0 + l + (uint64_t)G * m;
          if (j < o1 && l + G * m < kWkIds) {
            s_id[g][l + G * m] = a.index[j];
            if (VALUED) s_x[g][l + G * m] = a.val[j];
          }
        }
        __builtin_amdgcn_wave_barrier();
        c_end = j0 + kWkIds;
      }
      const int cb = (int)(j0 - (c_end - kWkIds));  // this trip's first id in the chunk
      const int nin = (int)((o1 - j0) < (uint64_t)kWkNB ? (o1 - j0) : (uint64_t)kWkNB);
      // the id -> key transform, run twice (for the loads, then for the check) rather than
      // holding 8 keys (16 VGPRs) across the loads: the kernel then fits 4 waves / SIMD unspilled
      auto key_of = [&](int i) {
        const uint64_t id = s_id[g][i];
        const uint64_t mm = a.max_index == ~0ull ? (id == ~0ull ? 0ull : id) : id % a.max_index;
        return a.keys_ready ? id : reverse_bytes(mm);
      };
      float2 eh[kWkNB];  // even lanes {w, vrow}, odd lanes the key
      float4 v[kWkNB];
#pragma unroll
      for (int t = 0; t < kWkNB; ++t) {
        const uint64_t key = key_of(cb + (t < nin ? t : nin - 1));
        const float* sl = reinterpret_cast<const float*>(ent_at(a.T, tbl_hash(key, a.T)));
        eh[t] = ld2(sl + ((l & 1) ? 6 : 0), ntf);
        v[t] = ld4(sl + 8 + 4 * l, ntf);
      }
      uint64_t key[kWkNB];
#pragma unroll
      for (int t = 0; t < kWkNB; ++t) {
        if (t >= nin) break;  // group-uniform
        key[t] = key_of(cb + t);
        const float k0 = __shfl(eh[t].x, gbase + 1, kWave), k1 = __shfl(eh[t].y, gbase + 1, kWave);
        uint64_t ek = ((uint64_t)__float_as_uint(k1) << 32) | (uint64_t)__float_as_uint(k0);
        float w = __shfl(eh[t].x, gbase, kWave);
        int vr = __float_as_int(__shfl(eh[t].y, gbase, kWave));
        float4 vv = v[t];
        if (ek != key[t] && ek != kEmptyKey) {  // a longer probe chain (group-uniform)
          uint64_t h = tbl_hash(key[t], a.T);
          for (uint64_t probe = 0; ek != key[t] && ek != kEmptyKey && probe < a.T.mask; ++probe) {
            h = (h + 1) & a.T.mask;
            ek = ent_at(a.T, h)->key;
          }
          if (ek == key[t]) {
            const Entry* e = ent_at(a.T, h);
            w = e->w;
            vr = e->vrow;
            vv = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(e) + 8 + 4 * l);
          }
        }
        // absent (inserted by this training step's backward): w = 0, no V
        if (ek != key[t]) { w = 0.f; vr = -1; }
        const float x = VALUED ? s_x[g][cb + t] : 1.f;
        // SpMV::Times skips w == 0 (spmv.h:124-125)
        if (w != 0.f) acc = VALUED ? acc + w * x : acc + w;
        // V is visible only if present and not (l1_shrk && w == 0) (sgd_updater.cc:40-43)
        if (vr >= 0 && !(a.l1_shrk && w == 0.f)) {
          const float vk[4] = {vv.x, vv.y, vv.z, vv.w};
          const float xx = x * x;  // XX_ (fm_loss.h:86-92)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            xv[k] = VALUED ? xv[k] + vk[k] * x : xv[k] + vk[k];
            const float q = vk[k] * vk[k];  // VV (fm_loss.h:95-101)
            xxvv[k] = VALUED ? xxvv[k] + q * xx : xxvv[k] + q;
          }
        }
      }
    }
    fwd_row_out<G, 4, 4 * G>(a, r, l, gbase, acc, xv, xxvv, &loss);
  }
  if (a.part) return;  // block-uniform: no loss partial in split mode
  for (int off = 32; off > 0; off >>= 1) loss += __shfl_xor(loss, off, kWave);
  if (lane_id() == 0) red[threadIdx.x / kWave] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0;
    for (int i = 0; i < kFmNT / kWave; ++i) s += red[i];
    a.loss_part[blockIdx.x] = s;
  }
}

// blocks of kernel K resident at once on this device (at most want): a grid whose blocks loop
template <auto K>
static int64_t resident_grid(int64_t want) {
  static int per_cu = 0;  // per kernel
  int dev = 0, cus = 0;
  if (per_cu <= 0 &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, K, kFmNT, 0) != hipSuccess)
    per_cu = 0;
  if (per_cu <= 0 || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return want;
  return std::min<int64_t>(want, (int64_t)per_cu * cus);
}

// Lane layout for V_dim d.  vec: float4 chunks (the fused path's 16-byte aligned rows, d a
// multiple of 4); otherwise scalar coordinates (the pulled interleaved layout is unaligned).
void lanes_for(int d, bool vec, int* G, int* CPL, bool* use_vec) {
  if (d <= 0) {
    *G = 1; *CPL = 1; *use_vec = false;
    return;
  }
  if (vec && d % 4 == 0) {
    int cpl = 4;
    while (d / cpl > 64) cpl *= 2;
    int n = (d + cpl - 1) / cpl, g = 1;
    while (g < n) g <<= 1;
    *G = g; *CPL = cpl; *use_vec = true;
    return;
  }
  int g = next_pow2_lanes(d);
  int cpl = (d + g - 1) / g, c2 = 1;
  while (c2 < cpl) c2 <<= 1;
  *G = g; *CPL = c2; *use_vec = false;
}

#define DFX_SCALAR_SET(X) X(1, 1, false) X(2, 1, false) X(4, 1, false) X(8, 1, false) \
  X(16, 1, false) X(32, 1, false) X(64, 1, false) X(64, 2, false) X(64, 4, false)     \
  X(64, 8, false) X(64, 16, false)
#define DFX_VEC_SET(X) X(1, 4, true) X(2, 4, true) X(4, 4, true) X(8, 4, true) X(16, 4, true) \
  X(32, 4, true) X(64, 4, true) X(64, 8, true) X(64, 16, true)

template <int MODE, bool PACKED>
static int launch_fwd_gc(const FwdArgs& a, int G, int CPL, bool vec, hipStream_t st) {
  const int64_t rpb = kFmNT / G;
  dim3 grid((unsigned)((a.B + rpb - 1) / rpb));
  if (a.B <= 0) return DFX_OK;
#define DFX_FWD(GG, CC, VV)                                                                  \
  if (G == GG && CPL == CC && vec == VV) {                                                   \
    hipLaunchKernelGGL((k_fm_fwd<GG, CC, MODE, PACKED, VV>), grid, dim3(kFmNT), 0, st, a);  \
    DFX_HIP(hipGetLastError());                                                              \
    return DFX_OK;                                                                           \
  }
  DFX_SCALAR_SET(DFX_FWD)
  if constexpr (PACKED || MODE >= kFused) { DFX_VEC_SET(DFX_FWD) }
#undef DFX_FWD
  set_error("unsupported V_dim");
  return DFX_ERR_ARG;
}

template <int MODE, bool PACKED>
int launch_fwd(const FwdArgs& a, hipStream_t st) {
  int G, CPL;
  bool vec;
  lanes_for(a.d, PACKED, &G, &CPL, &vec);
  return launch_fwd_gc<MODE, PACKED>(a, G, CPL, vec, st);
}

int launch_fwd_fused(const FwdArgs& a, hipStream_t st, int* nblk, bool spread) {
  int G, CPL;
  bool vec;
  lanes_for(a.d, true, &G, &CPL, &vec);
  const int64_t rpb = kFmNT / G;
  *nblk = (int)((a.B + rpb - 1) / rpb);
  // fat slots: one trip per nnz (G lanes x float4 = d exactly; even / odd lanes hold the
  // entry's halves, so G >= 2: d = 8 and 16 — other fat V_dims take the probe walk below)
  const bool fat = a.T.es != 0 && !a.no_fat_fwd && vec && CPL == 4 && 4 * G == a.d && G >= 2;
  if (a.index && a.B > 0 && spread && fat) {
    // the fat forward (k_fm_fwd_walk), on a resident grid (its groups loop over rows)
#define DFX_FWDWALK(GG)                                                                   \
    if (G == GG) {                                                                        \
      if (a.val) {                                                                        \
        *nblk = (int)resident_grid<k_fm_fwd_walk<GG, true>>(*nblk);                       \
        hipLaunchKernelGGL((k_fm_fwd_walk<GG, true>), dim3((unsigned)*nblk), dim3(kFmNT), 0, \
                           st, a);                                                        \
      } else {                                                                            \
        *nblk = (int)resident_grid<k_fm_fwd_walk<GG, false>>(*nblk);                      \
        hipLaunchKernelGGL((k_fm_fwd_walk<GG, false>), dim3((unsigned)*nblk), dim3(kFmNT), \
                           0, st, a);                                                     \
      }                                                                                   \
      DFX_HIP(hipGetLastError());                                                         \
      return DFX_OK;                                                                      \
    }
    DFX_FWDWALK(2) DFX_FWDWALK(4)
#undef DFX_FWDWALK
  }
  if (a.index && spread && a.d == 0 && a.lr_lanes && a.B > 0 && !a.part) {
    // LR (V_dim 0): four lanes per row, each finding a quarter of a 32-nnz chunk's entries with
    // all their loads in flight, the w x summed in nnz order (kwarg lr_lanes; 0: one thread per
    // row, k_fm_fwd)
    *nblk = (int)((a.B + kFmNT / 4 - 1) / (kFmNT / 4));
    hipLaunchKernelGGL((k_fm_fwd_probe<4, 4>), dim3((unsigned)*nblk), dim3(kFmNT), 0, st, a);
    DFX_HIP(hipGetLastError());
    return DFX_OK;
  }
  if (a.index && spread && vec && CPL == 4 && G >= 4 && G <= 32 && a.B > 0) {
    // kwarg fwd_cpl = 8 at V_dim >= 64 (a multiple of 8): two float4 per lane, half the lanes
    int C = 4;
    if (a.cpl == 8 && a.d >= 64 && a.d % 8 == 0 && G >= 8) {
      G /= 2;
      C = 8;
      *nblk = (int)((a.B + kFmNT / G - 1) / (kFmNT / G));
    }
    const dim3 grid((unsigned)*nblk);
#define DFX_FWDP(GG, CC)                                                                 \
    if (G == GG && C == CC) {                                                            \
      hipLaunchKernelGGL((k_fm_fwd_probe<GG, CC>), grid, dim3(kFmNT), 0, st, a);          \
      DFX_HIP(hipGetLastError());                                                        \
      return DFX_OK;                                                                     \
    }
    DFX_FWDP(4, 4) DFX_FWDP(8, 4) DFX_FWDP(16, 4) DFX_FWDP(32, 4)
    DFX_FWDP(4, 8) DFX_FWDP(8, 8) DFX_FWDP(16, 8)
#undef DFX_FWDP
  }
  if (a.index) return launch_fwd_gc<kFusedProbe, true>(a, G, CPL, vec, st);
  return launch_fwd_gc<kFused, true>(a, G, CPL, vec, st);
}

// sharded store: forward over pulled records [V(d) | w | live | 0 | 0] (16-byte aligned rows
// when d % 4 == 0), addressed through wpos / vpos
int launch_fwd_records(const FwdArgs& a, hipStream_t st, int* nblk) {
  int G, CPL;
  bool vec;
  lanes_for(a.d, true, &G, &CPL, &vec);
  const int64_t rpb = kFmNT / G;
  *nblk = (int)((a.B + rpb - 1) / rpb);
  return launch_fwd_gc<kFused, false>(a, G, CPL, vec, st);
}

// ---- backward: sorted-key segmented reduction --------------------------------------------
// p of row r for a backward that also reads the row's XV*p: from the XV*p row when p shares
// its last line (4d % 128 != 0: d = 16's 68 bytes in one 128-byte line), else from the
// compact per-row array (d = 64 / 128: p would be a line of its own in a 384 / 640-byte row,
// where the 400-KB array stays in the L2); the split owner has only the rows (p == nullptr)
__device__ inline float row_p(const BwdArgs& a, uint32_t r, int d, int64_t xs) {
  if (a.p && (xs <= d || (4 * d) % 128 == 0)) return a.p[r];
  return a.XVp[(int64_t)r * xs + d];
}
template <int G, int CPL, bool FUSED, bool VEC>
__global__ __launch_bounds__(kFmNT) void k_fm_bwd(BwdArgs a) {
  constexpr int SPB = kFmNT / G;
  constexpr int UNR = CPL <= 4 ? 4 : 2;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t u = (int64_t)blockIdx.x * SPB + g;
  const int64_t nseg = a.nseg_host >= 0 ? a.nseg_host : (int64_t)a.ds->u_count;
  __shared__ int red[kFmNT / kWave];
  __shared__ int redn[kFmNT / kWave];
  __shared__ int redi[kFmNT / kWave];
  __shared__ unsigned redl[kFmNT / kWave], redo[kFmNT / kWave];
  int dnew = 0, ninit = 0, nins = 0;
  unsigned nlive = 0, nlocc = 0;  // keys with V in this step, and their occurrences (roofline)
  if (u < nseg) {
    const bool ntb = (a.nt & kNtBwdTable) != 0, nto = (a.nt & kNtBwdOcc) != 0;
    const uint32_t s0 = ldnt(a.segstart + u, nto), s1 = ldnt(a.segstart + u + 1, nto);
    const uint32_t cidx = a.segcol ? a.segcol[u] : (uint32_t)u;
    const bool valued = a.occ_x != nullptr;
    const int d = a.d;
    const int64_t xs = a.xs > d ? a.xs : d;
    const uint32_t len = s1 - s0;
    // ---- level-2 loads, mutually independent: the key's table entry (or its positions in
    // the pulled layout) and the first UNR occurrences of its segment
    int wq = -1, vq = -1, vrow = -1;
    uint32_t sl = 0;
    float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
    float fc = 0.f;
    bool home = false;  // the key's entry was read at its home slot already
    bool dead = false;  // the key has no slot (failed insert): nothing is written for it
    bool spec = false;  // fat slots: V / Vaux of the home slot loaded beside the entry
    float vcur[CPL], ccur[CPL];
    if (FUSED) {
      if (a.insert_keys) {
        // Get's find-or-insert (model_[key]) here instead of a separate pass: the home slot
        // first (every lane), a longer chain or an insert by the group's first lane
        const uint64_t key = ldnt(a.uniq + cidx, nto);
        const uint64_t hh = tbl_hash(key, a.T);
        // the whole home entry in two 16-byte loads issued together: {w, vrow, sqrt_g, z} and
        // {fea_cnt, pad, key}; a key found at home (the common case) needs no second trip
        const float* eh = reinterpret_cast<const float*>(ent_at(a.T, hh));
        const float4 h0 = ld4(eh, ntb), h1 = ld4(eh + 4, ntb);
        if (a.T.es && !a.no_fat_spec) {  // a key at home has V there: one trip for the key
          load_coords<CPL, VEC>(row_V(a.T, (int64_t)hh), l, d, vcur, ntb);
          load_coords<CPL, VEC>(row_C(a.T, (int64_t)hh), l, d, ccur, ntb);
          spec = true;
        }
        const uint64_t ek =
            ((uint64_t)__float_as_uint(h1.w) << 32) | (uint64_t)__float_as_uint(h1.z);
        home = ek == key;
        h = h0;
        fc = h1.x;
        int s = (int)hh;
        if (!home) {
          int s0 = 0;
          if (l == 0) {
            bool inserted;
            const int64_t r = tbl_insert(a.T, key, &inserted);
            if (r < 0) atomicOr(&a.dsw->err, insert_error(r));
            s0 = r < 0 ? (int)kNoSlot : (int)r;
            nins = inserted ? 1 : 0;
          }
          s = __shfl(s0, (int)(threadIdx.x % kWave) - l, kWave);
        }
        sl = (uint32_t)s;
      } else {
        sl = a.slot[cidx];
      }
      dead = sl == kNoSlot;
      if (dead) {  // not in the table (the error word says why): read as absent, no update
        h = make_float4(0.f, __int_as_float(-1), 0.f, 0.f);
        fc = 0.f;
      } else if (!home) {
        const Entry* en = ent_at(a.T, sl);
        h = *reinterpret_cast<const float4*>(en);  // w, vrow, sqrt_g, z
        fc = en->fea_cnt;
      }
    } else if (a.rec_S) {
      wq = (int)((int64_t)cidx * a.rec_S + d);
      vq = (d > 0 && a.W[wq + 1] != 0.f) ? (int)((int64_t)cidx * a.rec_S) : -1;
    } else {
      wq = a.wpos ? a.wpos[cidx] : (int)cidx;
      vq = d > 0 ? a.vpos[cidx] : -1;
    }
    uint32_t row[UNR];
    float x[UNR];
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      const uint32_t i = s0 + ((uint32_t)t < len ? (uint32_t)t : 0u);
      row[t] = occ_get(a, i, valued, nto, &x[t]);
    }
    // ---- level 3: V / Vaux (or grad / W) of the key, p and XV*p of the occurrences' rows
    float gw = 0.f;
    float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
    float g0[CPL];
    const float* zp = a.zpad + ((cidx & 255u) << 4);
    if (FUSED) {
      e = make_float4(h.x, h.z, h.w, fc);  // {w, sqrt_g, z, fea_cnt}
      vrow = __float_as_int(h.y);
      // V was pulled iff present and not (l1_shrk && w == 0) (SGDUpdater::Get, :40-43)
      vq = (vrow >= 0 && !(a.Pm.l1_shrk && e.x == 0.f)) ? vrow : -1;
      if (!(spec && home && vq >= 0)) {  // (fat slots: at home, vrow == the home slot)
        load_coords<CPL, VEC>(vq >= 0 ? row_V(a.T, vq) : zp, l, d, vcur, ntb);
        load_coords<CPL, VEC>(vq >= 0 ? row_C(a.T, vq) : zp, l, d, ccur, ntb);
      }
#pragma unroll
      for (int k = 0; k < CPL; ++k) g0[k] = 0.f;
    } else if (a.rec_S) {
      load_coords<CPL, VEC>(vq >= 0 ? a.W + vq : zp, l, d, vcur);
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        g0[k] = 0.f;
        ccur[k] = 0.f;
      }
    } else {
      gw = a.grad[wq < 0 ? 0 : wq];
      if (wq < 0) gw = 0.f;
      load_coords<CPL, VEC>(vq >= 0 ? a.W + vq : zp, l, d, vcur);
      load_coords<CPL, VEC>(vq >= 0 ? a.grad + vq : zp, l, d, g0);
#pragma unroll
      for (int k = 0; k < CPL; ++k) ccur[k] = 0.f;
    }
    float pr[UNR], xr[UNR][CPL];
    // A key without V (lazy V: most keys of a Zipf batch) needs only p of its rows, not their
    // XV*p.  Outside fat slots vq is known here from the entry the V / Vaux loads above already
    // waited for, so the condition adds no memory round trip and saves d floats per occurrence
    // of such a key; with fat slots (kernel-uniform) V came with the entry and the rows load
    // beside it, unconditionally, as before.
    const bool xv_spec = !FUSED || (a.T.es && !a.no_fat_spec);
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      pr[t] = xs > d ? a.XVp[(int64_t)row[t] * xs + d] : a.p[row[t]];
      if (xv_spec)
        load_coords<CPL, VEC>(d > 0 ? a.XVp + (int64_t)row[t] * xs : zp, l, d, xr[t]);
      else
        load_coords<CPL, VEC>(d > 0 && vq >= 0 ? a.XVp + (int64_t)row[t] * xs : zp, l, d, xr[t]);
    }
    float xxp = 0.f;
    float acc[CPL];
    // ---- pass 1: g_w and XXp (SpMV::TransTimes, spmv.h:139-171: skip p == 0)
    // ---- pass 2: grad_u = (g0 - V*XXp) + sum (XV_ p) x (fm_loss.h:185-202, spmm.h:127-159)
    // Both sums run in occurrence order; a segment of <= UNR occurrences (the common case)
    // is computed from the registers loaded above.
    if (len <= (uint32_t)UNR) {
#pragma unroll
      for (int t = 0; t < UNR; ++t) {
        if ((uint32_t)t < len && pr[t] != 0.f) {
          if (valued) {
            gw += pr[t] * x[t];
            xxp += pr[t] * (x[t] * x[t]);
          } else {
            gw += pr[t];
            xxp += pr[t];
          }
        }
      }
      if (vq >= 0) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] = g0[k] - vcur[k] * xxp;
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          if ((uint32_t)t < len) {
#pragma unroll
            for (int k = 0; k < CPL; ++k)
              acc[k] = valued ? acc[k] + xr[t][k] * x[t] : acc[k] + xr[t][k];
          }
        }
      }
    } else if (a.choff && len > (uint32_t)kChunkOcc) {
      // a long segment (a skewed key): its chunks' partial sums (k_fm_bwd_chunks), combined in
      // chunk order, all in double and rounded once — the sums differ from the reference's
      // sequential float sums only by that float rounding (reordering error)
      const uint32_t c0 = a.choff[u];
      const uint32_t nc = hot_chunks_read((len + kChunkOcc - 1) / kChunkOcc);
      const int P = d + 2;
      double gwd = 0, xxpd = 0, accp[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) accp[k] = 0;
      for (uint32_t c = 0; c < nc; ++c) {
        const double* pc = a.part + (int64_t)(c0 + c) * P;
        gwd += pc[0];
        xxpd += pc[1];
        if (vq >= 0) {
#pragma unroll
          for (int k = 0; k < CPL; ++k) {
            const int cd = l * CPL + k;
            accp[k] += cd < d ? pc[2 + cd] : 0.0;
          }
        }
      }
      gw = (float)gwd;
      xxp = (float)xxpd;
      if (vq >= 0) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] = (float)((double)(g0[k] - vcur[k] * xxp) + accp[k]);
      }
    } else if (G >= 8) {
      // Wide groups (V_dim >= 64): the group walks G occurrences per trip — lane l reads
      // occurrence i0 + l's row, value and p, so G of the random p reads are in flight at once
      // — and the sums take the terms from the lanes by shuffles in occurrence order: the same
      // terms in the same order as the per-lane walk below (bit-identical), G / UNR times fewer
      // round trips on a skewed key's long segment.  The V sums then read WU XV*p rows per
      // sub-trip, their row ids shuffled from the lanes that loaded them.
      constexpr int WU = CPL <= 4 ? 4 : 2;
      const int gb = (int)(threadIdx.x % kWave) - l;
      for (uint32_t i0 = s0; i0 < s1; i0 += G) {
        const uint32_t i = i0 + (uint32_t)l < s1 ? i0 + (uint32_t)l : s1 - 1;
        float xl;
        const uint32_t rl = occ_get(a, i, valued, false, &xl);
        const float pl = row_p(a, rl, d, xs);
        const uint32_t n = s1 - i0 < (uint32_t)G ? s1 - i0 : (uint32_t)G;
#pragma unroll
        for (int t = 0; t < G; ++t) {
          const float pt = __shfl(pl, gb + t, kWave);
          const float xt = __shfl(xl, gb + t, kWave);
          if ((uint32_t)t < n && pt != 0.f) {
            if (valued) {
              gw += pt * xt;
              xxp += pt * (xt * xt);
            } else {
              gw += pt;
              xxp += pt;
            }
          }
        }
      }
      if (vq >= 0) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] = g0[k] - vcur[k] * xxp;
        for (uint32_t i0 = s0; i0 < s1; i0 += G) {
          const uint32_t i = i0 + (uint32_t)l < s1 ? i0 + (uint32_t)l : s1 - 1;
          float xl;
          const uint32_t rl = occ_get(a, i, valued, false, &xl);
          const uint32_t n = s1 - i0 < (uint32_t)G ? s1 - i0 : (uint32_t)G;
#pragma unroll
          for (int t0 = 0; t0 < G; t0 += WU) {
            if ((uint32_t)t0 >= n) break;  // group-uniform: the segment's last trip
            float xrw[WU][CPL], xw[WU];
#pragma unroll
            for (int u = 0; u < WU; ++u) {
              const uint32_t r = (uint32_t)__shfl((int)rl, gb + t0 + u, kWave);
              xw[u] = __shfl(xl, gb + t0 + u, kWave);
              load_coords<CPL, VEC>(a.XVp + (int64_t)r * xs, l, d, xrw[u]);
            }
#pragma unroll
            for (int u = 0; u < WU; ++u) {
              if ((uint32_t)(t0 + u) < n) {
#pragma unroll
                for (int k = 0; k < CPL; ++k)
                  acc[k] = valued ? acc[k] + xrw[u][k] * xw[u] : acc[k] + xrw[u][k];
              }
            }
          }
        }
      }
    } else {
      // Both walks keep the next trip's rows in flight beside this trip's row reads (the
      // segment's occ_row / occ_x are contiguous; the p / XV*p reads are the random ones), so a
      // trip costs one memory round trip instead of two.  Same terms, same order.
      uint32_t rw[UNR];
      float xw[UNR];
#pragma unroll
      for (int t = 0; t < UNR; ++t) {  // the first trip's rows: already loaded (level 2)
        rw[t] = row[t];
        xw[t] = x[t];
      }
      for (uint32_t i0 = s0; i0 < s1; i0 += UNR) {
        float pw[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t)
          pw[t] = row_p(a, rw[t], d, xs);
        const uint32_t in = i0 + UNR;
        uint32_t rn[UNR];
        float xn[UNR];
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          const uint32_t i = in + t < s1 ? in + t : s1 - 1;
          xn[t] = 1.f;
          rn[t] = in < s1 ? occ_get(a, i, valued, false, &xn[t]) : 0u;
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          if (i0 + t < s1 && pw[t] != 0.f) {
            if (valued) {
              gw += pw[t] * xw[t];
              xxp += pw[t] * (xw[t] * xw[t]);
            } else {
              gw += pw[t];
              xxp += pw[t];
            }
          }
        }
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          rw[t] = rn[t];
          xw[t] = xn[t];
        }
      }
      if (vq >= 0) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] = g0[k] - vcur[k] * xxp;
#pragma unroll
        for (int t = 0; t < UNR; ++t) {
          rw[t] = row[t];
          xw[t] = x[t];
        }
        for (uint32_t i0 = s0; i0 < s1; i0 += UNR) {
          float xrw[UNR][CPL];
#pragma unroll
          for (int t = 0; t < UNR; ++t)
            load_coords<CPL, VEC>(a.XVp + (int64_t)rw[t] * xs, l, d, xrw[t]);
          // the next trip's rows, in flight beside this trip's XV*p rows
          const uint32_t in = i0 + UNR;
          uint32_t rn[UNR];
          float xn[UNR];
#pragma unroll
          for (int t = 0; t < UNR; ++t) {
            const uint32_t i = in + t < s1 ? in + t : s1 - 1;
            xn[t] = 1.f;
            rn[t] = in < s1 ? occ_get(a, i, valued, false, &xn[t]) : 0u;
          }
#pragma unroll
          for (int t = 0; t < UNR; ++t) {
            if (i0 + t < s1) {
#pragma unroll
              for (int k = 0; k < CPL; ++k)
                acc[k] = valued ? acc[k] + xrw[t][k] * xw[t] : acc[k] + xrw[t][k];
            }
          }
#pragma unroll
          for (int t = 0; t < UNR; ++t) {
            rw[t] = rn[t];
            xw[t] = xn[t];
          }
        }
      }
    }
    if (!FUSED && a.rec_S) {
      // the whole gradient record: gV (zeros unless V was pulled), gw, live, padding
      float* gr = a.grad + (int64_t)cidx * a.rec_S;
      if (vq < 0) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] = 0.f;
      }
      store_coords<CPL, VEC>(gr, l, d, acc);
      if (l == 0) {
        gr[d] = gw;
        gr[d + 1] = vq >= 0 ? 1.f : 0.f;
        for (int k = d + 2; k < a.rec_S; ++k) gr[k] = 0.f;
      }
    } else if (!FUSED) {
      if (l == 0 && wq >= 0) a.grad[wq] = gw;
      if (vq >= 0) store_coords<CPL, VEC>(a.grad + vq, l, d, acc);
    } else {
      // Update(kGradient): UpdateW (FTRL), then UpdateV (AdaGrad) if V was pulled
      bool tr;
      const int dw = ftrl_update(a.Pm, gw, &e, &tr);
      if (vq >= 0) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) adagrad_update(a.Pm, acc[k], &vcur[k], &ccur[k]);
        store_coords<CPL, VEC>(row_V(a.T, vq), l, d, vcur, ntb);
        store_coords<CPL, VEC>(row_C(a.T, vq), l, d, ccur, ntb);
      }
      if (l == 0) {
        if (!dead) ent_store_hot(ent_at(a.T, sl), e, vrow, ntb);
        dnew = dead ? 0 : dw;
        // InitV on a 0 -> nonzero transition (sgd_updater.cc:118-121); e.w is fea_cnt
        const bool need =
            !dead && tr && d > 0 && vrow < 0 && e.w > (float)a.Pm.V_threshold;
        a.flags[u] = need ? 1u : 0u;
        // InitV's slot: it reads the slots of flagged keys only (in the steady state none)
        if (need && a.insert_keys) a.slot[cidx] = sl;
        ninit = need ? 1 : 0;
        nlive = vq >= 0 ? 1u : 0u;
        nlocc = vq >= 0 ? len : 0u;
      }
    }
  }
  if (FUSED) {
    // new_w, and the InitV requests (dsw->n_init gates the InitV pass on the device)
    for (int off = 32; off > 0; off >>= 1) {
      dnew += __shfl_xor(dnew, off, kWave);
      ninit += __shfl_xor(ninit, off, kWave);
      nins += __shfl_xor(nins, off, kWave);
      nlive += __shfl_xor(nlive, off, kWave);
      nlocc += __shfl_xor(nlocc, off, kWave);
    }
    if (lane_id() == 0) {
      red[threadIdx.x / kWave] = dnew;
      redn[threadIdx.x / kWave] = ninit;
      redi[threadIdx.x / kWave] = nins;
      redl[threadIdx.x / kWave] = nlive;
      redo[threadIdx.x / kWave] = nlocc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int s = 0, q = 0, i2 = 0;
      unsigned long long lv = 0, lo = 0;
      for (int i = 0; i < kFmNT / kWave; ++i) {
        s += red[i];
        q += redn[i];
        i2 += redi[i];
        lv += redl[i];
        lo += redo[i];
      }
      // one-word atomics serialise (~88 per us) and a cold model has a new w in
      // nearly every block: the counts go to a stripe of their own line; n_init is a gate only
      unsigned long long* nw = (unsigned long long*)&a.dsw->new_w;
      unsigned long long* nk = &a.dsw->n_keys;
      if (a.stripes) {
        nw = a.stripes + (blockIdx.x % kBwStripes) * 16;
        nk = nw + 1;
      }
      if (s) atomicAdd(nw, (unsigned long long)(long long)s);
      if (q && __hip_atomic_load(&a.dsw->n_init, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
        atomicOr(&a.dsw->n_init, 1u);
      if (i2) atomicAdd(nk, (unsigned long long)i2);
      if (a.live_part) a.live_part[blockIdx.x] = make_uint2((unsigned)lv, (unsigned)lo);
    }
  }
}

// ---- the fused backward in two passes, for wide V_dim (G >= 32 lanes per key) ------------
// With d = 128 a key's group is 32 lanes, and under lazy V (C5: V_threshold, Zipf keys) most
// keys carry no V: their group does a w-only update on lane 0 while 31 lanes wait, two keys per
// wave, a latency-bound walk (profiles/r3/kernel_summary_c5.md).  Pass W takes one lane per key
// — the entry's find-or-insert, g_w and XXp over the key's occurrences in order, FTRL, the InitV
// flag — and lists each key whose V was pulled with its XXp; pass V takes G lanes per listed key
// for the sum of (XV*p) x in occurrence order and AdaGrad.  Every term and its order are
// k_fm_bwd's, so the model is bit-identical; the list's order (block-aggregated appends) changes
// only which group updates which key.  Both passes loop over a resident grid.  Measured on C5
// (same box, kwarg bwd_two_pass): first 1.53 -> 1.85 ms — a wave of pass W ran as long as its
// longest key's serial walk, a hot key's ~1750 chunk partials one round trip each; with those
// pre-summed (k_chunk_hotsum) the two passes take 0.74 ms against the one kernel's 1.17
// (C5 65.7 -> 92.3 M ex/s): the default at >= 32 lanes per key (V_dim >= 128).
constexpr int kBwdWNT = 256;

__global__ __launch_bounds__(kBwdWNT) void k_fm_bwd_w(BwdArgs a) {
  __shared__ int red[kBwdWNT / kWave], redn[kBwdWNT / kWave], redi[kBwdWNT / kWave];
  __shared__ unsigned redl[kBwdWNT / kWave], redo[kBwdWNT / kWave];
  __shared__ uint32_t wcnt[kBwdWNT / kWave], wbase;
  const int64_t nseg = a.nseg_host >= 0 ? a.nseg_host : (int64_t)a.ds->u_count;
  const int d = a.d;
  const int64_t xs = a.xs > d ? a.xs : d;
  const bool valued = a.occ_x != nullptr;
  int dnew = 0, ninit = 0, nins = 0;
  unsigned nlive = 0, nlocc = 0;
  const int64_t stride = (int64_t)gridDim.x * kBwdWNT;
  // every lane runs the same number of rounds (the list append is block-aggregated)
  const int64_t rounds = (nseg + stride - 1) / stride;
  for (int64_t rd = 0; rd < rounds; ++rd) {
    const int64_t u = rd * stride + (int64_t)blockIdx.x * kBwdWNT + threadIdx.x;
    bool listed = false;
    uint4 item = make_uint4(0u, 0u, 0u, 0u);
    if (u < nseg) {
      const uint32_t s0 = a.segstart[u], s1 = a.segstart[u + 1];
      const uint32_t len = s1 - s0;
      const uint32_t cidx = (uint32_t)u;
      uint32_t sl = 0;
      bool home = false;
      float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
      float fc = 0.f;
      if (a.insert_keys) {
        const uint64_t key = a.uniq[cidx];
        const uint64_t hh = tbl_hash(key, a.T);
        const float4* eh = reinterpret_cast<const float4*>(ent_at(a.T, hh));
        const float4 h0 = eh[0], h1 = eh[1];
        const uint64_t ek =
            ((uint64_t)__float_as_uint(h1.w) << 32) | (uint64_t)__float_as_uint(h1.z);
        home = ek == key;
        h = h0;
        fc = h1.x;
        int64_t s = (int64_t)hh;
        if (!home) {
          bool inserted;
          s = tbl_insert(a.T, key, &inserted);
          if (s < 0) atomicOr(&a.dsw->err, insert_error(s));
          nins += inserted ? 1 : 0;
        }
        sl = s < 0 ? kNoSlot : (uint32_t)s;
      } else {
        sl = a.slot[cidx];
      }
      const bool dead = sl == kNoSlot;
      if (dead) {
        h = make_float4(0.f, __int_as_float(-1), 0.f, 0.f);
        fc = 0.f;
      } else if (!home) {
        const Entry* en = ent_at(a.T, sl);
        h = *reinterpret_cast<const float4*>(en);
        fc = en->fea_cnt;
      }
      float4 e = make_float4(h.x, h.z, h.w, fc);  // {w, sqrt_g, z, fea_cnt}
      const int vrow = __float_as_int(h.y);
      const int vq = (vrow >= 0 && !(a.Pm.l1_shrk && e.x == 0.f)) ? vrow : -1;
      float gw = 0.f, xxp = 0.f;
      if (a.choff && len > (uint32_t)kChunkOcc) {
        const uint32_t c0 = a.choff[u];
        const uint32_t nc = hot_chunks_read((len + kChunkOcc - 1) / kChunkOcc);
        double gwd = 0, xxpd = 0;
        for (uint32_t c = 0; c < nc; ++c) {
          const double* pc = a.part + (int64_t)(c0 + c) * (d + 2);
          gwd += pc[0];
          xxpd += pc[1];
        }
        gw = (float)gwd;
        xxp = (float)xxpd;
      } else {
        // WU occurrences per trip, the next trip's rows in flight beside this trip's p reads
        // (one lane per key: a warm key's walk is this pass's longest chain); same order
        constexpr int WU = 8;
        uint32_t rw[WU];
        float xw[WU];
#pragma unroll
        for (int t = 0; t < WU; ++t) {
          const uint32_t i = s0 + t < s1 ? s0 + t : s1 - 1;
          rw[t] = occ_get(a, i, valued, false, &xw[t]);
        }
        for (uint32_t i0 = s0; i0 < s1; i0 += WU) {
          float pw[WU];
#pragma unroll
          for (int t = 0; t < WU; ++t)
            // (this pass reads no XV*p: the compact array whenever there is one)
            pw[t] = a.p ? a.p[rw[t]] : a.XVp[(int64_t)rw[t] * xs + d];
          const uint32_t in = i0 + WU;
          uint32_t rn[WU];
          float xn[WU];
#pragma unroll
          for (int t = 0; t < WU; ++t) {
            const uint32_t i = in + t < s1 ? in + t : s1 - 1;
            xn[t] = 1.f;
            rn[t] = in < s1 ? occ_get(a, i, valued, false, &xn[t]) : 0u;
          }
#pragma unroll
          for (int t = 0; t < WU; ++t) {
            if (i0 + t < s1 && pw[t] != 0.f) {
              if (valued) {
                gw += pw[t] * xw[t];
                xxp += pw[t] * (xw[t] * xw[t]);
              } else {
                gw += pw[t];
                xxp += pw[t];
              }
            }
          }
#pragma unroll
          for (int t = 0; t < WU; ++t) {
            rw[t] = rn[t];
            xw[t] = xn[t];
          }
        }
      }
      // Update(kGradient): UpdateW (FTRL); UpdateV by pass V if V was pulled
      bool tr;
      const int dw = ftrl_update(a.Pm, gw, &e, &tr);
      if (!dead) ent_store_hot(ent_at(a.T, sl), e, vrow);
      dnew += dead ? 0 : dw;
      const bool need = !dead && tr && d > 0 && vrow < 0 && e.w > (float)a.Pm.V_threshold;
      a.flags[u] = need ? 1u : 0u;
      if (need && a.insert_keys) a.slot[cidx] = sl;
      ninit += need ? 1 : 0;
      if (vq >= 0) {
        listed = true;
        // {first occurrence, or first chunk partial of a chunked key; V row; XXp; length}: pass
        // V starts on the key's walk without reading segstart / choff again
        const uint32_t first = (a.choff && len > (uint32_t)kChunkOcc) ? a.choff[u] : s0;
        item = make_uint4(first, (uint32_t)vq, __float_as_uint(xxp), len);
        nlive += 1u;
        nlocc += len;
      }
    }
    // the listed keys of this block: one append (returning atomics on one word serialise,
    // DESIGN.md (d); a wave each was 9.3 k of them at C5)
    const uint64_t m = __ballot(listed);
    const int wv = threadIdx.x / kWave;
    if (lane_id() == 0) wcnt[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int i = 0; i < kBwdWNT / kWave; ++i) {
        const uint32_t c = wcnt[i];
        wcnt[i] = t;
        t += c;
      }
      wbase = t ? atomicAdd(a.vcount, t) : 0u;
    }
    __syncthreads();
    if (listed) a.vlist[wbase + wcnt[wv] + (uint32_t)__popcll(m & lanemask_lt())] = item;
    __syncthreads();
  }
  for (int off = 32; off > 0; off >>= 1) {
    dnew += __shfl_xor(dnew, off, kWave);
    ninit += __shfl_xor(ninit, off, kWave);
    nins += __shfl_xor(nins, off, kWave);
    nlive += __shfl_xor(nlive, off, kWave);
    nlocc += __shfl_xor(nlocc, off, kWave);
  }
  if (lane_id() == 0) {
    red[threadIdx.x / kWave] = dnew;
    redn[threadIdx.x / kWave] = ninit;
    redi[threadIdx.x / kWave] = nins;
    redl[threadIdx.x / kWave] = nlive;
    redo[threadIdx.x / kWave] = nlocc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0, q = 0, i2 = 0;
    unsigned long long lv = 0, lo = 0;
    for (int i = 0; i < kBwdWNT / kWave; ++i) {
      s += red[i];
      q += redn[i];
      i2 += redi[i];
      lv += redl[i];
      lo += redo[i];
    }
    a.wstat[blockIdx.x] = make_int4(s, q, i2, 0);
    if (a.live_part) a.live_part[blockIdx.x] = make_uint2((unsigned)lv, (unsigned)lo);
  }
}

// pass W's per-block counts into the step's counters (by pass V's first block: pass W's blocks
// each adding theirs serialised on the three words)
__device__ inline void bwd_fold_wstat(const BwdArgs& a) {
  __shared__ long long rs[kFmNT / kWave];
  __shared__ unsigned rq[kFmNT / kWave];
  __shared__ unsigned long long ri[kFmNT / kWave];
  long long s = 0;
  unsigned q = 0;
  unsigned long long i2 = 0;
  for (int i = threadIdx.x; i < a.nwstat; i += kFmNT) {
    const int4 w = a.wstat[i];
    s += w.x;
    q += (unsigned)w.y;
    i2 += (unsigned long long)w.z;
  }
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off, kWave);
    q += __shfl_xor(q, off, kWave);
    i2 += __shfl_xor(i2, off, kWave);
  }
  if (lane_id() == 0) {
    rs[threadIdx.x / kWave] = s;
    rq[threadIdx.x / kWave] = q;
    ri[threadIdx.x / kWave] = i2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kFmNT / kWave; ++i) {
      s += rs[i];
      q += rq[i];
      i2 += ri[i];
    }
    if (s) atomicAdd((unsigned long long*)&a.dsw->new_w, (unsigned long long)s);
    if (q) atomicAdd(&a.dsw->n_init, q);
    if (i2) atomicAdd(&a.dsw->n_keys, i2);
  }
}

template <int G, int CPL>
__global__ __launch_bounds__(kFmNT) void k_fm_bwd_v(BwdArgs a) {
  constexpr int EPB = kFmNT / G;
  constexpr int UNR = CPL <= 4 ? 8 : 2;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  if (blockIdx.x == 0) bwd_fold_wstat(a);
  const int64_t n = (int64_t)*a.vcount;
  const int d = a.d;
  const int64_t xs = a.xs > d ? a.xs : d;
  const bool valued = a.occ_x != nullptr;
  for (int64_t j = (int64_t)blockIdx.x * EPB + g; j < n; j += (int64_t)gridDim.x * EPB) {
    const uint4 it = a.vlist[j];
    const int vq = (int)it.y;
    const float xxp = __uint_as_float(it.z);
    const uint32_t len = it.w;
    const uint32_t s0 = it.x, s1 = s0 + len;  // (it.x is the first chunk of a chunked key)
    float vcur[CPL], ccur[CPL], acc[CPL];
    load_coords<CPL, true>(row_V(a.T, vq), l, d, vcur);
    load_coords<CPL, true>(row_C(a.T, vq), l, d, ccur);
    // grad_u = (g0 - V*XXp) + sum (XV_ p) x, g0 = 0 (fm_loss.h:185-202, spmm.h:127-159)
    if (a.choff && len > (uint32_t)kChunkOcc) {
      const uint32_t c0 = it.x;
      const uint32_t nc = hot_chunks_read((len + kChunkOcc - 1) / kChunkOcc);
      double accp[CPL];
#pragma unroll
      for (int k = 0; k < CPL; ++k) accp[k] = 0;
      for (uint32_t c = 0; c < nc; ++c) {
        const double* pc = a.part + (int64_t)(c0 + c) * (d + 2);
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const int cd = l * CPL + k;
          accp[k] += cd < d ? pc[2 + cd] : 0.0;
        }
      }
#pragma unroll
      for (int k = 0; k < CPL; ++k)
        acc[k] = (float)((double)(0.f - vcur[k] * xxp) + accp[k]);
    } else {
#pragma unroll
      for (int k = 0; k < CPL; ++k) acc[k] = 0.f - vcur[k] * xxp;
      // G occurrences per trip: lane l reads occurrence i0 + l's row and value, UNR XV*p rows
      // in flight per sub-trip with their row ids shuffled from those lanes (occurrence order)
      const int gb = (int)(threadIdx.x % kWave) - l;
      for (uint32_t i0 = s0; i0 < s1; i0 += G) {
        const uint32_t i = i0 + (uint32_t)l < s1 ? i0 + (uint32_t)l : s1 - 1;
        float xl;
        const uint32_t rl = occ_get(a, i, valued, false, &xl);
        const uint32_t nt = s1 - i0 < (uint32_t)G ? s1 - i0 : (uint32_t)G;
#pragma unroll
        for (int t0 = 0; t0 < G; t0 += UNR) {
          if ((uint32_t)t0 >= nt) break;  // group-uniform
          float xw[UNR], xrw[UNR][CPL];
#pragma unroll
          for (int t = 0; t < UNR; ++t) {
            const uint32_t r = (uint32_t)__shfl((int)rl, gb + t0 + t, kWave);
            xw[t] = __shfl(xl, gb + t0 + t, kWave);
            load_coords<CPL, true>(a.XVp + (int64_t)r * xs, l, d, xrw[t]);
          }
#pragma unroll
          for (int t = 0; t < UNR; ++t) {
            if ((uint32_t)(t0 + t) < nt) {
#pragma unroll
              for (int k = 0; k < CPL; ++k)
                acc[k] = valued ? acc[k] + xrw[t][k] * xw[t] : acc[k] + xrw[t][k];
            }
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) adagrad_update(a.Pm, acc[k], &vcur[k], &ccur[k]);
    store_coords<CPL, true>(row_V(a.T, vq), l, d, vcur);
    store_coords<CPL, true>(row_C(a.T, vq), l, d, ccur);
  }
}

// one group per chunk of a long segment: partial {g_w, XXp, sum (XV p) x} over its
// kChunkOcc occurrences in order (the same terms as k_fm_bwd's walk)
template <int G, int CPL, bool VEC>
__device__ __attribute__((always_inline)) inline void chunk_one(const BwdArgs& a, int64_t ch,
                                                                int l) {
  constexpr int UNR = 4;
  const uint32_t u = a.chunk_seg[ch];
  const uint32_t s0 = a.segstart[u] + (uint32_t)(ch - a.choff[u]) * kChunkOcc;
  const uint32_t send = a.segstart[u + 1];
  const uint32_t s1 = s0 + kChunkOcc < send ? s0 + kChunkOcc : send;
  const bool valued = a.occ_x != nullptr;
  const int d = a.d;
  const int64_t xs = a.xs > d ? a.xs : d;
  double gw = 0, xxp = 0, acc[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) acc[k] = 0;
  if constexpr (G >= 8) {
    // G occurrences per trip, lane l reading occurrence i0 + l's row, value and p; the terms
    // shuffled from the lanes in occurrence order (bit-identical to the walk below), WU XV*p
    // rows in flight per sub-trip
    constexpr int WU = 8;
    const int gb = (int)(threadIdx.x % kWave) - l;
    for (uint32_t i0 = s0; i0 < s1; i0 += G) {
      const uint32_t i = i0 + (uint32_t)l < s1 ? i0 + (uint32_t)l : s1 - 1;
      float xl;
      const uint32_t rl = occ_get(a, i, valued, false, &xl);
      const float pl = row_p(a, rl, d, xs);
      const uint32_t n = s1 - i0 < (uint32_t)G ? s1 - i0 : (uint32_t)G;
#pragma unroll
      for (int t0 = 0; t0 < G; t0 += WU) {
        if ((uint32_t)t0 >= n) break;  // group-uniform
        float xw[WU], pw[WU], xr[WU][CPL];
#pragma unroll
        for (int u = 0; u < WU; ++u) {
          const uint32_t r = (uint32_t)__shfl((int)rl, gb + t0 + u, kWave);
          pw[u] = __shfl(pl, gb + t0 + u, kWave);
          xw[u] = __shfl(xl, gb + t0 + u, kWave);
          load_coords<CPL, VEC>(d > 0 ? a.XVp + (int64_t)r * xs : a.zpad, l, d, xr[u]);
        }
#pragma unroll
        for (int u = 0; u < WU; ++u) {
          if ((uint32_t)(t0 + u) >= n) continue;
          if (pw[u] != 0.f) {  // SpMV::TransTimes skips p == 0
            gw += valued ? (double)(pw[u] * xw[u]) : (double)pw[u];
            xxp += valued ? (double)(pw[u] * (xw[u] * xw[u])) : (double)pw[u];
          }
#pragma unroll
          for (int k = 0; k < CPL; ++k)
            acc[k] += valued ? (double)(xr[u][k] * xw[u]) : (double)xr[u][k];
        }
      }
    }
  }
  for (uint32_t i0 = s0; G < 8 && i0 < s1; i0 += UNR) {
    uint32_t rw[UNR];
    float xw[UNR], pw[UNR], xr[UNR][CPL];
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      const uint32_t i = i0 + t < s1 ? i0 + t : s1 - 1;
      rw[t] = occ_get(a, i, valued, false, &xw[t]);
    }
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      pw[t] = row_p(a, rw[t], d, xs);
      load_coords<CPL, false>(d > 0 ? a.XVp + (int64_t)rw[t] * xs : a.zpad, l, d, xr[t]);
    }
#pragma unroll
    for (int t = 0; t < UNR; ++t) {
      if (i0 + t >= s1) continue;
      if (pw[t] != 0.f) {  // SpMV::TransTimes skips p == 0
        // each term as the reference forms it in float, summed in double
        gw += valued ? (double)(pw[t] * xw[t]) : (double)pw[t];
        xxp += valued ? (double)(pw[t] * (xw[t] * xw[t])) : (double)pw[t];
      }
#pragma unroll
      for (int k = 0; k < CPL; ++k)
        acc[k] += valued ? (double)(xr[t][k] * xw[t]) : (double)xr[t][k];
    }
  }
  double* pc = a.part + ch * (d + 2);
  if (l == 0) {
    pc[0] = gw;
    pc[1] = xxp;
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int cd = l * CPL + k;
    if (cd < d) pc[2 + cd] = acc[k];
  }
}
// a bounded grid strides over the chunks: a batch with none (uniform keys) pays for a few
// thousand blocks that exit at once on every step otherwise
constexpr int kChunkGrid = 2048;
template <int G, int CPL, bool VEC = false>
__global__ __launch_bounds__(kFmNT) void k_fm_bwd_chunks(BwdArgs a) {
  constexpr int CPB = kFmNT / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int64_t nch = (int64_t)*a.nchunks;
  for (int64_t ch = (int64_t)blockIdx.x * CPB + g; ch < nch; ch += (int64_t)gridDim.x * CPB)
    chunk_one<G, CPL, VEC>(a, ch, l);
}

// A key of >= kHotChunks chunks (the hottest keys of a skewed batch: C5's top key has ~3500
// chunks of 128 occurrences) gets its chunk partials pre-summed in two fixed-shape levels, and
// the total written over its first chunk's partial; the backward then reads that one partial.
// Level 1 (k_chunk_hotgroup): a thread per (chunk, value) sums the kHotGroup chunks of its
// group in chunk order into the group's first chunk.  Level 2 (k_chunk_hotsum): a wave per hot
// key sums the group totals in R = 64 / (d + 2) interleaved slices, then the slices in order.
// Both orders are fixed by the batch, in double: deterministic.  Round 4 walked all of a hot
// key's partials serially (~110 round trips of 16 loads for the top key), C5's longest chain
// after the chunks.
constexpr int kHotGroup = 32, kHotNT = 1024, kHotGrid = 256;
__device__ inline void hotgroup_one(const BwdArgs& a, int64_t i) {
  const int P = a.d + 2;
  const int64_t ch = i / P;
  const int j = (int)(i - ch * P);
  const uint32_t u = a.chunk_seg[ch];
  const uint32_t c0 = a.choff[u];
  const uint32_t k = (uint32_t)ch - c0;
  if (k % kHotGroup) return;
  const uint32_t len = a.segstart[u + 1] - a.segstart[u];
  const uint32_t nc = (len + kChunkOcc - 1) / kChunkOcc;
  if (nc < kHotChunks) return;
  const uint32_t n = nc - k < (uint32_t)kHotGroup ? nc - k : (uint32_t)kHotGroup;
  const double* pj = a.part + ch * P + j;
  double v[kHotGroup];
#pragma unroll
  for (int q = 0; q < kHotGroup; ++q) v[q] = (uint32_t)q < n ? pj[(int64_t)q * P] : 0.0;
  double s = 0;
#pragma unroll
  for (int q = 0; q < kHotGroup; ++q)
    if ((uint32_t)q < n) s += v[q];
  a.part[ch * P + j] = s;
}
__global__ __launch_bounds__(256) void k_chunk_hotgroup(BwdArgs a) {
  const int64_t n = (int64_t)*a.nchunks * (a.d + 2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    hotgroup_one(a, i);
}
__device__ inline void hotsum_key(const BwdArgs& a, uint32_t c0, uint32_t nc, double* part_w) {
  const int P = a.d + 2;
  const uint32_t ng = (nc + kHotGroup - 1) / kHotGroup;  // group totals, kHotGroup apart
  const int R = P <= 64 ? 64 / P : 1;                   // slices
  constexpr int U = 8;
  const int l = threadIdx.x & 63;
  for (int j0 = 0; j0 < P; j0 += 64) {  // P > 64: value blocks of 64, one slice
    const int r = R > 1 ? l / P : 0, j = R > 1 ? l % P : j0 + l;
    double s = 0;
    if (r < R && j < P) {
      const double* pj = a.part + (int64_t)c0 * P + j;
      const int64_t gs = (int64_t)kHotGroup * P;
      uint32_t g = (uint32_t)r;
      for (; g + (uint32_t)(U - 1) * R < ng; g += (uint32_t)U * R) {
        double v[U];
#pragma unroll
        for (int q = 0; q < U; ++q) v[q] = pj[(int64_t)(g + (uint32_t)q * R) * gs];
#pragma unroll
        for (int q = 0; q < U; ++q) s += v[q];
      }
      for (; g < ng; g += (uint32_t)R) s += pj[(int64_t)g * gs];
    }
    if (R > 1) {
      part_w[l] = s;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (l < P) {
        double tot = 0;
        for (int q = 0; q < R; ++q) tot += part_w[q * P + l];
        a.part[(int64_t)c0 * P + l] = tot;
      }
      return;
    }
    if (j < P) a.part[(int64_t)c0 * P + j] = s;
  }
}
// kHotGrid blocks scan the chunk table kHotNT chunks at a time (a block per tile, tiles strided
// over the grid), list the tile's hot keys (first chunks of segments of >= kHotChunks chunks)
// in LDS, then sum the listed keys a wave per key.
__global__ __launch_bounds__(kHotNT) void k_chunk_hotsum(BwdArgs a) {
  __shared__ double part_w[kHotNT];
  __shared__ uint32_t s_c0[kHotNT], s_nc[kHotNT];
  __shared__ int s_n;
  const uint32_t nch = *a.nchunks;
  const int w = threadIdx.x >> 6;
  for (uint32_t base = blockIdx.x * (uint32_t)kHotNT; base < nch; base += gridDim.x * (uint32_t)kHotNT) {
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const uint32_t ch = base + threadIdx.x;
    if (ch < nch) {
      const uint32_t u = a.chunk_seg[ch];
      if (ch == a.choff[u]) {
        const uint32_t len = a.segstart[u + 1] - a.segstart[u];
        const uint32_t nc = (len + kChunkOcc - 1) / kChunkOcc;
        if (nc >= kHotChunks) {
          const int i = atomicAdd(&s_n, 1);
          s_c0[i] = ch;
          s_nc[i] = nc;
        }
      }
    }
    __syncthreads();
    const int n = s_n;
    for (int i = w; i < n; i += kHotNT / 64) hotsum_key(a, s_c0[i], s_nc[i], part_w + w * 64);
    __syncthreads();
  }
}

// row_p reads p from the [XV*p | p] row only when the row holds it (xs > d): rows of d floats
// need the per-row array (a null p there would read the next row's first XV*p)
static int check_row_p(const BwdArgs& a) {
  DFX_CHECK_ARG(!(a.d > 0 && a.xs <= a.d && !a.p),
                "backward: XV*p rows without p need the per-row p array");
  return DFX_OK;
}

int launch_bwd_chunks(const BwdArgs& a, int64_t chunk_bound, hipStream_t st, bool aligned) {
  if (chunk_bound <= 0 || !a.choff) return DFX_OK;
  DFX_TRY(check_row_p(a));
  int G, CPL;
  bool vec;
  // aligned (the fused steps' 16-byte XV*p rows, V_dim a multiple of 4): float4 per lane, a
  // chunk on d / 4 lanes (same per-coordinate sums: the partials are bit-identical)
  lanes_for(a.d, aligned && a.d >= 64, &G, &CPL, &vec);
  const int64_t cpb = kFmNT / G;
  dim3 grid((unsigned)std::min<int64_t>(kChunkGrid, (chunk_bound + cpb - 1) / cpb));
#define DFX_BWDC(GG, CC, VV)                                                              \
  if (G == GG && CPL == CC && vec == VV) {                                                \
    hipLaunchKernelGGL((k_fm_bwd_chunks<GG, CC, VV>), grid, dim3(kFmNT), 0, st, a);      \
    DFX_HIP(hipGetLastError());                                                           \
    if (chunk_bound >= (int64_t)kHotChunks) {                                             \
      hipLaunchKernelGGL(k_chunk_hotgroup,                                                  \
                         dim3((unsigned)std::min<int64_t>(kChunkGrid, (chunk_bound * (a.d + 2) + 255) / 256)), \
                         dim3(256), 0, st, a);                                              \
      hipLaunchKernelGGL(k_chunk_hotsum,                                                    \
                         dim3((unsigned)std::min<int64_t>(kHotGrid, (chunk_bound + kHotNT - 1) / kHotNT)), \
                         dim3(kHotNT), 0, st, a);                                           \
      DFX_HIP(hipGetLastError());                                                         \
    }                                                                                     \
    return DFX_OK;                                                                        \
  }
  DFX_SCALAR_SET(DFX_BWDC)
  DFX_BWDC(16, 4, true) DFX_BWDC(32, 4, true) DFX_BWDC(64, 4, true)
#undef DFX_BWDC
  set_error("unsupported V_dim");
  return DFX_ERR_ARG;
}

// The fused backward would fill every wave slot (8 waves / SIMD); reserving 32 KiB of LDS per
// block caps it at 5 blocks (20 waves) per CU, so the Localizer and AUC lanes' blocks always
// find slots beside it — their look-back chains then do not stall behind it.  Same-box A/B:
// +3 % step throughput, the backward itself unchanged (5 waves / SIMD already saturate its
// random-line traffic).  The context kwarg bwd_lds overrides (bytes, 0 = no cap).
constexpr size_t kBwdLdsCap = 32768;
// The one-kernel fused backward (V_dim < 128) since round 4's lighter lanes (bucket Localizer,
// radix AUC): 16 KiB, i.e. up to 10 blocks by LDS (8 by wave slots).  Same-box A/B at C3:
// 32 KiB 123.4, 20 KiB 126.9, 16 KiB 127.7 M ex/s (backward 0.53 -> 0.42 ms).  Round 5's close:
// 12 KiB, C3 +0.25 to +0.5 % over eight same-box rounds, C2 and the C4 shard a tie.
constexpr size_t kBwdLdsCapFused = 12288;

// Lane layout of a fused backward.  kwarg bwd_cpl = 8 at V_dim >= 64 (float4-aligned rows):
// two float4 per lane, half the lanes per key — a key's walk (entry, rows, update) is latency
// bound, and the keys of a batch that carry no V (lazy V) keep only lane 0 busy, so fewer lanes
// per key are more keys in flight per wave.  Every coordinate's terms stay one lane's, in the
// same order: bit-identical to the 4-per-lane layout.
static void bwd_lanes(const BwdArgs& a, bool aligned, int* G, int* CPL, bool* vec) {
  lanes_for(a.d, aligned, G, CPL, vec);
  const int from = a.cpl_from > 0 ? a.cpl_from : 64;
  if (!(*vec && *CPL == 4 && a.d >= from && a.d <= 512)) return;
  for (int c = a.cpl; c >= 8; c /= 2) {  // 16 -> 8 when d is not a multiple of 16
    const int g = *G * 4 / c;
    if (g >= 2 && a.d % c == 0) {
      *G = g;
      *CPL = c;
      return;
    }
  }
}

template <bool FUSED>
int launch_bwd(const BwdArgs& a, int64_t nseg_bound, hipStream_t st, bool aligned = FUSED,
               long lds = -1) {
  const size_t lds_bytes = lds >= 0 ? (size_t)lds : (FUSED ? kBwdLdsCapFused : 0);
  if (nseg_bound <= 0) return DFX_OK;
  int G, CPL;
  bool vec;
  bwd_lanes(a, aligned, &G, &CPL, &vec);
  const int64_t spb = kFmNT / G;
  dim3 grid((unsigned)((nseg_bound + spb - 1) / spb));
#define DFX_BWD(GG, CC, VV)                                                              \
  if (G == GG && CPL == CC && vec == VV) {                                               \
    hipLaunchKernelGGL((k_fm_bwd<GG, CC, FUSED, VV>), grid, dim3(kFmNT), lds_bytes, st, a);  \
    DFX_HIP(hipGetLastError());                                                          \
    return DFX_OK;                                                                       \
  }
  DFX_SCALAR_SET(DFX_BWD)
  DFX_VEC_SET(DFX_BWD)
  if constexpr (FUSED) {
    DFX_BWD(2, 8, true) DFX_BWD(4, 8, true) DFX_BWD(8, 8, true) DFX_BWD(16, 8, true)
    DFX_BWD(32, 8, true) DFX_BWD(64, 8, true)
    DFX_BWD(4, 16, true) DFX_BWD(8, 16, true) DFX_BWD(16, 16, true)
  }
#undef DFX_BWD
  set_error("unsupported V_dim");
  return DFX_ERR_ARG;
}

// the two-pass backward's resident grid (blocks per pass)
constexpr int64_t kBwdPassBlocks = 4096;
constexpr int64_t kBwdPassVBlocks = 32768;

// V_dim whose backward runs in two passes (k_fm_bwd_w + k_fm_bwd_v): G >= 32 lanes per key
bool bwd_two_pass(int d) {
  int G, CPL;
  bool vec;
  lanes_for(d, true, &G, &CPL, &vec);
  return vec && CPL == 4 && G >= 32;
}

int launch_bwd_fused(const BwdArgs& a, int64_t nseg_bound, hipStream_t st, long lds) {
  DFX_TRY(check_row_p(a));
  if (!a.vlist) return launch_bwd<true>(a, nseg_bound, st, true, lds);
  if (nseg_bound <= 0) return DFX_OK;
  int G, CPL;
  bool vec;
  lanes_for(a.d, true, &G, &CPL, &vec);
  if (!(vec && CPL == 4 && (G == 32 || G == 64))) {
    set_error("two-pass backward: V_dim a multiple of 4, 32 or 64 lanes per key");
    return DFX_ERR_ARG;
  }
  // pass V keeps one float4 per lane: two per lane measured worse (C5 92.2 -> 87.1 M ex/s,
  // pass V holds only the keys with V, whose walks fill its lanes)
  const size_t lds_bytes = lds >= 0 ? (size_t)lds : kBwdLdsCap;
  DFX_HIP(hipMemsetAsync(a.vcount, 0, sizeof(uint32_t), st));
  const int64_t gw = std::min<int64_t>((nseg_bound + kBwdWNT - 1) / kBwdWNT, kBwdPassBlocks);
  if (!a.wstat || gw > a.nwstat) {
    set_error("two-pass backward: block counts reserved for fewer blocks than launched");
    return DFX_ERR_ARG;
  }
  BwdArgs b = a;
  b.nwstat = (int32_t)gw;
  hipLaunchKernelGGL(k_fm_bwd_w, dim3((unsigned)gw), dim3(kBwdWNT), 0, st, b);
  const int64_t epb = kFmNT / G;
  // pass V: enough blocks that a group takes about one listed key (blocks past the list exit
  // at once) — the list's keys differ widely in walk length, and a resident grid's stride
  // loop stacked several long walks on one group
  const int64_t gv = std::min<int64_t>((nseg_bound + epb - 1) / epb, kBwdPassVBlocks);
  if (G == 32)
    hipLaunchKernelGGL((k_fm_bwd_v<32, 4>), dim3((unsigned)gv), dim3(kFmNT), lds_bytes, st, b);
  else
    hipLaunchKernelGGL((k_fm_bwd_v<64, 4>), dim3((unsigned)gv), dim3(kFmNT), lds_bytes, st, b);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

int bwd_two_pass_reserve(Context* c, Workspace& ws, int64_t nseg_bound, BwdArgs* g) {
  g->vlist = nullptr;
  g->vcount = nullptr;
  if (c->bwd_two_pass == 0 || !bwd_two_pass(c->P.V_dim) || nseg_bound <= 0) return DFX_OK;
  const int64_t nw = bwd_fused_blocks(c->P.V_dim, nseg_bound, true, 0);
  DFX_TRY(ws.vlist.ensure((size_t)(nseg_bound + 1 + nw) * sizeof(uint4)));
  g->vlist = ws.vlist.as<uint4>();
  g->vcount = reinterpret_cast<uint32_t*>(g->vlist + nseg_bound);
  g->wstat = reinterpret_cast<int4*>(g->vlist + nseg_bound + 1);
  g->nwstat = (int32_t)nw;
  return DFX_OK;
}

// blocks of the fused backward over nseg_bound keys (the size of BwdArgs::live_part)
int64_t bwd_fused_blocks(int d, int64_t nseg_bound, bool two_pass, int cpl) {
  if (two_pass) return std::min<int64_t>((nseg_bound + kBwdWNT - 1) / kBwdWNT, kBwdPassBlocks);
  int G, CPL;
  bool vec;
  BwdArgs a{};
  a.d = d;
  a.cpl = cpl & 0xFF;
  a.cpl_from = cpl >> 8;
  bwd_lanes(a, true, &G, &CPL, &vec);
  const int64_t spb = kFmNT / G;
  return (nseg_bound + spb - 1) / spb;
}

// the diagnostic live-V counts of one backward: its blocks' partials into the counters
__global__ void k_sum_live(const uint2* part, int64_t n, DevState* ds) {
  __shared__ unsigned long long r0[1024 / kWave], r1[1024 / kWave];
  unsigned long long a = 0, b = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    a += part[i].x;
    b += part[i].y;
  }
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, kWave);
    b += __shfl_xor(b, off, kWave);
  }
  if (lane_id() == 0) {
    r0[threadIdx.x / kWave] = a;
    r1[threadIdx.x / kWave] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x / kWave); ++i) {
      a += r0[i];
      b += r1[i];
    }
    ds->live_keys += a;
    ds->live_occ += b;
  }
}

int sum_live(const uint2* part, int64_t n, DevState* ds, hipStream_t st) {
  hipLaunchKernelGGL(k_sum_live, dim3(1), dim3(1024), 0, st, part, n, ds);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}

// sharded store: per-key gradient records in the pulled-record layout (aligned rows)
int launch_bwd_positions(const BwdArgs& a, int64_t nseg_bound, hipStream_t st) {
  return launch_bwd<false>(a, nseg_bound, st, true);
}

// ---- standalone CalcGrad support: CSC order of a compacted block ------------------------
__global__ void k_csc_prep(int64_t B, const uint64_t* __restrict__ offs,
                           const uint32_t* __restrict__ col, uint32_t* __restrict__ keys,
                           uint32_t* __restrict__ pos, uint32_t* __restrict__ rowid) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
    keys[j] = col[j];
    pos[j] = (uint32_t)j;
    rowid[j] = (uint32_t)r;
  }
}

// segments of the sorted column list: head flags -> scan -> segstart/segcol
__global__ void k_csc_heads(const uint32_t* k0, const uint32_t* k1, int64_t n,
                            const DevState* ds, uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* K = ds->sortmeta[31] ? k1 : k0;
  flags[i] = (i == 0 || K[i] != K[i - 1]) ? 1u : 0u;
}

__global__ void k_csc_segs(const uint32_t* k0, const uint32_t* k1, const uint32_t* p0,
                           const uint32_t* p1, int64_t n, const DevState* ds,
                           const uint32_t* excl, uint32_t* segstart, uint32_t* segcol,
                           const uint32_t* total, const uint32_t* rowid, const float* val,
                           uint32_t* occ_row, float* occ_x) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* K = ds->sortmeta[31] ? k1 : k0;
  const uint32_t* P = ds->sortmeta[31] ? p1 : p0;
  const uint32_t pos = P[i];
  occ_row[i] = rowid[pos];
  if (val) occ_x[i] = val[pos];
  const bool head = (i == 0 || K[i] != K[i - 1]);
  if (head) {
    segstart[excl[i]] = (uint32_t)i;
    segcol[excl[i]] = K[i];
  }
  if (i == n - 1) segstart[*total] = (uint32_t)n;
}

int get_nbits(int64_t n) {
  int b = 0;
  while (b < 32 && ((int64_t)1 << b) < n) ++b;
  return b;
}

}  // namespace dfx

using namespace dfx;

extern "C" int dfx_fm_predict(dfx_ctx* ctx, int64_t B, int64_t nnz, const uint64_t* offset,
                              const uint32_t* col, const float* value, const float* weights,
                              const int32_t* w_pos, const int32_t* V_pos, int64_t n_cols,
                              int V_dim, float* pred) {
  DFX_CHECK_ARG(ctx, "null ctx");
  DFX_CHECK_ARG(B >= 0 && nnz >= 0 && V_dim >= 0 && V_dim <= 1024, "fm_predict: bad sizes");
  DFX_CHECK_ARG(V_dim == 0 || (w_pos && V_pos), "fm_predict: V_dim > 0 needs w_pos and V_pos");
  if (B == 0) return DFX_OK;
  DFX_CHECK_ARG(offset && pred && (nnz == 0 || (col && weights)), "fm_predict: null buffer");
  (void)n_cols;
  FwdArgs a{};
  a.B = B; a.offs = offset; a.col = col; a.val = value; a.W = weights; a.wpos = w_pos;
  a.vpos = V_pos; a.Vbase = weights; a.zpad = ctx->c.zpad; a.d = V_dim; a.pred = pred;
  return launch_fwd<kPredict, false>(a, ctx->c.stream);
}

extern "C" int dfx_fm_calcgrad(dfx_ctx* ctx, int64_t B, int64_t nnz, const uint64_t* offset,
                               const uint32_t* col, const float* value, const float* label,
                               const float* row_weight, const float* weights,
                               const int32_t* w_pos, const int32_t* V_pos, int64_t n_cols,
                               int V_dim, const float* pred, float* grad) {
  DFX_CHECK_ARG(ctx, "null ctx");
  Context* c = &ctx->c;
  DFX_CHECK_ARG(B >= 0 && nnz >= 0 && V_dim >= 0 && V_dim <= 1024, "fm_calcgrad: bad sizes");
  DFX_CHECK_ARG(V_dim == 0 || (w_pos && V_pos), "fm_calcgrad: V_dim > 0 needs w_pos and V_pos");
  DFX_CHECK_ARG(n_cols >= 0 && n_cols < 0xFFFFFFFFll, "fm_calcgrad: bad n_cols");
  if (B == 0 || nnz == 0) return DFX_OK;
  DFX_CHECK_ARG(offset && col && label && weights && pred && grad, "fm_calcgrad: null buffer");
  Workspace& ws = c->ws;
  DFX_TRY(ws.p.ensure(B * 4));
  if (V_dim > 0) DFX_TRY(ws.XVp.ensure((size_t)B * V_dim * 4));
  DFX_TRY(ws.vals0.ensure(nnz * 4));
  DFX_TRY(ws.vals1.ensure(nnz * 4));
  DFX_TRY(ws.keys0.ensure(nnz * 4));
  DFX_TRY(ws.keys1.ensure(nnz * 4));
  DFX_TRY(ws.rowid.ensure(nnz * 4));
  DFX_TRY(ws.flags.ensure((nnz + 1) * 4));
  DFX_TRY(ws.segstart.ensure((nnz + 1) * 4));
  DFX_TRY(ws.slot.ensure((nnz + 1) * 4));
  DFX_TRY(ws.occ_row.ensure(nnz * 4));
  DFX_TRY(ws.occ_x.ensure(nnz * 4));
  DFX_TRY(ws.cnt.ensure(4 * 4));
  DFX_TRY(ws.col.ensure((nnz + 1) * 4));                                      // chunk offsets
  DFX_TRY(ws.vpos.ensure(max_chunks(nnz) * 4));                         // chunk -> segment
  DFX_TRY(ws.Vb.ensure((size_t)max_chunks(nnz) * (V_dim + 2) * 8));    // chunk partials
  // 1) p and XV*p per row
  FwdArgs a{};
  a.B = B; a.offs = offset; a.col = col; a.val = value; a.W = weights; a.wpos = w_pos;
  a.vpos = V_pos; a.Vbase = weights; a.zpad = c->zpad; a.d = V_dim; a.label = label;
  a.rw = row_weight; a.pred_in = pred; a.p_out = ws.p.as<float>(); a.XVp = ws.XVp.as<float>();
  DFX_TRY((launch_fwd<kGradPrep, false>(a, c->stream)));
  // 2) CSC order: stable sort of (col, pos); occurrences' rows/values in that order
  uint32_t* k0 = ws.keys0.as<uint32_t>();
  uint32_t* k1 = ws.keys1.as<uint32_t>();
  hipLaunchKernelGGL(k_csc_prep, dim3((B + 255) / 256), dim3(256), 0, c->stream, B, offset, col,
                     k0, ws.vals0.as<uint32_t>(), ws.rowid.as<uint32_t>());
  DFX_TRY(radix_sort_pairs<uint32_t>(main_lane(c), k0, ws.vals0.as<uint32_t>(), k1,
                                     ws.vals1.as<uint32_t>(), nnz, 0, get_nbits(n_cols),
                                     nullptr, c->ds->sortmeta));
  uint32_t* flags = ws.flags.as<uint32_t>();
  uint32_t* total = ws.cnt.as<uint32_t>();
  hipLaunchKernelGGL(k_csc_heads, dim3((nnz + 255) / 256), dim3(256), 0, c->stream, k0, k1, nnz,
                     c->ds, flags);
  DFX_TRY(scan_u32(c, flags, nnz, total));
  hipLaunchKernelGGL(k_csc_segs, dim3((nnz + 255) / 256), dim3(256), 0, c->stream, k0, k1,
                     ws.vals0.as<uint32_t>(), ws.vals1.as<uint32_t>(), nnz, c->ds, flags,
                     ws.segstart.as<uint32_t>(), ws.slot.as<uint32_t>(), total,
                     ws.rowid.as<uint32_t>(), value, ws.occ_row.as<uint32_t>(),
                     ws.occ_x.as<float>());
  // 3) long segments (skewed keys) in chunks, combined in double (as in the fused step)
  DFX_HIP(hipMemcpyAsync(&c->ds->u_count, total, sizeof(uint32_t), hipMemcpyDeviceToDevice,
                         c->stream));
  // the plan's gate open: it counts every segment's chunks (k_chunk_plan), none is skipped
  DFX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&c->ds->n_init), 1, 1, c->stream));
  uint32_t* choff = ws.col.as<uint32_t>();
  uint32_t* chunk_seg = ws.vpos.as<uint32_t>();
  uint32_t* nchunks = total + 1;
  DFX_TRY(chunk_plan(main_lane(c), nnz, ws.segstart.as<uint32_t>(), choff, chunk_seg, nchunks));
  // 4) segmented reduction into grad
  BwdArgs b{};
  b.segstart = ws.segstart.as<uint32_t>();
  b.ds = c->ds;
  b.nseg_host = -1;
  b.segcol = ws.slot.as<uint32_t>();
  b.occ_row = ws.occ_row.as<uint32_t>();
  b.occ_x = value ? ws.occ_x.as<float>() : nullptr;
  b.zpad = c->zpad;
  b.p = ws.p.as<float>(); b.XVp = ws.XVp.as<float>(); b.d = V_dim;
  b.wpos = w_pos; b.vpos = V_pos; b.W = weights; b.grad = grad;
  b.choff = choff; b.chunk_seg = chunk_seg; b.nchunks = nchunks; b.part = ws.Vb.as<double>();
  // the number of segments is device-side (ds->u_count, set above), where k_fm_bwd reads it
  DFX_TRY(launch_bwd_chunks(b, max_chunks(nnz), c->stream, false));
  DFX_TRY(launch_bwd<false>(b, nnz, c->stream));
  // n_init served as the chunk plan's gate; it counts the fused step's InitV requests
  DFX_HIP(hipMemsetAsync(&c->ds->n_init, 0, sizeof(uint32_t), c->stream));
  return DFX_OK;
}

__global__ void k_get_pos(int64_t n, const int32_t* lens, const uint32_t* excl, int32_t* w_pos,
                          int32_t* V_pos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int l = lens[i];
  const int p = (int)excl[i];
  w_pos[i] = l == 0 ? -1 : p;
  V_pos[i] = l > 1 ? p + 1 : -1;
}

__global__ void k_copy_i32_u32(int64_t n, const int32_t* a, uint32_t* b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (uint32_t)a[i];
}

// SGDLearner::GetPos (sgd_learner.cc:151-165)
extern "C" int dfx_get_pos(dfx_ctx* ctx, int64_t n, const int32_t* lens, int32_t* w_pos,
                           int32_t* V_pos) {
  DFX_CHECK_ARG(ctx, "null ctx");
  if (n <= 0) return DFX_OK;
  DFX_CHECK_ARG(lens && w_pos && V_pos, "get_pos: null buffer");
  Context* c = &ctx->c;
  DFX_TRY(c->ws.flags.ensure((n + 1) * 4));
  uint32_t* ex = c->ws.flags.as<uint32_t>();
  hipLaunchKernelGGL(k_copy_i32_u32, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, lens, ex);
  DFX_TRY(scan_u32(c, ex, n, nullptr));
  hipLaunchKernelGGL(k_get_pos, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, lens, ex,
                     w_pos, V_pos);
  DFX_HIP(hipGetLastError());
  return DFX_OK;
}
