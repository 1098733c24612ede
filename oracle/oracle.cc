// =====================================================================================
//  oracle/oracle.cc — CPU restatement of DiFacto's data-parallel hot path.
//
//  TEST INFRASTRUCTURE ONLY.  Nothing in the product (libdifacto_amd.so, difacto_amd/,
//  the C++ host adapters) links, imports or calls this file.  Only tests/, the
//  __graft_entry__.smoke() checker and bench.py's `cpu_baseline` leg load it.
//
//  Parity status: PINNED.  The reference (/root/reference) cannot be built here: its
//  dmlc-core and ps-lite submodules are empty and building it would need stand-in
//  headers, which this project does not write.  This restatement is instead checked
//  (tests/test_oracle.py) against every known-answer value the reference's own tests
//  hold for this path:
//    * Localizer.Base / BaseHash   tests/cpp/localizer_test.cc:26-27,48  (65111856, 9648, 478817)
//    * FMLoss.NoV / HasV           tests/cpp/fm_loss_test.cc:35,39,78,82 (147.4672, 90.5817,
//                                                                         330.628, 1237.8)
//    * SGDLearner.Basic            tests/cpp/sgd_learner_test.cc:10-30   (20-epoch objv trace)
//  on the reference's own fixture tests/data (copied to tests/golden/rcv1_100.libsvm).
//
//  Every function cites the reference lines whose arithmetic it restates.  Float
//  conventions copied on purpose: fp32 everywhere, row-ordered
//  sums, `float += double` in Predict, clip only when V_dim > 0, counts as float,
//  glibc expf / rand_r.  Build with -ffp-contract=off (the reference x86-64 build has
//  no FMA contraction).
// =====================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

typedef float real_t;
typedef uint64_t feaid_t;

namespace {

// include/difacto/base.h:39-51 — nibble-level reversal (swap 32,16,8,4-bit halves).
inline feaid_t ReverseBytes(feaid_t x) {
  x = x << 32 | x >> 32;
  x = (x & 0x0000FFFF0000FFFFULL) << 16 | (x & 0xFFFF0000FFFF0000ULL) >> 16;
  x = (x & 0x00FF00FF00FF00FFULL) << 8 | (x & 0xFF00FF00FF00FF00ULL) >> 8;
  x = (x & 0x0F0F0F0F0F0F0F0FULL) << 4 | (x & 0xF0F0F0F0F0F0F0F0ULL) >> 4;
  return x;
}

struct KeyPos { feaid_t k; uint32_t i; };

// src/sgd/sgd_param.h:79-123 (SGDUpdaterParam, defaults) + fm_loss.h:19-27 (V_dim)
struct UpdaterParam {
  float l1 = 1, l2 = 0, V_l2 = .01f, lr = .01f, lr_beta = 1, V_lr = .01f, V_lr_beta = 1,
        V_init_scale = .01f;
  int V_dim = 0, V_threshold = 10;
  bool l1_shrk = true;
  unsigned seed = 0;
  // not a reference parameter: sum64=1 makes orc_train_step sum every gradient column in
  // double and round once (the exact trajectory the C5 drift test measures both the device
  // and the reference against)
  bool sum64 = false;
};

bool ParseKW(const char* kwargs, UpdaterParam* p) {
  if (!kwargs) return true;
  std::string s(kwargs);
  for (char& c : s) if (c == ',' || c == '\n' || c == ';') c = ' ';
  std::istringstream is(s);
  std::string tok;
  while (is >> tok) {
    auto eq = tok.find('=');
    if (eq == std::string::npos) continue;
    std::string k = tok.substr(0, eq), v = tok.substr(eq + 1);
    std::istringstream vs(v);
    if (k == "l1") vs >> p->l1;
    else if (k == "l2") vs >> p->l2;
    else if (k == "V_l2") vs >> p->V_l2;
    else if (k == "lr") vs >> p->lr;
    else if (k == "lr_beta") vs >> p->lr_beta;
    else if (k == "V_lr") vs >> p->V_lr;
    else if (k == "V_lr_beta") vs >> p->V_lr_beta;
    else if (k == "V_init_scale") vs >> p->V_init_scale;
    else if (k == "V_dim") vs >> p->V_dim;
    else if (k == "V_threshold") vs >> p->V_threshold;
    else if (k == "l1_shrk") p->l1_shrk = !(v == "0" || v == "false");
    else if (k == "seed") vs >> p->seed;
    else if (k == "sum64") p->sum64 = !(v == "0" || v == "false");
  }
  return true;
}

// src/sgd/sgd_updater.h:20-69 — per-feature state.
struct Entry {
  real_t fea_cnt = 0;
  real_t w = 0, sqrt_g = 0, z = 0;
  std::vector<real_t> V;  // [V(d) | Vaux(d)] ; empty == nullptr in the reference
  int size = 1;
  bool empty() const { return w == 0 && size == 1; }
};

struct Updater {
  UpdaterParam param;
  std::unordered_map<feaid_t, Entry> model;
  float new_w = 0;

  // sgd_updater.cc:144-152
  void InitV(Entry* e) {
    int n = param.V_dim;
    e->V.assign(2 * n, 0.f);
    for (int i = 0; i < n; ++i) {
      e->V[i] = (rand_r(&param.seed) / (real_t)RAND_MAX - 0.5) * param.V_init_scale;
    }
    e->size = 1 + n;
  }
  // sgd_updater.cc:105-131 (FTRL)
  void UpdateW(real_t gw, Entry* e) {
    real_t sg = e->sqrt_g;
    real_t w = e->w;
    gw += w * param.l2;
    e->sqrt_g = std::sqrt(sg * sg + gw * gw);
    e->z -= gw - (e->sqrt_g - sg) / param.lr * w;
    real_t z = e->z;
    real_t l1 = param.l1;
    if (z <= l1 && z >= -l1) {
      e->w = 0;
    } else {
      real_t eta = (param.lr_beta + e->sqrt_g) / param.lr;
      e->w = (z > 0 ? z - l1 : z + l1) / eta;
    }
    if (w == 0 && e->w != 0) {
      ++new_w;
      if (param.V_dim > 0 && e->V.empty() && e->fea_cnt > param.V_threshold) InitV(e);
    } else if (w != 0 && e->w == 0) {
      --new_w;
    }
  }
  // sgd_updater.cc:133-142 (AdaGrad)
  void UpdateV(real_t const* gV, Entry* e) {
    int n = param.V_dim;
    for (int i = 0; i < n; ++i) {
      real_t g = gV[i] + param.V_l2 * e->V[i];
      real_t cg = e->V[i + n];
      e->V[i + n] = std::sqrt(cg * cg + g * g);
      float eta = param.V_lr / (e->V[i + n] + param.V_lr_beta);
      e->V[i] -= eta * g;
    }
  }
};

thread_local std::string g_err;

}  // namespace

extern "C" {

const char* orc_last_error() { return g_err.c_str(); }

uint64_t orc_reverse_bytes(uint64_t x) { return ReverseBytes(x); }

// ---------------------------------------------------------------------------------
// Localizer::Compact = CountUniqIndex (localizer.cc:11-49) + RemapIndex (:53-107).
// Input RowBlock<feaid_t>: offs[B+1] (offs[0] must be 0, as BatchReader produces),
// ids[nnz].  Outputs: uniq[U] (sorted, reversed keys), cnt[U] (float, nullable),
// col[nnz] (u32 column = rank).  Returns U.  Because the dictionary is built from
// the same block, every index matches, so offsets/values/labels pass through
// unchanged (RemapIndex keeps all of them) and max_index = U-1.
// nnz == 0: the reference reads pair_[0] out of bounds (localizer.cc:34); defined here
// as U = 0.
// ---------------------------------------------------------------------------------
int64_t orc_localize(int64_t B, const uint64_t* offs, const uint64_t* ids, uint64_t max_index,
                     uint64_t* uniq, float* cnt, uint32_t* col) {
  if (B <= 0) return 0;
  size_t nnz = offs[B];
  if (nnz == 0) return 0;
  std::vector<KeyPos> pr(nnz);
  for (size_t i = 0; i < nnz; ++i) { pr[i].k = ReverseBytes(ids[i] % max_index); pr[i].i = (uint32_t)i; }
  // ParallelSort (parallel_sort.h:14-39) is an unstable merge sort; ranks do not depend
  // on the order among equal keys, so any sort gives the same outputs.
  std::sort(pr.begin(), pr.end(), [](const KeyPos& a, const KeyPos& b) { return a.k < b.k; });
  int64_t U = 0;
  feaid_t curr = pr[0].k;
  real_t c = 0;
  for (size_t i = 0; i < nnz; ++i) {
    if (pr[i].k != curr) {
      uniq[U] = curr;
      if (cnt) cnt[U] = c;
      ++U;
      curr = pr[i].k;
      c = 0;
    }
    ++c;
    col[pr[i].i] = (uint32_t)U;  // merge-join with the dictionary == run rank
  }
  uniq[U] = curr;
  if (cnt) cnt[U] = c;
  ++U;
  return U;
}

// ---------------------------------------------------------------------------------
// FMLoss::Predict (fm_loss.h:67-119); with V_dim == 0 it is also LogitLoss::Predict
// (logit_loss.h:41-57).  pred accumulates (+=).  w_pos may be NULL when V_dim == 0
// (then w = weights[col]); V_pos is required when V_dim > 0.
// Sums run in (row, nnz) order exactly like SpMV::Times (spmv.h:107-134) and
// SpMM::Times (spmm.h:93-122), which are row-partitioned and therefore thread-count
// independent.
// ---------------------------------------------------------------------------------
void orc_fm_predict(int64_t B, const uint64_t* offs, const uint32_t* col, const float* val,
                    const float* weights, const int32_t* w_pos, const int32_t* V_pos, int V_dim,
                    float* pred) {
  std::vector<real_t> xv(V_dim), xxvv(V_dim);
  for (int64_t r = 0; r < B; ++r) {
    real_t y = pred[r];
    // SpMV::Times: skip w == 0 and w_pos == -1 (spmv.h:124-125,173-181)
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      real_t w;
      if (w_pos) { int p = w_pos[c]; w = p == -1 ? 0 : weights[p]; } else { w = weights[c]; }
      if (w == 0) continue;
      if (val) y += w * val[j]; else y += w;
    }
    if (V_dim == 0) { pred[r] = y; continue; }
    std::fill(xv.begin(), xv.end(), 0.f);
    std::fill(xxvv.begin(), xxvv.end(), 0.f);
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      int p = V_pos[col[j]];
      if (p == -1) continue;
      const float* V = weights + p;
      if (val) {
        real_t x = val[j];
        real_t xx = x * x;                 // XX_ (fm_loss.h:86-92)
        for (int l = 0; l < V_dim; ++l) {
          xv[l] += V[l] * x;
          real_t vv = V[l] * V[l];         // VV (fm_loss.h:95-101)
          xxvv[l] += vv * xx;
        }
      } else {
        for (int l = 0; l < V_dim; ++l) { xv[l] += V[l]; real_t vv = V[l] * V[l]; xxvv[l] += vv; }
      }
    }
    real_t s = 0;
    for (int l = 0; l < V_dim; ++l) s += xv[l] * xv[l] - xxvv[l];   // fm_loss.h:110-113
    y += .5 * s;                                                   // float += double (:114)
    y = y > 20 ? 20 : (y < -20 ? -20 : y);                         // clip (:118)
    pred[r] = y;
  }
}

// ---------------------------------------------------------------------------------
// FMLoss::CalcGrad (fm_loss.h:148-203) / LogitLoss::CalcGrad (logit_loss.h:71-103).
// grad accumulates (pre-zeroed by the caller).  ncol = number of columns (U).
// Column sums run in ascending (row, nnz) order, which is what the column-range
// partitioned SpMV/SpMM::TransTimes (spmv.h:139-171, spmm.h:127-159) produce for any
// thread count.
// ---------------------------------------------------------------------------------
}  // extern "C"

// A = float: the reference's arithmetic.  A = double (sum64): the same float terms, every
// column sum in double (the caller rounds once) — test infrastructure, not a reference mode.
template <typename A>
static void CalcGrad(int64_t B, const uint64_t* offs, const uint32_t* col, const float* val,
                     const float* label, const float* rweight, const float* weights,
                     const int32_t* w_pos, const int32_t* V_pos, int64_t ncol, int V_dim,
                     const float* pred, A* grad) {
  std::vector<real_t> p(B);
  for (int64_t i = 0; i < B; ++i) {                 // fm_loss.h:155-165
    real_t y = label[i] > 0 ? 1 : -1;
    if (rweight) p[i] = -y / (1 + std::exp(y * pred[i])) * rweight[i];
    else p[i] = -y / (1 + std::exp(y * pred[i]));
  }
  // grad_w = X' p  (SpMV::TransTimes with y_pos = w_pos; skips p == 0)
  for (int64_t r = 0; r < B; ++r) {
    real_t pr = p[r];
    if (pr == 0) continue;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      if ((int64_t)c >= ncol) continue;
      A* g;
      if (w_pos) { int q = w_pos[c]; if (q == -1) continue; g = grad + q; } else { g = grad + c; }
      if (val) *g += pr * val[j]; else *g += pr;
    }
  }
  if (V_dim == 0) return;
  // XXp = (X.*X)' p  (fm_loss.h:176-182)
  std::vector<A> XXp(ncol, 0.f);
  for (int64_t r = 0; r < B; ++r) {
    real_t pr = p[r];
    if (pr == 0) continue;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      if ((int64_t)c >= ncol) continue;
      if (val) { real_t xx = val[j] * val[j]; XXp[c] += pr * xx; } else { XXp[c] += pr; }
    }
  }
  // grad_V -= diag(XXp) V  (fm_loss.h:185-192)
  for (int64_t c = 0; c < ncol; ++c) {
    int q = V_pos[c];
    if (q == -1) continue;
    for (int l = 0; l < V_dim; ++l) grad[q + l] -= weights[q + l] * XXp[c];
  }
  // XV_ = X V, then XV_ *= p  (fm_loss.h:81-83, 196-199)
  std::vector<real_t> XVp((size_t)B * V_dim, 0.f);
  for (int64_t r = 0; r < B; ++r) {
    real_t* t = XVp.data() + (size_t)r * V_dim;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      int q = V_pos[col[j]];
      if (q == -1) continue;
      const float* V = weights + q;
      if (val) { real_t x = val[j]; for (int l = 0; l < V_dim; ++l) t[l] += V[l] * x; }
      else { for (int l = 0; l < V_dim; ++l) t[l] += V[l]; }
    }
    for (int l = 0; l < V_dim; ++l) t[l] *= p[r];
  }
  // grad_V += X' diag(p) X V  (SpMM::TransTimes, y_pos = V_pos; no p==0 skip)
  for (int64_t r = 0; r < B; ++r) {
    const real_t* t = XVp.data() + (size_t)r * V_dim;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      if ((int64_t)c >= ncol) continue;
      int q = V_pos[c];
      if (q == -1) continue;
      A* g = grad + q;
      if (val) { real_t x = val[j]; for (int l = 0; l < V_dim; ++l) g[l] += t[l] * x; }
      else { for (int l = 0; l < V_dim; ++l) g[l] += t[l]; }
    }
  }
}

// CalcGrad of a 1-step-stale split step (test infrastructure; DESIGN.md (e), split stale): the
// forward ran on an older model (fw_weights / fw_V_pos: what it read, so p and XV_ are the stale
// forward's), the backward reads the model as it is when the update runs (bw_weights / bw_w_pos /
// bw_V_pos: the gradient's layout and the V of the diag(XXp) V term).  With fw == bw this is
// CalcGrad<float> term for term.
static void CalcGradStale(int64_t B, const uint64_t* offs, const uint32_t* col, const float* val,
                          const float* label, const float* rweight, const float* fw_weights,
                          const int32_t* fw_V_pos, const float* bw_weights,
                          const int32_t* bw_w_pos, const int32_t* bw_V_pos, int64_t ncol,
                          int V_dim, const float* pred, float* grad) {
  std::vector<real_t> p(B);
  for (int64_t i = 0; i < B; ++i) {
    real_t y = label[i] > 0 ? 1 : -1;
    if (rweight) p[i] = -y / (1 + std::exp(y * pred[i])) * rweight[i];
    else p[i] = -y / (1 + std::exp(y * pred[i]));
  }
  for (int64_t r = 0; r < B; ++r) {
    real_t pr = p[r];
    if (pr == 0) continue;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      if ((int64_t)c >= ncol) continue;
      float* g;
      if (bw_w_pos) { int q = bw_w_pos[c]; if (q == -1) continue; g = grad + q; } else { g = grad + c; }
      if (val) *g += pr * val[j]; else *g += pr;
    }
  }
  if (V_dim == 0) return;
  std::vector<float> XXp(ncol, 0.f);
  for (int64_t r = 0; r < B; ++r) {
    real_t pr = p[r];
    if (pr == 0) continue;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      if ((int64_t)c >= ncol) continue;
      if (val) { real_t xx = val[j] * val[j]; XXp[c] += pr * xx; } else { XXp[c] += pr; }
    }
  }
  for (int64_t c = 0; c < ncol; ++c) {
    int q = bw_V_pos[c];
    if (q == -1) continue;
    for (int l = 0; l < V_dim; ++l) grad[q + l] -= bw_weights[q + l] * XXp[c];
  }
  std::vector<real_t> XVp((size_t)B * V_dim, 0.f);
  for (int64_t r = 0; r < B; ++r) {
    real_t* t = XVp.data() + (size_t)r * V_dim;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      int q = fw_V_pos[col[j]];
      if (q == -1) continue;
      const float* V = fw_weights + q;
      if (val) { real_t x = val[j]; for (int l = 0; l < V_dim; ++l) t[l] += V[l] * x; }
      else { for (int l = 0; l < V_dim; ++l) t[l] += V[l]; }
    }
    for (int l = 0; l < V_dim; ++l) t[l] *= p[r];
  }
  for (int64_t r = 0; r < B; ++r) {
    const real_t* t = XVp.data() + (size_t)r * V_dim;
    for (uint64_t j = offs[r]; j < offs[r + 1]; ++j) {
      uint32_t c = col[j];
      if ((int64_t)c >= ncol) continue;
      int q = bw_V_pos[c];
      if (q == -1) continue;
      float* g = grad + q;
      if (val) { real_t x = val[j]; for (int l = 0; l < V_dim; ++l) g[l] += t[l] * x; }
      else { for (int l = 0; l < V_dim; ++l) g[l] += t[l]; }
    }
  }
}

extern "C" {

void orc_fm_calcgrad_stale(int64_t B, const uint64_t* offs, const uint32_t* col,
                           const float* val, const float* label, const float* rweight,
                           const float* fw_weights, const int32_t* fw_V_pos,
                           const float* bw_weights, const int32_t* bw_w_pos,
                           const int32_t* bw_V_pos, int64_t ncol, int V_dim, const float* pred,
                           float* grad) {
  CalcGradStale(B, offs, col, val, label, rweight, fw_weights, fw_V_pos, bw_weights, bw_w_pos,
                bw_V_pos, ncol, V_dim, pred, grad);
}

void orc_fm_calcgrad(int64_t B, const uint64_t* offs, const uint32_t* col, const float* val,
                     const float* label, const float* rweight, const float* weights,
                     const int32_t* w_pos, const int32_t* V_pos, int64_t ncol, int V_dim,
                     const float* pred, float* grad) {
  CalcGrad<float>(B, offs, col, val, label, rweight, weights, w_pos, V_pos, ncol, V_dim, pred,
                  grad);
}

// Loss::Evaluate (loss.h:57-66): sum log(1+exp(-y pred)), y = label>0 ? 1 : -1.
double orc_evaluate(int64_t B, const float* label, const float* pred) {
  double objv = 0;
  for (int64_t i = 0; i < B; ++i) {
    double y = label[i] > 0 ? 1 : -1;
    objv += std::log(1 + std::exp(-y * (double)pred[i]));
  }
  return objv;
}

// BinClassMetric::AUC (bin_class_metric.h:35-57).  Returns AUC * n like the reference.
float orc_auc(int64_t n, const float* label, const float* pred) {
  struct E { float label; float predict; };
  std::vector<E> buf(n);
  for (int64_t i = 0; i < n; ++i) { buf[i].label = label[i]; buf[i].predict = pred[i]; }
  std::sort(buf.begin(), buf.end(), [](const E& a, const E& b) { return a.predict < b.predict; });
  real_t area = 0, cum_tp = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (buf[i].label > 0) cum_tp += 1; else area += cum_tp;
  }
  if (cum_tp == 0 || cum_tp == n) return 1;
  area /= cum_tp * (n - cum_tp);
  return (area < 0.5 ? 1 - area : area) * n;
}

// SGDLearner::GetPos (sgd_learner.cc:151-165)
void orc_get_pos(int64_t n, const int32_t* len, int32_t* w_pos, int32_t* V_pos) {
  int p = 0;
  for (int64_t i = 0; i < n; ++i) {
    int l = len[i];
    w_pos[i] = l == 0 ? -1 : p;
    V_pos[i] = l > 1 ? p + 1 : -1;
    p += l;
  }
}

// ---------------------------------------------------------------------------------
// SGDUpdater (sgd_updater.cc:34-152)
// ---------------------------------------------------------------------------------
void* orc_updater_create(const char* kwargs) {
  Updater* u = new Updater();
  ParseKW(kwargs, &u->param);
  return u;
}
void orc_updater_destroy(void* h) { delete static_cast<Updater*>(h); }
int orc_updater_vdim(void* h) { return static_cast<Updater*>(h)->param.V_dim; }
unsigned orc_updater_seed(void* h) { return static_cast<Updater*>(h)->param.seed; }
float orc_updater_new_w(void* h) { return static_cast<Updater*>(h)->new_w; }
int64_t orc_updater_size(void* h) { return (int64_t)static_cast<Updater*>(h)->model.size(); }

// SGDUpdater::Get (sgd_updater.cc:34-58).  vals must hold U*(1+d); lens U (or NULL if
// d == 0).  Returns the number of values written.  Inserts missing keys like model_[k].
int64_t orc_updater_get(void* h, const uint64_t* keys, int64_t U, float* vals, int32_t* lens) {
  Updater* up = static_cast<Updater*>(h);
  int d = up->param.V_dim;
  int64_t p = 0;
  for (int64_t i = 0; i < U; ++i) {
    Entry& e = up->model[keys[i]];
    vals[p++] = e.w;
    if (!e.V.empty() && !(up->param.l1_shrk && (e.w == 0))) {
      memcpy(vals + p, e.V.data(), d * sizeof(real_t));
      p += d;
      lens[i] = d + 1;
    } else if (d != 0) {
      lens[i] = 1;
    }
  }
  return p;
}

// SGDUpdater::Update (sgd_updater.cc:60-102).  type 1 = kFeaCount, 3 = kGradient.
// Returns 0, or -1 on a CHECK failure (message in orc_last_error()).
int orc_updater_update(void* h, const uint64_t* keys, int64_t U, int type, const float* vals,
                       int64_t nvals, const int32_t* lens) {
  Updater* up = static_cast<Updater*>(h);
  int d = up->param.V_dim;
  if (type == 1) {
    if (nvals != U) { g_err = "kFeaCount: vals.size != keys.size"; return -1; }
    for (int64_t i = 0; i < U; ++i) {
      Entry& e = up->model[keys[i]];
      e.fea_cnt += vals[i];
      if (d > 0 && e.V.empty() && e.w != 0 && e.fea_cnt > up->param.V_threshold) up->InitV(&e);
    }
    return 0;
  } else if (type == 3) {
    bool w_only = lens == nullptr;
    if (w_only && nvals != U) { g_err = "kGradient: vals.size != keys.size"; return -1; }
    int64_t p = 0;
    for (int64_t i = 0; i < U; ++i) {
      Entry& e = up->model[keys[i]];
      up->UpdateW(vals[p++], &e);
      if (!w_only && lens[i] > 1) {
        if (lens[i] != d + 1) { g_err = "lens[i] != V_dim+1"; return -1; }
        if (e.V.empty()) { g_err = "gradient for a key without V"; return -1; }
        up->UpdateV(vals + p, &e);
        p += d;
      }
    }
    if (p != nvals) { g_err = "kGradient: values.size mismatch"; return -1; }
    return 0;
  }
  g_err = "UNKNOWN value_type";
  return -1;
}

// SGDUpdater::Evaluate (sgd_updater.cc:12-30): penalty and nnz.
double orc_updater_penalty(void* h, int64_t* nnz_out) {
  Updater* up = static_cast<Updater*>(h);
  double objv = 0;
  int64_t nnz = 0;
  int dim = up->param.V_dim;
  for (const auto& it : up->model) {
    const Entry& e = it.second;
    if (e.w) ++nnz;
    objv += up->param.l1 * std::fabs(e.w) + .5 * up->param.l2 * e.w * e.w;
    if (!e.V.empty()) {
      nnz += dim;
      for (int i = 0; i < dim; ++i) objv += .5 * up->param.l2 * e.V[i] * e.V[i];
    }
  }
  if (nnz_out) *nnz_out = nnz;
  return objv;
}

// Reads back one entry (test helper).  Returns 0 if absent, else 1 and fills
// state[4] = {w, sqrt_g, z, fea_cnt} and V/Vaux (2d floats) when present (has_v=1).
int orc_updater_entry(void* h, uint64_t key, float* state, float* V, int* has_v) {
  Updater* up = static_cast<Updater*>(h);
  auto it = up->model.find(key);
  if (it == up->model.end()) return 0;
  const Entry& e = it->second;
  state[0] = e.w; state[1] = e.sqrt_g; state[2] = e.z; state[3] = e.fea_cnt;
  *has_v = e.V.empty() ? 0 : 1;
  if (!e.V.empty() && V) memcpy(V, e.V.data(), e.V.size() * sizeof(float));
  return 1;
}

// SGDUpdater::Save (sgd_updater.h:84-106 + SGDEntry::SaveEntry :35-48).
int orc_updater_save(void* h, const char* path, int save_aux) {
  Updater* up = static_cast<Updater*>(h);
  FILE* f = fopen(path, "wb");
  if (!f) { g_err = "cannot open file"; return -1; }
  bool aux = save_aux != 0;
  fwrite(&aux, sizeof(bool), 1, f);
  for (const auto& it : up->model) {
    const Entry& e = it.second;
    if (e.empty()) continue;
    fwrite(&it.first, sizeof(feaid_t), 1, f);
    fwrite(&e.size, sizeof(int), 1, f);
    fwrite(&e.w, sizeof(real_t), 1, f);
    if (aux) { fwrite(&e.sqrt_g, sizeof(real_t), 1, f); fwrite(&e.z, sizeof(real_t), 1, f); }
    if (e.size == 1) continue;
    int n = e.size - 1;
    fwrite(e.V.data(), sizeof(real_t), n, f);
    if (aux) fwrite(e.V.data() + n, sizeof(real_t), n, f);
  }
  fclose(f);
  return 0;
}

// SGDUpdater::Dump (sgd_updater.h:108-139): one text line per non-empty entry, fields
// tab-separated, floats through an ostream's default formatting (as dmlc::ostream does)
int orc_updater_dump(void* h, const char* path, int dump_aux, int need_reverse) {
  Updater* up = static_cast<Updater*>(h);
  std::ofstream os(path);
  if (!os) { g_err = "cannot open file"; return -1; }
  for (const auto& it : up->model) {
    const Entry& e = it.second;
    if (e.empty()) continue;
    os << (need_reverse ? ReverseBytes(it.first) : it.first);
    os << '\t' << e.size << '\t' << e.w;
    if (dump_aux) os << '\t' << e.sqrt_g << '\t' << e.z;
    if (e.size > 1) {
      const int n = e.size - 1;
      for (int i = 0; i < n; ++i) os << '\t' << e.V[i];
      if (dump_aux)
        for (int i = n; i < 2 * n; ++i) os << '\t' << e.V[i];
    }
    os << '\n';
  }
  return os.good() ? 0 : -1;
}

// SGDUpdater::Load (sgd_updater.h:84-96 + SGDEntry::LoadEntry :50-68).
int orc_updater_load(void* h, const char* path) {
  Updater* up = static_cast<Updater*>(h);
  FILE* f = fopen(path, "rb");
  if (!f) { g_err = "cannot open file"; return -1; }
  bool aux;
  if (fread(&aux, sizeof(bool), 1, f) != 1) { fclose(f); return 0; }
  feaid_t key;
  while (fread(&key, sizeof(feaid_t), 1, f) == 1) {
    Entry& e = up->model[key];
    if (fread(&e.size, sizeof(int), 1, f) != 1 || fread(&e.w, sizeof(real_t), 1, f) != 1) {
      fclose(f); g_err = "truncated model file"; return -1;
    }
    if (aux && (fread(&e.sqrt_g, sizeof(real_t), 1, f) != 1 || fread(&e.z, sizeof(real_t), 1, f) != 1)) {
      fclose(f); g_err = "truncated model file"; return -1;
    }
    if (e.size == 1) continue;
    int n = e.size - 1;
    e.V.assign(2 * n, 0.f);
    if (fread(e.V.data(), sizeof(real_t), n, f) != (size_t)n) { fclose(f); g_err = "truncated"; return -1; }
    if (aux && fread(e.V.data() + n, sizeof(real_t), n, f) != (size_t)n) { fclose(f); g_err = "truncated"; return -1; }
  }
  up->new_w = up->model.size();
  fclose(f);
  return 0;
}

// ---------------------------------------------------------------------------------
// One local-mode minibatch, in the order of SGDLearner::IterateData
// (sgd_learner.cc:201-317) with the StoreLocal serialisation of SURVEY §3.1:
//   Localizer::Compact -> [Push(kFeaCount) if push_cnt] -> Pull(kWeight) -> GetPos ->
//   Predict -> Evaluate -> AUC -> CalcGrad -> Push(kGradient)      (training)
// train == 0 stops after AUC (validation / prediction jobs).
// out[0] = loss (Evaluate), out[1] = AUC*n, out[2] = nrows.  pred_out (nullable, B).
// ---------------------------------------------------------------------------------
int orc_train_step(void* h, int64_t B, const uint64_t* offs, const uint64_t* ids, const float* val,
                   const float* label, const float* rweight, uint64_t max_index, int push_cnt,
                   int train, double* out, float* pred_out) {
  Updater* up = static_cast<Updater*>(h);
  int d = up->param.V_dim;
  if (B <= 0) { out[0] = out[1] = out[2] = 0; return 0; }
  size_t nnz = offs[B];
  std::vector<uint64_t> uniq(nnz ? nnz : 1);
  std::vector<float> cnt(nnz ? nnz : 1);
  std::vector<uint32_t> col(nnz ? nnz : 1);
  int64_t U = orc_localize(B, offs, ids, max_index, uniq.data(), cnt.data(), col.data());
  if (push_cnt && d > 0) {
    if (orc_updater_update(h, uniq.data(), U, 1, cnt.data(), U, nullptr)) return -1;
  }
  std::vector<float> vals(U * (1 + d) + 1);
  std::vector<int32_t> lens(d > 0 ? U + 1 : 1), w_pos(U + 1), V_pos(U + 1);
  int64_t nv = orc_updater_get(h, uniq.data(), U, vals.data(), d > 0 ? lens.data() : nullptr);
  if (d > 0) orc_get_pos(U, lens.data(), w_pos.data(), V_pos.data());
  std::vector<float> pred(B, 0.f);
  orc_fm_predict(B, offs, col.data(), val, vals.data(), d > 0 ? w_pos.data() : nullptr,
                 d > 0 ? V_pos.data() : nullptr, d, pred.data());
  out[0] = orc_evaluate(B, label, pred.data());
  out[1] = orc_auc(B, label, pred.data());
  out[2] = (double)B;
  if (pred_out) memcpy(pred_out, pred.data(), B * sizeof(float));
  if (!train) return 0;
  std::vector<float> grad(nv, 0.f);
  if (up->param.sum64) {
    std::vector<double> g64(nv, 0.);
    CalcGrad<double>(B, offs, col.data(), val, label, rweight, vals.data(),
                     d > 0 ? w_pos.data() : nullptr, d > 0 ? V_pos.data() : nullptr, U, d,
                     pred.data(), g64.data());
    for (int64_t i = 0; i < nv; ++i) grad[i] = (float)g64[i];
  } else {
    orc_fm_calcgrad(B, offs, col.data(), val, label, rweight, vals.data(),
                    d > 0 ? w_pos.data() : nullptr, d > 0 ? V_pos.data() : nullptr, U, d,
                    pred.data(), grad.data());
  }
  return orc_updater_update(h, uniq.data(), U, 3, grad.data(), nv, d > 0 ? lens.data() : nullptr);
}

// glibc rand_r, exposed so tests can pin the device LCG restatement against it.
int orc_rand_r(unsigned* seed) { return rand_r(seed); }

}  // extern "C"
