// =====================================================================================
//  oracle/cpu_ref.cc — the reference's CPU hot path, restated WITH its threading, as the
//  CPU baseline that bench.py times on the GPU box's host cores.
//
//  TEST / MEASUREMENT INFRASTRUCTURE ONLY: only bench.py's `cpu_baseline` leg and tests/ load
//  it.  The arithmetic is oracle.cc's (the pinned restatement); what this file adds is the
//  reference's parallel structure, so that the baseline runs the way the reference runs:
//    * Localizer::Compact (localizer.cc:11-107): pairs built under `omp parallel for`,
//      ParallelSort (parallel_sort.h:14-39: recursive halves on std::threads down to a grain
//      of max(n / nthreads + 5, 16384), std::sort leaves, std::inplace_merge), a sequential
//      run-length pass and a sequential merge-join remap into a compacted RowBlock;
//    * SGDUpdater over std::unordered_map (sgd_updater.h:178), single-threaded like StoreLocal's
//      inline Push / Pull (store_local.h);
//    * FMLoss::Predict (fm_loss.h:67-119): SpMV::Times / SpMM::Times row-range split over the
//      OpenMP team (spmv.h:107-134, spmm.h:93-122, Range::Segment range.h:19-29), the VV and
//      final-sum loops under `omp parallel for`;
//    * Loss::Evaluate (loss.h:57-66, float reduction) and BinClassMetric::AUC
//      (bin_class_metric.h:35-57);
//    * FMLoss::CalcGrad (fm_loss.h:148-203): SpMV::TransTimes / SpMM::TransTimes column-range
//      split (every thread walks all rows, writes only its columns; spmv.h:139-171,
//      spmm.h:127-159);
//    * SGDLearner::IterateData (sgd_learner.cc:201-317): the reader thread localizes batch t+1
//      while the executor thread runs batch t (pull -> predict -> evaluate -> AUC -> calcgrad ->
//      push), at most two batches in flight (:310-312); blk_nthreads_ OpenMP threads in each.
//  Row- and column-range splits keep every sum in the sequential order, so predictions and
//  gradients are bitwise those of oracle.cc for any thread count (tests/test_oracle.py).
// =====================================================================================
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

typedef float real_t;
typedef uint64_t feaid_t;

namespace {

inline feaid_t ReverseBytes(feaid_t x) {  // include/difacto/base.h:39-51
  x = x << 32 | x >> 32;
  x = (x & 0x0000FFFF0000FFFFULL) << 16 | (x & 0xFFFF0000FFFF0000ULL) >> 16;
  x = (x & 0x00FF00FF00FF00FFULL) << 8 | (x & 0xFF00FF00FF00FF00ULL) >> 8;
  x = (x & 0x0F0F0F0F0F0F0F0FULL) << 4 | (x & 0xF0F0F0F0F0F0F0F0ULL) >> 4;
  return x;
}

// range.h:19-29
inline void Segment(size_t begin, size_t end, int idx, int nparts, size_t* b, size_t* e) {
  const double itv = static_cast<double>(end - begin) / nparts;
  *b = static_cast<size_t>(begin + itv * idx);
  *e = idx == nparts - 1 ? end : static_cast<size_t>(begin + itv * (idx + 1));
}

// parallel_sort.h:14-39
template <typename T, class Fn>
void ParallelSort_(T* data, size_t len, size_t grain, const Fn& cmp) {
  if (len <= grain) {
    std::sort(data, data + len, cmp);
  } else {
    std::thread thr(ParallelSort_<T, Fn>, data, len / 2, grain, cmp);
    ParallelSort_(data + len / 2, len - len / 2, grain, cmp);
    thr.join();
    std::inplace_merge(data, data + len / 2, data + len, cmp);
  }
}
template <typename T, class Fn>
void ParallelSort(std::vector<T>* arr, int nthreads, const Fn& cmp) {
  const size_t grain = std::max(arr->size() / nthreads + 5, (size_t)1024 * 16);
  ParallelSort_(arr->data(), arr->size(), grain, cmp);
}

struct Block {  // dmlc::RowBlock<unsigned> after Compact, + the batch's feature ids
  size_t size = 0;
  std::vector<uint64_t> offset;
  std::vector<unsigned> index;
  const float* value = nullptr;
  const float* label = nullptr;
  std::vector<feaid_t> uniq;
  std::vector<real_t> cnt;
};

// Localizer::Compact = CountUniqIndex (localizer.cc:11-49) + RemapIndex (:53-107)
void Compact(const uint64_t* offs, const uint64_t* ids, const float* val, const float* label,
             size_t B, int nt, bool want_cnt, Block* o) {
  struct Pair { feaid_t k; unsigned i; };
  const size_t n = offs[B];
  std::vector<Pair> pair(n);
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < n; ++i) {
    pair[i].k = ReverseBytes(ids[i] % ~0ull);
    pair[i].i = (unsigned)i;
  }
  ParallelSort(&pair, nt, [](const Pair& a, const Pair& b) { return a.k < b.k; });
  o->uniq.clear();
  o->cnt.clear();
  if (n) {
    feaid_t curr = pair[0].k;
    real_t c = 0;
    for (size_t i = 0; i < n; ++i) {
      if (pair[i].k != curr) {
        o->uniq.push_back(curr);
        if (want_cnt) o->cnt.push_back(c);
        curr = pair[i].k;
        c = 0;
      }
      ++c;
    }
    o->uniq.push_back(curr);
    if (want_cnt) o->cnt.push_back(c);
  }
  std::vector<unsigned> remapped(n, 0);
  size_t d = 0, p = 0;
  while (d < o->uniq.size() && p < n) {
    if (o->uniq[d] < pair[p].k) {
      ++d;
    } else {
      if (o->uniq[d] == pair[p].k) remapped[pair[p].i] = (unsigned)(d + 1);
      ++p;
    }
  }
  o->size = B;
  o->offset.assign(B + 1, 0);
  o->index.resize(n);
  size_t k = 0;
  for (size_t i = 0; i < B; ++i) {
    for (size_t j = offs[i]; j < offs[i + 1]; ++j) o->index[k++] = remapped[j] - 1;
    o->offset[i + 1] = k;
  }
  o->value = val;
  o->label = label;
}

struct Param {
  float l1 = 1, l2 = 0, V_l2 = .01f, lr = .01f, lr_beta = 1, V_lr = .01f, V_lr_beta = 1,
        V_init_scale = .01f;
  int V_dim = 0, V_threshold = 10;
  bool l1_shrk = true;
  unsigned seed = 0;
};

void ParseKW(const char* kwargs, Param* p) {
  if (!kwargs) return;
  std::string s(kwargs);
  for (char& c : s)
    if (c == ',') c = ' ';
  std::istringstream is(s);
  std::string tok;
  while (is >> tok) {
    auto eq = tok.find('=');
    if (eq == std::string::npos) continue;
    std::string k = tok.substr(0, eq);
    std::istringstream vs(tok.substr(eq + 1));
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
    else if (k == "seed") vs >> p->seed;
    else if (k == "l1_shrk") p->l1_shrk = tok.substr(eq + 1) != "0";
  }
}

// sgd_updater.h:20-69 / sgd_updater.cc:34-152 (arithmetic as oracle.cc)
struct Entry {
  real_t fea_cnt = 0, w = 0, sqrt_g = 0, z = 0;
  real_t* V = nullptr;  // [V(d) | Vaux(d)]
  ~Entry() { delete[] V; }
};

struct Updater {
  Param P;
  std::unordered_map<feaid_t, Entry> model;
  void InitV(Entry* e) {
    const int n = P.V_dim;
    e->V = new real_t[2 * n];
    for (int i = 0; i < n; ++i)
      e->V[i] = (rand_r(&P.seed) / (real_t)RAND_MAX - 0.5) * P.V_init_scale;
    std::memset(e->V + n, 0, n * sizeof(real_t));
  }
  void Get(const std::vector<feaid_t>& keys, std::vector<real_t>* vals, std::vector<int>* lens) {
    const int d = P.V_dim;
    vals->clear();
    lens->assign(keys.size(), 1);
    for (size_t i = 0; i < keys.size(); ++i) {
      Entry& e = model[keys[i]];
      vals->push_back(e.w);
      if (e.V && !(P.l1_shrk && e.w == 0)) {
        vals->insert(vals->end(), e.V, e.V + d);
        (*lens)[i] = d + 1;
      }
    }
  }
  void PushCnt(const std::vector<feaid_t>& keys, const std::vector<real_t>& cnt) {
    for (size_t i = 0; i < keys.size(); ++i) {
      Entry& e = model[keys[i]];
      e.fea_cnt += cnt[i];
      if (P.V_dim > 0 && !e.V && e.w != 0 && e.fea_cnt > P.V_threshold) InitV(&e);
    }
  }
  void PushGrad(const std::vector<feaid_t>& keys, const std::vector<real_t>& g,
                const std::vector<int>& lens) {
    const int d = P.V_dim;
    size_t p = 0;
    for (size_t i = 0; i < keys.size(); ++i) {
      Entry& e = model[keys[i]];
      real_t gw = g[p++];
      real_t sg = e.sqrt_g, w = e.w;
      gw += w * P.l2;
      e.sqrt_g = std::sqrt(sg * sg + gw * gw);
      e.z -= gw - (e.sqrt_g - sg) / P.lr * w;
      if (e.z <= P.l1 && e.z >= -P.l1) {
        e.w = 0;
      } else {
        real_t eta = (P.lr_beta + e.sqrt_g) / P.lr;
        e.w = (e.z > 0 ? e.z - P.l1 : e.z + P.l1) / eta;
      }
      if (w == 0 && e.w != 0 && d > 0 && !e.V && e.fea_cnt > P.V_threshold) InitV(&e);
      if (d > 0 && lens[i] > 1) {
        for (int l = 0; l < d; ++l) {
          real_t gv = g[p + l] + P.V_l2 * e.V[l];
          real_t cg = e.V[l + d];
          e.V[l + d] = std::sqrt(cg * cg + gv * gv);
          float eta = P.V_lr / (e.V[l + d] + P.V_lr_beta);
          e.V[l] -= eta * gv;
        }
        p += d;
      }
    }
  }
};

// SGDLearner::GetPos (sgd_learner.cc:151-165)
void GetPos(const std::vector<int>& len, std::vector<int>* wp, std::vector<int>* vp) {
  wp->resize(len.size());
  vp->resize(len.size());
  int p = 0;
  for (size_t i = 0; i < len.size(); ++i) {
    (*wp)[i] = len[i] == 0 ? -1 : p;
    (*vp)[i] = len[i] > 1 ? p + 1 : -1;
    p += len[i];
  }
}

// FMLoss::Predict (fm_loss.h:67-119) with the reference's thread partitioning
void Predict(const Block& D, const std::vector<real_t>& W, const std::vector<int>& wp,
             const std::vector<int>& vp, int d, int nt, std::vector<real_t>* pred,
             std::vector<real_t>* XV) {
  const size_t B = D.size;
  pred->assign(B, 0.f);
#pragma omp parallel num_threads(nt)
  {  // SpMV::Times, rows split (spmv.h:107-134)
    size_t b, e;
    Segment(0, B, omp_get_thread_num(), omp_get_num_threads(), &b, &e);
    for (size_t i = b; i < e; ++i)
      for (size_t j = D.offset[i]; j < D.offset[i + 1]; ++j) {
        const int q = d > 0 ? wp[D.index[j]] : (int)D.index[j];
        const real_t x = q < 0 ? 0.f : W[q];
        if (x == 0) continue;
        (*pred)[i] += D.value ? x * D.value[j] : x;
      }
  }
  if (d == 0) return;
  XV->assign(B * d, 0.f);
  std::vector<real_t> XXVV(B * d, 0.f), VV(W.size(), 0.f);
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < vp.size(); ++i) {
    const int p = vp[i];
    if (p < 0) continue;
    for (int l = 0; l < d; ++l) VV[p + l] = W[p + l] * W[p + l];
  }
#pragma omp parallel num_threads(nt)
  {  // SpMM::Times twice (X V and (X.*X)(V.*V)), rows split (spmm.h:93-122)
    size_t b, e;
    Segment(0, B, omp_get_thread_num(), omp_get_num_threads(), &b, &e);
    for (size_t i = b; i < e; ++i) {
      real_t* y = XV->data() + i * d;
      real_t* yy = XXVV.data() + i * d;
      for (size_t j = D.offset[i]; j < D.offset[i + 1]; ++j) {
        const int p = vp[D.index[j]];
        if (p < 0) continue;
        if (D.value) {
          const real_t v = D.value[j], xx = v * v;
          for (int l = 0; l < d; ++l) y[l] += W[p + l] * v;
          for (int l = 0; l < d; ++l) yy[l] += VV[p + l] * xx;
        } else {
          for (int l = 0; l < d; ++l) y[l] += W[p + l];
          for (int l = 0; l < d; ++l) yy[l] += VV[p + l];
        }
      }
    }
  }
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < B; ++i) {
    const real_t* t = XV->data() + i * d;
    const real_t* tt = XXVV.data() + i * d;
    real_t s = 0;
    for (int l = 0; l < d; ++l) s += t[l] * t[l] - tt[l];
    (*pred)[i] += .5 * s;
  }
  for (auto& p : *pred) p = p > 20 ? 20 : (p < -20 ? -20 : p);
}

// Loss::Evaluate (loss.h:57-66)
real_t Evaluate(const float* label, const std::vector<real_t>& pred, int nt) {
  real_t objv = 0;
#pragma omp parallel for reduction(+ : objv) num_threads(nt)
  for (size_t i = 0; i < pred.size(); ++i) {
    real_t y = label[i] > 0 ? 1 : -1;
    objv += log(1 + exp(-y * pred[i]));
  }
  return objv;
}

// BinClassMetric::AUC (bin_class_metric.h:35-57)
real_t AUC(const float* label, const std::vector<real_t>& pred, int nt) {
  struct E { real_t label, predict; };
  const size_t n = pred.size();
  std::vector<E> buf(n);
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < n; ++i) {
    buf[i].label = label[i];
    buf[i].predict = pred[i];
  }
  std::sort(buf.begin(), buf.end(), [](const E& a, const E& b) { return a.predict < b.predict; });
  real_t area = 0, cum_tp = 0;
  for (size_t i = 0; i < n; ++i) {
    if (buf[i].label > 0) cum_tp += 1; else area += cum_tp;
  }
  if (cum_tp == 0 || cum_tp == n) return 1;
  area /= cum_tp * (n - cum_tp);
  return (area < 0.5 ? 1 - area : area) * n;
}

// FMLoss::CalcGrad (fm_loss.h:148-203) with the reference's thread partitioning
void CalcGrad(const Block& D, const std::vector<real_t>& W, const std::vector<int>& wp,
              const std::vector<int>& vp, int d, int nt, const std::vector<real_t>& pred,
              std::vector<real_t>* XV, std::vector<real_t>* grad) {
  const size_t B = D.size, ncol = D.uniq.size();
  grad->assign(W.size(), 0.f);
  std::vector<real_t> p(B);
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < B; ++i) {
    real_t y = D.label[i] > 0 ? 1 : -1;
    p[i] = -y / (1 + std::exp(y * pred[i]));
  }
  std::vector<real_t> XXp(d > 0 ? ncol : 0, 0.f);
#pragma omp parallel num_threads(nt)
  {  // SpMV::TransTimes: X' p into grad (w) and (X.*X)' p into XXp, columns split
    size_t cb, ce;
    Segment(0, ncol, omp_get_thread_num(), omp_get_num_threads(), &cb, &ce);
    for (size_t i = 0; i < B; ++i) {
      const real_t pi = p[i];
      if (pi == 0) continue;
      for (size_t j = D.offset[i]; j < D.offset[i + 1]; ++j) {
        const unsigned k = D.index[j];
        if (k < cb || k >= ce) continue;
        const int q = d > 0 ? wp[k] : (int)k;
        if (q >= 0) (*grad)[q] += D.value ? pi * D.value[j] : pi;
      }
    }
    if (d > 0) {
      for (size_t i = 0; i < B; ++i) {
        const real_t pi = p[i];
        if (pi == 0) continue;
        for (size_t j = D.offset[i]; j < D.offset[i + 1]; ++j) {
          const unsigned k = D.index[j];
          if (k < cb || k >= ce) continue;
          XXp[k] += D.value ? pi * (D.value[j] * D.value[j]) : pi;
        }
      }
    }
  }
  if (d == 0) return;
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < ncol; ++i) {
    const int q = vp[i];
    if (q < 0) continue;
    for (int l = 0; l < d; ++l) (*grad)[q + l] -= W[q + l] * XXp[i];
  }
#pragma omp parallel for num_threads(nt)
  for (size_t i = 0; i < B; ++i) {
    real_t* t = XV->data() + i * d;
    for (int l = 0; l < d; ++l) t[l] *= p[i];
  }
#pragma omp parallel num_threads(nt)
  {  // SpMM::TransTimes, columns split (spmm.h:127-159)
    size_t cb, ce;
    Segment(0, ncol, omp_get_thread_num(), omp_get_num_threads(), &cb, &ce);
    for (size_t i = 0; i < B; ++i) {
      const real_t* x = XV->data() + i * d;
      for (size_t j = D.offset[i]; j < D.offset[i + 1]; ++j) {
        const unsigned k = D.index[j];
        if (k < cb || k >= ce) continue;
        const int q = vp[k];
        if (q < 0) continue;
        real_t* y = grad->data() + q;
        if (D.value) {
          const real_t v = D.value[j];
          for (int l = 0; l < d; ++l) y[l] += x[l] * v;
        } else {
          for (int l = 0; l < d; ++l) y[l] += x[l];
        }
      }
    }
  }
}

struct Result { double loss = 0, auc = 0, nrows = 0; };

// wall seconds per phase (executor thread + Localizer), summed over calls
double g_phase[6];  // localize, get, predict, evaluate+auc, calcgrad, update
inline double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// the executor body (sgd_learner.cc:204-267) with StoreLocal's inline pull / push
void Execute(Updater* up, const Block& D, int nt, bool train, Result* res,
             float* pred_out) {
  const int d = up->P.V_dim;
  std::vector<real_t> vals, pred, XV, grad;
  std::vector<int> lens, wp, vp;
  double t = Now(), t1;
  up->Get(D.uniq, &vals, &lens);
  if (d > 0) GetPos(lens, &wp, &vp);
  t1 = Now(); g_phase[1] += t1 - t; t = t1;
  Predict(D, vals, wp, vp, d, nt, &pred, &XV);
  t1 = Now(); g_phase[2] += t1 - t; t = t1;
  res->nrows += D.size;
  res->loss += Evaluate(D.label, pred, nt);
  res->auc += AUC(D.label, pred, nt);
  t1 = Now(); g_phase[3] += t1 - t; t = t1;
  if (pred_out) std::memcpy(pred_out, pred.data(), pred.size() * sizeof(real_t));
  if (!train) return;
  CalcGrad(D, vals, wp, vp, d, nt, pred, &XV, &grad);
  t1 = Now(); g_phase[4] += t1 - t; t = t1;
  up->PushGrad(D.uniq, grad, lens);
  g_phase[5] += Now() - t;
}

}  // namespace

extern "C" {

void* cref_create(const char* kwargs) {
  Updater* u = new Updater();
  ParseKW(kwargs, &u->P);
  return u;
}
void cref_destroy(void* h) { delete static_cast<Updater*>(h); }
int64_t cref_size(void* h) { return (int64_t)static_cast<Updater*>(h)->model.size(); }
unsigned cref_seed(void* h) { return static_cast<Updater*>(h)->P.seed; }

// One local-mode step on the calling thread (Compact, [count push], execute).  out[3] =
// {loss, AUC*n, nrows}; pred_out optional.
void cref_step(void* h, int nt, int64_t B, const uint64_t* offs, const uint64_t* ids,
               const float* val, const float* label, int push_cnt, int train, double* out,
               float* pred_out) {
  Updater* up = static_cast<Updater*>(h);
  Block D;
  const bool cnt = push_cnt && up->P.V_dim > 0;
  const double tc = Now();
  Compact(offs, ids, val, label, (size_t)B, nt, cnt, &D);
  g_phase[0] += Now() - tc;
  if (cnt) up->PushCnt(D.uniq, D.cnt);
  Result r;
  Execute(up, D, nt, train != 0, &r, pred_out);
  out[0] = r.loss;
  out[1] = r.auc;
  out[2] = r.nrows;
}

// SGDLearner::IterateData over nb batches (epoch >= 1: no count push): the calling thread
// localizes (the reader loop), an executor thread runs the batches in order, at most two in
// flight.  Returns the wall seconds; out[3] = {loss, AUC*n, nrows}.
double cref_iterate(void* h, int nt, int nb, const int64_t* B, const uint64_t* const* offs,
                    const uint64_t* const* ids, const float* const* val,
                    const float* const* label, double* out) {
  Updater* up = static_cast<Updater*>(h);
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Block*> q;
  int remains = 0;  // issued and not finished (AsyncLocalTracker::NumRemains)
  bool done = false;
  Result res;
  const auto t0 = std::chrono::steady_clock::now();
  std::thread exec([&]() {
    for (;;) {
      Block* b;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&]() { return done || !q.empty(); });
        if (q.empty()) return;
        b = q.front();
        q.pop_front();
      }
      Execute(up, *b, nt, true, &res, nullptr);
      delete b;
      {
        std::lock_guard<std::mutex> lk(mu);
        --remains;
      }
      cv.notify_all();
    }
  });
  for (int i = 0; i < nb; ++i) {
    Block* b = new Block();
    const double tc = Now();
    Compact(offs[i], ids[i], val ? val[i] : nullptr, label[i], (size_t)B[i], nt, false, b);
    g_phase[0] += Now() - tc;
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&]() { return remains <= 1; });  // sgd_learner.cc:310-312
    q.push_back(b);
    ++remains;
    cv.notify_all();
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&]() { return remains == 0; });
    done = true;
  }
  cv.notify_all();
  exec.join();
  const double dt =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  out[0] = res.loss;
  out[1] = res.auc;
  out[2] = res.nrows;
  return dt;
}

int cref_max_threads() { return omp_get_num_procs(); }

// seconds per phase since the last call: localize, get, predict, evaluate+AUC, calcgrad,
// update (then reset)
void cref_phases(double* out) {
  for (int i = 0; i < 6; ++i) {
    out[i] = g_phase[i];
    g_phase[i] = 0;
  }
}

}  // extern "C"
