// dist_store.cc — see dist_store.h.  Host code against the C-ABI and the ShardExchange
// interface (no HIP headers).
#include "dist_store.h"

#include <condition_variable>
#include <mutex>

#include "gpu_adapters.h"

namespace difacto {

namespace {

enum Op { kOpCount = 1, kOpPull = 2, kOpGrad = 3, kOpBarrier = 4 };

// one worker's call of a round
struct Req {
  int op = 0;
  const SArray<feaid_t>* keys = nullptr;
  const SArray<real_t>* vals = nullptr;
  const SArray<int>* lens = nullptr;
  SArray<real_t>* out_vals = nullptr;
  SArray<int>* out_lens = nullptr;
};

std::string CtxKw(const KWArgs& kw) {
  std::string s;
  for (const auto& p : kw) {
    if (!s.empty()) s += ",";
    s += p.first + "=" + p.second;
  }
  return s;
}

std::vector<int64_t> Offsets(const std::vector<int64_t>& rows) {
  std::vector<int64_t> o(rows.size() + 1, 0);
  for (size_t i = 0; i < rows.size(); ++i) o[i + 1] = o[i] + rows[i];
  return o;
}

// the server of a key: floor(key * N / 2^64), as the device phases split (dist.hip owner_of)
inline int OwnerOf(feaid_t k, int n) {
  return (int)(((unsigned __int128)k * (unsigned)n) >> 64);
}

}  // namespace

struct GpuDistStore::Core {
  std::vector<dfx_ctx*> ctxs;  // owned
  std::unique_ptr<ShardExchange> ex;
  int N = 0, L = 0, S = 0, d = 0;
  bool agg_sum = false;
  std::vector<std::unique_ptr<Store>> workers;

  // the round's rendezvous: the last of the L workers to call runs the round for all
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<Req> reqs;

  struct Bufs {
    explicit Bufs(dfx_ctx* c)
        : keys(c), rkeys(c), cnt(c), rcnt(c), recs(c), rrecs(c), icnt(c), iall(c) {}
    DevArray<uint64_t> keys, rkeys;
    DevArray<float> cnt, rcnt, recs, rrecs;
    DevArray<int64_t> icnt, iall;
  };
  std::vector<std::unique_ptr<Bufs>> bufs;
  std::vector<float> host;

  void Setup();
  ~Core() {
    workers.clear();
    for (dfx_ctx* c : ctxs) (void)dfx_sync(c);
    ex.reset();
    for (dfx_ctx* c : ctxs) (void)dfx_ctx_destroy(c);
  }

  void Round(int l, const Req& r) {
    std::unique_lock<std::mutex> lk(mu);
    reqs[l] = r;
    const uint64_t g = gen;
    if (++arrived < L) {
      cv.wait(lk, [&]() { return gen != g; });
      return;
    }
    arrived = 0;
    lk.unlock();  // the other workers wait for gen to move
    Exec();
    lk.lock();
    ++gen;
    cv.notify_all();
  }

  void Sync() {
    for (dfx_ctx* c : ctxs) DfxCheck(dfx_sync(c), "dfx_sync");
  }

  // push_agg=sum: every owner's InitV request count, all-gathered, then the draws ranked over
  // all owners (after a count push and after every gradient push; dist_host.cc InitV)
  void InitV() {
    if (!agg_sum || d <= 0) return;
    std::vector<const void*> snd(L);
    std::vector<void*> rcv(L);
    for (int l = 0; l < L; ++l) {
      Bufs& b = *bufs[l];
      DfxCheck(dfx_dist_initv_local(ctxs[l], 0, b.icnt.get()), "dfx_dist_initv_local");
      snd[l] = b.icnt.get();
      rcv[l] = b.iall.get();
    }
    ex->Wait(ex->Gather(snd, rcv, 8));
    for (int l = 0; l < L; ++l)
      DfxCheck(dfx_dist_initv_draw(ctxs[l], 0, bufs[l]->iall.get(), ex->rank(l), N),
               "dfx_dist_initv_draw");
  }

  void Exec();
};

void GpuDistStore::Core::Setup() {
  L = ex->nlocal();
  N = ex->nranks();
  S = dfx_dist_record_floats(ctxs[0]);
  d = dfx_ctx_vdim(ctxs[0]);
  agg_sum = dfx_dist_push_agg_sum(ctxs[0]) == 1;
  reqs.resize(L);
  for (int l = 0; l < L; ++l) {
    bufs.emplace_back(new Bufs(ctxs[l]));
    bufs.back()->icnt.ensure(1);
    bufs.back()->iall.ensure(N);
  }
}

void GpuDistStore::Core::Exec() {
  const int op = reqs[0].op;
  for (int l = 1; l < L; ++l)
    DFX_HOST_CHECK(reqs[l].op == op, "GpuDistStore: the workers' calls of a round differ");
  if (op == kOpBarrier) {
    std::vector<double> one(1, 1.0);
    ex->AllReduceSum(&one);
    return;
  }
  // split every worker's keys by owner (sorted keys: contiguous runs, kvstore_dist.h:101,111)
  std::vector<std::vector<int64_t>> send(L, std::vector<int64_t>(N, 0)), recv;
  std::vector<int64_t> U(L), R(L);
  std::vector<const void*> ks(L), cs(L), ps(L);
  std::vector<void*> kr(L), cr(L), pr(L);
  for (int l = 0; l < L; ++l) {
    const SArray<feaid_t>& k = *reqs[l].keys;
    U[l] = (int64_t)k.size();
    for (size_t i = 0; i < k.size(); ++i) {
      DFX_HOST_CHECK(i == 0 || k[i - 1] <= k[i], "fea_ids must in non-decreasing order");
      ++send[l][OwnerOf(k[i], N)];
    }
    Bufs& b = *bufs[l];
    b.keys.ensure(U[l]);
    if (U[l]) DfxCheck(dfx_memcpy(ctxs[l], b.keys.get(), k.data(), U[l] * 8, 0), "upload keys");
    ks[l] = b.keys.get();
    if (op == kOpCount) {
      const SArray<real_t>& c = *reqs[l].vals;
      DFX_HOST_CHECK((int64_t)c.size() == U[l], "kFeaCount: one count per key");
      b.cnt.ensure(U[l]);
      if (U[l]) DfxCheck(dfx_memcpy(ctxs[l], b.cnt.get(), c.data(), U[l] * 4, 0), "upload counts");
      cs[l] = b.cnt.get();
    }
  }
  ex->ExchangeCounts(send, &recv);
  for (int l = 0; l < L; ++l) {
    R[l] = Offsets(recv[l]).back();
    Bufs& b = *bufs[l];
    b.rkeys.ensure(R[l]);
    kr[l] = b.rkeys.get();
    if (op == kOpCount) {
      b.rcnt.ensure(R[l]);
      cr[l] = b.rcnt.get();
    }
  }
  const int hk = ex->Start(0, ks, send, kr, recv, 8, true);
  const int hc = op == kOpCount ? ex->Start(0, cs, send, cr, recv, 4, true) : -1;
  ex->Wait(hk);
  if (hc >= 0) ex->Wait(hc);
  // every call begins its own owner step: table slots may move at a sync point in between
  for (int l = 0; l < L; ++l) {
    const std::vector<int64_t> offs = Offsets(recv[l]);
    DfxCheck(dfx_dist_owner_begin(ctxs[l], 0, bufs[l]->rkeys.get(), offs.data(), N,
                                  op == kOpCount ? bufs[l]->rcnt.get() : nullptr),
             "dfx_dist_owner_begin");
  }
  if (op == kOpCount) {
    InitV();
    Sync();
    return;
  }
  if (op == kOpPull) {
    for (int l = 0; l < L; ++l) {
      Bufs& b = *bufs[l];
      b.recs.ensure((size_t)R[l] * S);
      DfxCheck(dfx_dist_owner_pull(ctxs[l], 0, b.recs.get()), "dfx_dist_owner_pull");
      ps[l] = b.recs.get();
      b.rrecs.ensure((size_t)U[l] * S);
      pr[l] = b.rrecs.get();
    }
    ex->Wait(ex->Start(1, ps, recv, pr, send, (size_t)S * 4, true));
    // records [V(d) | w | live | 0 0] -> Get layout (sgd_updater.cc:34-58): w, then V when live
    for (int l = 0; l < L; ++l) {
      const Req& q = reqs[l];
      host.resize((size_t)U[l] * S);
      bufs[l]->rrecs.download(host.data(), host.size());
      std::vector<real_t> vals;
      vals.reserve((size_t)U[l] * (1 + d));
      std::vector<int> lens;
      for (int64_t i = 0; i < U[l]; ++i) {
        const float* r = host.data() + i * S;
        vals.push_back(r[d]);
        if (d > 0) {
          const bool live = r[d + 1] != 0.f;
          if (live) vals.insert(vals.end(), r, r + d);
          lens.push_back(live ? d + 1 : 1);
        }
      }
      q.out_vals->CopyFrom(vals.data(), vals.size());
      if (q.out_lens) {
        if (d > 0) {
          q.out_lens->CopyFrom(lens.data(), lens.size());
        } else {
          q.out_lens->clear();
        }
      }
    }
    Sync();
    return;
  }
  // kGradient: Get-layout gradients (the lens of the pull) -> records [gV | gw | live | 0 0]
  for (int l = 0; l < L; ++l) {
    const Req& q = reqs[l];
    const SArray<real_t>& g = *q.vals;
    const SArray<int>& lens = *q.lens;
    DFX_HOST_CHECK(d == 0 || (int64_t)lens.size() == U[l], "kGradient: one length per key");
    host.assign((size_t)U[l] * S, 0.f);
    size_t p = 0;
    for (int64_t i = 0; i < U[l]; ++i) {
      const int len = d > 0 ? lens[i] : 1;
      DFX_HOST_CHECK(len == 1 || len == d + 1, "kGradient: lengths must be 1 or 1 + V_dim");
      DFX_HOST_CHECK(p + len <= g.size(), "kGradient: fewer values than the lengths say");
      float* r = host.data() + i * S;
      r[d] = g[p];
      if (len > 1) {
        std::memcpy(r, g.data() + p + 1, d * sizeof(float));
        r[d + 1] = 1.f;
      }
      p += len;
    }
    DFX_HOST_CHECK(p == g.size(), "kGradient: more values than the lengths say");
    Bufs& b = *bufs[l];
    b.recs.ensure(host.size());
    if (!host.empty())
      DfxCheck(dfx_memcpy(ctxs[l], b.recs.get(), host.data(), host.size() * 4, 0), "upload grads");
    // the host staging is reused by the next worker: let the copy finish first
    DfxCheck(dfx_sync(ctxs[l]), "dfx_sync");
    ps[l] = b.recs.get();
    b.rrecs.ensure((size_t)R[l] * S);
    pr[l] = b.rrecs.get();
  }
  ex->Wait(ex->Start(1, ps, send, pr, recv, (size_t)S * 4, true));
  for (int l = 0; l < L; ++l)
    DfxCheck(dfx_dist_owner_push(ctxs[l], 0, bufs[l]->rrecs.get()), "dfx_dist_owner_push");
  InitV();
  Sync();
}

namespace {

class DistWorker : public Store {
 public:
  DistWorker(GpuDistStore::Core* core, int local) : core_(core), l_(local) {}
  KWArgs Init(const KWArgs& kwargs) override { return kwargs; }
  int Push(const SArray<feaid_t>& fea_ids, int val_type, const SArray<real_t>& vals,
           const SArray<int>& lens, const std::function<void()>& on_complete) override {
    DFX_HOST_CHECK(val_type == kFeaCount || val_type == kGradient,
                   "GpuDistStore::Push: kFeaCount or kGradient");
    Req r;
    r.op = val_type == kFeaCount ? kOpCount : kOpGrad;
    r.keys = &fea_ids;
    r.vals = &vals;
    r.lens = &lens;
    core_->Round(l_, r);
    if (on_complete) on_complete();
    return time_++;
  }
  int Pull(const SArray<feaid_t>& fea_ids, int val_type, SArray<real_t>* vals, SArray<int>* lens,
           const std::function<void()>& on_complete) override {
    DFX_HOST_CHECK(val_type == kWeight, "GpuDistStore::Pull: kWeight");
    DFX_HOST_CHECK(vals != nullptr, "GpuDistStore::Pull: null vals");
    Req r;
    r.op = kOpPull;
    r.keys = &fea_ids;
    r.out_vals = vals;
    r.out_lens = lens;
    core_->Round(l_, r);
    if (on_complete) on_complete();
    return time_++;
  }
  void Wait(int) override {}  // every call completed before it returned
  int NumWorkers() override { return core_->N; }
  int NumServers() override { return core_->N; }
  int Rank() override { return core_->ex->rank(l_); }
  // the servers' updaters are the shard contexts (built from the store's kwargs)
  void SetUpdater(const std::shared_ptr<Updater>& updater) override { updater_ = updater; }
  void Barrier() override {
    Req r;
    r.op = kOpBarrier;
    core_->Round(l_, r);
  }

 private:
  GpuDistStore::Core* core_;
  int l_;
  int time_ = 0;
};

// Store::Create's product under a distributed launch: worker 0 of a GpuDistStore it owns
class OwningWorker : public Store {
 public:
  explicit OwningWorker(std::shared_ptr<GpuDistStore> ds) : ds_(ds), w_(ds->worker(0)) {}
  KWArgs Init(const KWArgs& kwargs) override { return w_->Init(kwargs); }
  int Push(const SArray<feaid_t>& fea_ids, int val_type, const SArray<real_t>& vals,
           const SArray<int>& lens, const std::function<void()>& on_complete) override {
    return w_->Push(fea_ids, val_type, vals, lens, on_complete);
  }
  int Pull(const SArray<feaid_t>& fea_ids, int val_type, SArray<real_t>* vals, SArray<int>* lens,
           const std::function<void()>& on_complete) override {
    return w_->Pull(fea_ids, val_type, vals, lens, on_complete);
  }
  void Wait(int t) override { w_->Wait(t); }
  int NumWorkers() override { return w_->NumWorkers(); }
  int NumServers() override { return w_->NumServers(); }
  int Rank() override { return w_->Rank(); }
  void SetUpdater(const std::shared_ptr<Updater>& updater) override { w_->SetUpdater(updater); }
  void Barrier() override { w_->Barrier(); }

 private:
  std::shared_ptr<GpuDistStore> ds_;
  Store* w_;
};

}  // namespace

GpuDistStore::GpuDistStore(std::unique_ptr<Core> core) : core_(std::move(core)) {
  core_->Setup();
  for (int l = 0; l < core_->L; ++l) core_->workers.emplace_back(new DistWorker(core_.get(), l));
}

GpuDistStore::~GpuDistStore() {}

std::shared_ptr<GpuDistStore> GpuDistStore::CreateLoopback(int nshards, const KWArgs& kwargs) {
  DFX_HOST_CHECK(nshards >= 1, "GpuDistStore: nshards >= 1");
  std::unique_ptr<Core> c(new Core());
  const std::string kw = CtxKw(kwargs);
  c->ctxs.assign(nshards, nullptr);
  for (auto& h : c->ctxs) DfxCheck(dfx_ctx_create(0, kw.c_str(), &h), "dfx_ctx_create");
  c->ex = MakeLoopbackExchange(c->ctxs);
  return std::shared_ptr<GpuDistStore>(new GpuDistStore(std::move(c)));
}

std::shared_ptr<GpuDistStore> GpuDistStore::CreateRccl(const KWArgs& kwargs) {
  const char* ws = std::getenv("WORLD_SIZE");
  const int world = ws ? std::atoi(ws) : 1;
  const int rank = std::getenv("RANK") ? std::atoi(std::getenv("RANK")) : 0;
  const int local = std::getenv("LOCAL_RANK") ? std::atoi(std::getenv("LOCAL_RANK")) : 0;
  std::string id_file;
  if (const char* f = std::getenv("DFX_COMM_ID_FILE")) {
    id_file = f;
  } else {
    const char* port = std::getenv("MASTER_PORT");
    id_file = std::string("/tmp/dfx_comm_") + (port ? port : "0");
  }
  std::unique_ptr<Core> c(new Core());
  c->ctxs.assign(1, nullptr);
  DfxCheck(dfx_ctx_create(local, CtxKw(kwargs).c_str(), &c->ctxs[0]), "dfx_ctx_create");
  c->ex = MakeRcclExchange(c->ctxs[0], rank, world, id_file);
  return std::shared_ptr<GpuDistStore>(new GpuDistStore(std::move(c)));
}

int GpuDistStore::nlocal() const { return core_->L; }
Store* GpuDistStore::worker(int local) const { return core_->workers.at(local).get(); }
dfx_ctx* GpuDistStore::shard(int local) const { return core_->ctxs.at(local); }
ShardExchange* GpuDistStore::exchange() const { return core_->ex.get(); }

std::shared_ptr<Store> CreateStore(const KWArgs& kwargs) {
  const char* ws = std::getenv("WORLD_SIZE");
  if (ws && std::atoi(ws) > 1)
    return std::make_shared<OwningWorker>(GpuDistStore::CreateRccl(kwargs));
  return std::make_shared<StoreGPU>();
}

}  // namespace difacto
