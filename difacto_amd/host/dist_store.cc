// dist_store.cc — see dist_store.h.  Host code against the C-ABI and the ShardExchange
// interface (no HIP headers).
#include "dist_store.h"

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <set>
#include <thread>

#include "gpu_adapters.h"

namespace difacto {

namespace {

enum Op { kOpNone = 0, kOpCount = 1, kOpPull = 2, kOpGrad = 3, kOpBarrier = 4, kOpReduce = 5 };
constexpr int kFlagStop = 6, kFlags = 7;  // per rank: its head ops (one-hot) and "stopping"

// one request of a worker, queued until a round serves it.  The SArrays are shared handles:
// the request keeps the caller's buffers alive (ps-lite's KVWorker holds them the same way)
struct Req {
  int op = kOpNone;
  int ts = -1;
  bool from_cb = false;  // issued by a callback of its worker
  SArray<feaid_t> keys;
  SArray<real_t> vals;
  SArray<int> lens;
  SArray<real_t>* out_vals = nullptr;
  SArray<int>* out_lens = nullptr;
  std::vector<double>* red = nullptr;  // kOpReduce: the process's values (one local worker's)
  std::function<void()> cb;
};

std::string CtxKw(const KWArgs& kw) {
  std::string s;
  for (const auto& p : kw) {
    if (!s.empty()) s += ",";
    s += p.first + "=" + p.second;
  }
  return s;
}

// kwarg store_sync=lockstep|async (GpuDistStore::Core::lockstep)
bool LockstepOf(const KWArgs& kw) {
  for (const auto& p : kw) {
    if (p.first != "store_sync") continue;
    DFX_HOST_CHECK(p.second == "lockstep" || p.second == "async",
                   "store_sync must be lockstep or async");
    return p.second == "lockstep";
  }
  return true;
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

// the worker whose callback the current thread is running (requests it issues are that
// worker's next ones: they go to the front of its queue, see Core::Enqueue)
thread_local int t_in_callback_of = -1;

}  // namespace

// KVStoreDist's request flow (kvstore_dist.h:90-175) for GPU shards: Push / Pull enqueue a
// request and return a timestamp; ONE progress thread per process serves the queues in
// rounds, all processes together, and runs each request's callback when it is done (ps-lite
// runs them on its receiving thread the same way).  So the reference's IterateData drives it
// unchanged: the reader thread's Push(kFeaCount) of batch k+1 and the executor's Pull /
// Push(kGradient) of batch k may overlap, and workers may hold different numbers of batches.
//
// A round: every process reports which kinds each local worker can have served (a host
// all-reduce — RCCL, or nothing at loopback); every process then serves the same ONE kind, the
// first servable of gradient push, pull, count push, barrier — lockstep (store_sync=lockstep,
// the default): when every worker has one; async: for the workers that have one at their head —
// as one exchange among all shards, in which the workers without a request send no keys.
// Order within a worker: FIFO, except that requests issued from a callback of its own go first
// (the pull's callback pushes the gradient: served before a count push of the next batch that
// the reader queued meanwhile), and in lockstep a pull or gradient push may overtake count
// pushes (the reader's look-ahead) — the sequential order count(k), pull(k), grad(k),
// count(k+1), ...  A barrier is served when it heads every worker's queue.
struct GpuDistStore::Core {
  std::vector<dfx_ctx*> ctxs;  // owned
  std::unique_ptr<ShardExchange> ex;
  int N = 0, L = 0, S = 0, d = 0;
  bool agg_sum = false;
  std::vector<std::unique_ptr<Store>> workers;

  std::mutex mu;
  std::condition_variable cv_done;
  std::vector<std::deque<Req>> q;      // per local worker
  std::vector<int> next_ts;            // per local worker
  std::vector<std::set<int>> done;     // completed timestamps >= done_low
  std::vector<int> done_low;           // every timestamp below it is complete
  bool stopping = false;
  // store_sync=lockstep (default): a sub-round of a kind runs when every worker has a request
  // of that kind (the synchronous step of push_agg=sum: every worker issues the same calls, an
  // idle worker empty ones); async: each worker's head request is served as it comes, as
  // ps-lite's server handles pushes in arrival order (workers may hold different numbers of
  // batches; which requests share a round depends on timing)
  bool lockstep = true;
  std::thread progress;
  std::string failure;                 // a round failed: every later call reports it

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
  void Stop() {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (!progress.joinable()) return;
      stopping = true;
    }
    progress.join();
  }
  ~Core() {
    Stop();
    workers.clear();
    for (dfx_ctx* c : ctxs) (void)dfx_sync(c);
    ex.reset();
    for (dfx_ctx* c : ctxs) (void)dfx_ctx_destroy(c);
  }

  int Enqueue(int l, Req r) {
    std::lock_guard<std::mutex> lk(mu);
    DFX_HOST_CHECK(failure.empty(), "GpuDistStore: " + failure);
    DFX_HOST_CHECK(!stopping, "GpuDistStore: a request after the store began to stop");
    r.ts = next_ts[l]++;
    const int ts = r.ts;
    if (t_in_callback_of == l) {
      // issued by a callback of this worker: ahead of what was queued meanwhile, after any
      // request the same callback issued before it
      r.from_cb = true;
      size_t pos = 0;
      while (pos < q[l].size() && q[l][pos].from_cb && q[l][pos].ts >= cb_first_ts_) ++pos;
      q[l].insert(q[l].begin() + pos, std::move(r));
    } else {
      q[l].push_back(std::move(r));
    }
    return ts;
  }
  int cb_first_ts_ = 1 << 30;  // requests of the running callback have ts >= this

  bool IsDone(int l, int ts) {
    return ts < done_low[l] || done[l].count(ts) != 0;
  }
  void MarkDone(int l, int ts) {
    done[l].insert(ts);
    while (done[l].count(done_low[l])) done[l].erase(done_low[l]++);
  }
  void Wait(int l, int ts) {
    std::unique_lock<std::mutex> lk(mu);
    // a callback runs on the progress thread, the only thread that completes requests: waiting
    // there for an unfinished one would hang
    DFX_HOST_CHECK(t_in_callback_of < 0 || IsDone(l, ts),
                   "GpuDistStore: Wait on an unfinished request from a request callback");
    cv_done.wait(lk, [&]() { return IsDone(l, ts) || !failure.empty(); });
    DFX_HOST_CHECK(failure.empty(), "GpuDistStore: " + failure);
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

  void Loop();
  // one sub-round of kind op among all shards: reqs[l] is local worker l's request, or null
  // (it takes part with no keys)
  void Exec(int op, const std::vector<Req*>& reqs);
};

void GpuDistStore::Core::Setup() {
  L = ex->nlocal();
  N = ex->nranks();
  S = dfx_dist_record_floats(ctxs[0]);
  d = dfx_ctx_vdim(ctxs[0]);
  agg_sum = dfx_dist_push_agg_sum(ctxs[0]) == 1;
  q.resize(L);
  next_ts.assign(L, 0);
  done.resize(L);
  done_low.assign(L, 0);
  for (int l = 0; l < L; ++l) {
    bufs.emplace_back(new Bufs(ctxs[l]));
    bufs.back()->icnt.ensure(1);
    bufs.back()->iall.ensure(N);
  }
  progress = std::thread([this]() { Loop(); });
}

void GpuDistStore::Core::Loop() {
  int idle_us = 0;
  // the request of kind op worker l can have served now, or -1.  Its queue is FIFO, except
  // that (lockstep) a pull or a gradient push may overtake count pushes queued ahead of it: a
  // count push is the reader thread's look-ahead to the next batch (IterateData issues it
  // while the executor still works on the previous batch), so the others run first
  auto find = [&](int l, int op) -> int {
    if (q[l].empty()) return -1;
    if (!lockstep || op == kOpCount || op == kOpBarrier || op == kOpReduce)
      return q[l].front().op == op ? 0 : -1;
    for (size_t i = 0; i < q[l].size(); ++i)
      if (q[l][i].op != kOpCount) return q[l][i].op == op ? (int)i : -1;
    return -1;
  };
  while (true) {
    // what every rank can serve this round, by a host all-reduce
    std::vector<double> flags((size_t)N * kFlags, 0.0);
    {
      std::lock_guard<std::mutex> lk(mu);
      for (int l = 0; l < L; ++l) {
        const size_t r = (size_t)ex->rank(l);
        for (int o : {kOpCount, kOpPull, kOpGrad, kOpBarrier, kOpReduce})
          if (find(l, o) >= 0) flags[r * kFlags + o] = 1.0;
        if (stopping) flags[r * kFlags + kFlagStop] = 1.0;
      }
    }
    try {
      ex->AllReduceSum(&flags);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu);
      failure = e.what();
      cv_done.notify_all();
      return;
    }
    int nop[kFlags] = {0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < N; ++r)
      for (int o = 1; o < kFlags; ++o) nop[o] += flags[(size_t)r * kFlags + o] != 0 ? 1 : 0;
    // one kind per round, the first servable of gradient push, pull, count push, barrier,
    // reduce: lockstep, when every worker has one; async, for whoever has one at its head.  A
    // barrier or a reduce needs everyone
    int kind = kOpNone;
    for (int o : {kOpGrad, kOpPull, kOpCount, kOpBarrier, kOpReduce}) {
      if (lockstep || o == kOpBarrier || o == kOpReduce ? nop[o] == N : nop[o] > 0) {
        kind = o;
        break;
      }
    }
    const bool work = kind != kOpNone;
    if (!work) {
      const bool pending = nop[kOpCount] || nop[kOpPull] || nop[kOpGrad] || nop[kOpBarrier] ||
                           nop[kOpReduce];
      if (nop[kFlagStop] == N) {
        // every process is stopping: the store is done.  Requests still queued can never be
        // served (lockstep: a worker issued calls the others did not)
        if (pending) {
          std::lock_guard<std::mutex> lk(mu);
          failure = "requests left at shutdown: in lockstep (store_sync=lockstep) every worker "
                    "must issue the same sequence of calls";
          cv_done.notify_all();
        }
        return;
      }
      idle_us = idle_us == 0 ? 20 : std::min(idle_us * 2, 1000);
      std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
      continue;
    }
    idle_us = 0;
    {
      const int op = kind;
      std::vector<Req> served(L);
      std::vector<Req*> reqs(L, nullptr);
      {
        std::lock_guard<std::mutex> lk(mu);
        for (int l = 0; l < L; ++l) {
          // what was reported at the start of the round is still there: only this thread
          // takes requests, and a callback of this thread adds them at the front
          const int i = find(l, op);
          if (i >= 0) {
            served[l] = std::move(q[l][i]);
            q[l].erase(q[l].begin() + i);
            reqs[l] = &served[l];
          }
        }
      }
      try {
        if (op == kOpBarrier) {
          std::vector<double> one(1, 1.0);
          ex->AllReduceSum(&one);
        } else if (op == kOpReduce) {
          // the process's values ride on one local worker's request; the exchange's own
          // collectives are issued by this thread only, so every rank issues them in one order
          std::vector<double>* v = nullptr;
          for (int l = 0; l < L; ++l)
            if (reqs[l] && reqs[l]->red) v = reqs[l]->red;
          if (v) ex->AllReduceSum(v);
        } else {
          Exec(op, reqs);
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu);
        failure = e.what();
        cv_done.notify_all();
        return;
      }
      for (int l = 0; l < L; ++l) {
        if (!reqs[l]) continue;
        if (served[l].cb) {
          // requests the callback issues are this worker's next ones
          {
            std::lock_guard<std::mutex> lk(mu);
            cb_first_ts_ = next_ts[l];
          }
          t_in_callback_of = l;
          served[l].cb();
          t_in_callback_of = -1;
          std::lock_guard<std::mutex> lk(mu);
          cb_first_ts_ = 1 << 30;
        }
        std::lock_guard<std::mutex> lk(mu);
        MarkDone(l, served[l].ts);
        cv_done.notify_all();
      }
    }
  }
}

void GpuDistStore::Core::Exec(int op, const std::vector<Req*>& reqs) {
  // split every worker's keys by owner (sorted keys: contiguous runs, kvstore_dist.h:101,111)
  std::vector<std::vector<int64_t>> send(L, std::vector<int64_t>(N, 0)), recv;
  std::vector<int64_t> U(L), R(L);
  std::vector<const void*> ks(L), cs(L), ps(L);
  std::vector<void*> kr(L), cr(L), pr(L);
  for (int l = 0; l < L; ++l) {
    const Req* rq = reqs[l];
    U[l] = rq ? (int64_t)rq->keys.size() : 0;
    for (int64_t i = 0; i < U[l]; ++i) {
      DFX_HOST_CHECK(i == 0 || rq->keys[i - 1] <= rq->keys[i],
                     "fea_ids must in non-decreasing order");
      ++send[l][OwnerOf(rq->keys[i], N)];
    }
    Bufs& b = *bufs[l];
    b.keys.ensure(U[l]);
    if (U[l])
      DfxCheck(dfx_memcpy(ctxs[l], b.keys.get(), rq->keys.data(), U[l] * 8, 0), "upload keys");
    ks[l] = b.keys.get();
    if (op == kOpCount) {
      DFX_HOST_CHECK(!rq || (int64_t)rq->vals.size() == U[l], "kFeaCount: one count per key");
      b.cnt.ensure(U[l]);
      if (U[l])
        DfxCheck(dfx_memcpy(ctxs[l], b.cnt.get(), rq->vals.data(), U[l] * 4, 0), "upload counts");
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
  // every sub-round begins its own owner step: table slots may move at a sync point in between
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
      const Req* rq = reqs[l];
      if (!rq) continue;
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
      rq->out_vals->CopyFrom(vals.data(), vals.size());
      if (rq->out_lens) {
        if (d > 0) {
          rq->out_lens->CopyFrom(lens.data(), lens.size());
        } else {
          rq->out_lens->clear();
        }
      }
    }
    Sync();
    return;
  }
  // kGradient: Get-layout gradients (the lens of the pull) -> records [gV | gw | live | 0 0]
  for (int l = 0; l < L; ++l) {
    const Req* rq = reqs[l];
    host.assign((size_t)U[l] * S, 0.f);
    if (rq) {
      const SArray<real_t>& g = rq->vals;
      const SArray<int>& lens = rq->lens;
      DFX_HOST_CHECK(d == 0 || U[l] == 0 || (int64_t)lens.size() == U[l],
                     "kGradient: one length per key");
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
    }
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
    r.keys = fea_ids;
    r.vals = vals;
    r.lens = lens;
    r.cb = on_complete;
    return core_->Enqueue(l_, std::move(r));
  }
  int Pull(const SArray<feaid_t>& fea_ids, int val_type, SArray<real_t>* vals, SArray<int>* lens,
           const std::function<void()>& on_complete) override {
    DFX_HOST_CHECK(val_type == kWeight, "GpuDistStore::Pull: kWeight");
    DFX_HOST_CHECK(vals != nullptr, "GpuDistStore::Pull: null vals");
    Req r;
    r.op = kOpPull;
    r.keys = fea_ids;
    r.out_vals = vals;
    r.out_lens = lens;
    r.cb = on_complete;
    return core_->Enqueue(l_, std::move(r));
  }
  void Wait(int ts) override { core_->Wait(l_, ts); }
  int NumWorkers() override { return core_->N; }
  int NumServers() override { return core_->N; }
  int Rank() override { return core_->ex->rank(l_); }
  // the servers' updaters are the shard contexts (built from the store's kwargs)
  void SetUpdater(const std::shared_ptr<Updater>& updater) override { updater_ = updater; }
  void Barrier() override {
    Req r;
    r.op = kOpBarrier;
    core_->Wait(l_, core_->Enqueue(l_, std::move(r)));
  }

 private:
  GpuDistStore::Core* core_;
  int l_;
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

GpuDistStore::~GpuDistStore() { core_->Stop(); }

void GpuDistStore::AllReduceSum(std::vector<double>* v) {
  DFX_HOST_CHECK(t_in_callback_of < 0, "GpuDistStore::AllReduceSum from a request callback");
  std::vector<int> ts(core_->L);
  for (int l = 0; l < core_->L; ++l) {
    Req r;
    r.op = kOpReduce;
    r.red = l == 0 ? v : nullptr;
    ts[l] = core_->Enqueue(l, std::move(r));
  }
  for (int l = 0; l < core_->L; ++l) core_->Wait(l, ts[l]);
}

std::shared_ptr<GpuDistStore> GpuDistStore::CreateLoopback(int nshards, const KWArgs& kwargs) {
  DFX_HOST_CHECK(nshards >= 1, "GpuDistStore: nshards >= 1");
  std::unique_ptr<Core> c(new Core());
  const std::string kw = CtxKw(kwargs);
  c->lockstep = LockstepOf(kwargs);
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
  const std::string id_file = CommIdFile();
  std::unique_ptr<Core> c(new Core());
  c->lockstep = LockstepOf(kwargs);
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
