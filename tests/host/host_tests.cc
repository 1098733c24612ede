// host_tests.cc — the reference's own hot-path gtests, restated against the C++ adapters
// (difacto_amd/host/gpu_adapters.h) so they run through the same plugin interfaces the
// reference's SGDLearner uses.  Needs a GPU; run by tests/test_host_cpp.py (-m gpu).
//
//   Localizer.Base / BaseHash   tests/cpp/localizer_test.cc:12-63
//   FMLoss.NoV / HasV           tests/cpp/fm_loss_test.cc:12-83
//   SGDLearner.Basic            tests/cpp/sgd_learner_test.cc:9-49 (interface and fused drivers)
//   + the two drivers agree on an FM V_dim=8 run, and Save/Load round-trips through a Stream
//
// Usage: host_tests <path to tests/golden/rcv1_100.libsvm>.  Exit status 0 == all passed.
//
// host_tests dist <data> shards=N|-1 epochs=E batch_size=B [model_out=P] [dfx_ctx kwargs]:
// SGDLearner::IterateData's executor (sgd_learner.cc:201-317: Compact -> Push(kFeaCount) + Wait
// -> Pull -> Predict / Evaluate / AUC -> CalcGrad -> Push(kGradient)) through the Store interface
// of a GpuDistStore (dist_store.h): N loopback workers, one thread each, or (shards=-1) one
// RCCL worker per process.  Worker r trains rows [r n / N, (r + 1) n / N) in batches of B, the
// workers stepping together (an idle worker passes empty batches).  Prints one line per epoch,
// "epoch E loss L auc A nrows R" summed over the workers, which tests/test_host_cpp.py compares
// with oracle/dist_oracle.py; model_out: each server saves its part (with aux) to P_part-<rank>.
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

#include "../../difacto_amd/host/dist_store.h"
#include "../../difacto_amd/host/gpu_adapters.h"
#include "../../difacto_amd/host/split_learner.h"

using namespace difacto;

static int g_fail = 0;
#define EXPECT(cond, ...)                                                     \
  do {                                                                        \
    if (!(cond)) {                                                            \
      std::printf("  FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond);           \
      std::printf(__VA_ARGS__);                                               \
      std::printf("\n");                                                      \
      ++g_fail;                                                               \
    }                                                                         \
  } while (0)

static feaid_t ReverseBytes(feaid_t x) {  // include/difacto/base.h:39-51 (test-side)
  x = x << 32 | x >> 32;
  x = (x & 0x0000FFFF0000FFFFULL) << 16 | (x & 0xFFFF0000FFFF0000ULL) >> 16;
  x = (x & 0x00FF00FF00FF00FFULL) << 8 | (x & 0xFF00FF00FF00FF00ULL) >> 8;
  x = (x & 0x0F0F0F0F0F0F0F0FULL) << 4 | (x & 0xF0F0F0F0F0F0F0F0ULL) >> 4;
  return x;
}

static void TestLocalizer(const RowBlockContainer<feaid_t>& data) {
  std::printf("Localizer.Base / BaseHash\n");
  auto ctx = std::make_shared<GpuContext>(0, KWArgs{{"max_keys", "16"}});
  for (feaid_t max_index : {~(feaid_t)0, (feaid_t)1000}) {
    GpuLocalizer lc(ctx, max_index);
    RowBlockContainer<unsigned> compacted;
    std::vector<feaid_t> uidx;
    std::vector<real_t> cnt;
    lc.Compact(data.GetBlock(), &compacted, &uidx, &cnt);
    uint64_t su = 0;
    double sc = 0;
    for (size_t i = 0; i < uidx.size(); ++i) {
      su += ReverseBytes(uidx[i]);
      sc += cnt[i];
      if (i) EXPECT(uidx[i - 1] < uidx[i], "uniq not ascending at %zu", i);
    }
    const uint64_t want = max_index == ~(feaid_t)0 ? 65111856ull : 478817ull;
    EXPECT(su == want, "sum uidx %llu want %llu", (unsigned long long)su,
           (unsigned long long)want);
    EXPECT(sc == 9648, "sum cnt %f", sc);
    EXPECT(compacted.index.size() == data.index.size(), "nnz kept");
    EXPECT(compacted.max_index + 1 == uidx.size(), "max_index");
    // the remap is a bijection onto the ranks: keys of equal ids share a column
    for (size_t j = 0; j < data.index.size(); ++j) {
      const feaid_t id = max_index == ~(feaid_t)0 ? data.index[j] : data.index[j] % max_index;
      if (ReverseBytes(uidx[compacted.index[j]]) != id) {
        EXPECT(false, "remap mismatch at nnz %zu", j);
        break;
      }
    }
  }
}

// FMLoss known answers: w[i] = id/5e4, V[i][j] = id*j/5e5 (fm_loss_test.cc:20-33,50-70)
static void TestFMLoss(const RowBlockContainer<feaid_t>& data, int d, double objv_want,
                       double objv_tol, double g2_want, double g2_tol) {
  std::printf("FMLoss.%s\n", d ? "HasV" : "NoV");
  auto ctx = std::make_shared<GpuContext>(0, KWArgs{{"max_keys", "16"}});
  GpuLocalizer lc(ctx);
  RowBlockContainer<unsigned> compacted;
  std::vector<feaid_t> uidx;
  lc.Compact(data.GetBlock(), &compacted, &uidx);
  const size_t U = uidx.size();
  SArray<real_t> w(U * (d + 1));
  SArray<int> w_pos, V_pos;
  for (size_t i = 0; i < U; ++i) {
    const double id = (double)ReverseBytes(uidx[i]);
    w[i * (d + 1)] = (real_t)(id / 5e4);
    for (int j = 1; j <= d; ++j) w[i * (d + 1) + j] = (real_t)(id * j / 5e5);
  }
  if (d) {
    SArray<int> lens(U, d + 1);
    GetPos(lens, &w_pos, &V_pos);
  }
  GpuFMLoss loss(d == 0);
  loss.Init({{"V_dim", std::to_string(d)}});
  auto blk = compacted.GetBlock();
  SArray<real_t> pred(blk.size);
  std::vector<SArray<char>> param = {SArray<char>(w), SArray<char>(w_pos), SArray<char>(V_pos)};
  loss.Predict(blk, param, &pred);
  const double objv = loss.Evaluate(blk.label, pred);
  EXPECT(std::fabs(objv - objv_want) < objv_tol, "objv %.6f want %.6f", objv, objv_want);
  SArray<real_t> grad(w.size());
  param.push_back(SArray<char>(pred));
  loss.CalcGrad(blk, param, &grad);
  double g2 = 0;
  for (real_t g : grad) g2 += (double)g * g;
  EXPECT(std::fabs(g2 - g2_want) < g2_tol, "|g|^2 %.6f want %.6f", g2, g2_want);
}

// SGDLearner.Basic: V_dim 0, l1 = l2 = lr = 1, one 100-row batch per epoch, 20 epochs
static void TestSGDLearnerBasic(const RowBlockContainer<feaid_t>& data, bool fused) {
  std::printf("SGDLearner.Basic (%s)\n", fused ? "fused dfx_train_step" : "interfaces");
  static const double objv[] = {69.314718, 69.314718, 67.151912, 61.414778, 56.244989,
                                53.218700, 51.248737, 49.846688, 48.650164, 47.698351,
                                46.924038, 46.388223, 45.970721, 45.499307, 45.102245,
                                44.798413, 44.565211, 44.386417, 44.240657, 44.109764};
  GpuSGDLearner learner({{"V_dim", "0"}, {"l2", "1"}, {"l1", "1"}, {"lr", "1"},
                         {"fused", fused ? "1" : "0"}, {"max_keys", "16384"}});
  for (int ep = 0; ep < 20; ++ep) {
    learner.ProcessBatch(data.GetBlock(), GpuSGDLearner::kTraining, ep == 0);
    const Progress prog = learner.TakeProgress();
    EXPECT(std::fabs(prog.loss - objv[ep]) < 5e-5, "epoch %d objv %.6f want %.6f", ep, prog.loss,
           objv[ep]);
    EXPECT(prog.nrows == 100, "nrows");
  }
}

// the interface driver and the fused step are two routes through the same kernels
static void TestDriversAgree(const RowBlockContainer<feaid_t>& data) {
  std::printf("FM V_dim=8: interface driver == fused step; Save/Load round trip\n");
  KWArgs kw = {{"V_dim", "8"}, {"V_threshold", "1"}, {"l1", "0.05"}, {"lr", "0.1"},
               {"V_lr", "0.01"}, {"max_keys", "16384"}};
  KWArgs kf = kw, ki = kw;
  kf.push_back({"fused", "1"});
  ki.push_back({"fused", "0"});
  GpuSGDLearner a(ki), b(kf);
  RowSlice h0 = Slice(data, 0, 50), h1 = Slice(data, 50, 100);
  for (int ep = 0; ep < 5; ++ep) {
    for (RowSlice* h : {&h0, &h1}) {
      a.ProcessBatch(h->blk, GpuSGDLearner::kTraining, ep == 0);
      b.ProcessBatch(h->blk, GpuSGDLearner::kTraining, ep == 0);
      const Progress pa = a.TakeProgress(), pb = b.TakeProgress();
      EXPECT(std::fabs(pa.loss - pb.loss) <= 1e-4 * std::fabs(pb.loss), "epoch %d loss %.7f vs %.7f",
             ep, pa.loss, pb.loss);
      EXPECT(std::fabs(pa.auc - pb.auc) <= 1e-4 * 50, "epoch %d auc %.7f vs %.7f", ep, pa.auc,
             pb.auc);
    }
  }
  // Save (with aux) -> Load into a fresh updater -> identical pulls
  const char* path = "/tmp/difacto_amd_host_test_model";
  {
    FileStream fo(path, "w");
    b.updater()->Save(true, &fo);
  }
  GpuSGDUpdater fresh;
  fresh.Init(kw);
  {
    FileStream fi(path, "r");
    fresh.Load(&fi);
  }
  auto ctx = std::make_shared<GpuContext>(0, KWArgs{{"max_keys", "16"}});
  GpuLocalizer lc(ctx);
  RowBlockContainer<unsigned> compacted;
  auto uidx = std::make_shared<std::vector<feaid_t>>();
  lc.Compact(data.GetBlock(), &compacted, uidx.get());
  SArray<feaid_t> keys(uidx);
  SArray<real_t> v0, v1;
  SArray<int> l0, l1;
  b.updater()->Get(keys, Store::kWeight, &v0, &l0);
  fresh.Get(keys, Store::kWeight, &v1, &l1);
  EXPECT(v0.size() == v1.size() && l0.size() == l1.size(), "pull sizes %zu %zu", v0.size(),
         v1.size());
  bool same = v0.size() == v1.size();
  for (size_t i = 0; same && i < v0.size(); ++i) same = v0[i] == v1[i];
  for (size_t i = 0; same && i < l0.size(); ++i) same = l0[i] == l1[i];
  EXPECT(same, "loaded model differs");
  std::remove(path);
}

static int RunDist(int argc, char** argv) {
  RowBlockContainer<feaid_t> data;
  if (argc < 3 || !ReadLibSVM(argv[2], &data)) {
    std::fprintf(stderr, "usage: %s dist <data> shards=N|-1 epochs=E batch_size=B ...\n", argv[0]);
    return 2;
  }
  int shards = 1, epochs = 1;
  size_t bs = 10;
  std::string model_out, vdim = "0";
  KWArgs kw;
  for (int i = 3; i < argc; ++i) {
    const std::string a = argv[i];
    const size_t eq = a.find('=');
    if (eq == std::string::npos) return 2;
    const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
    if (k == "shards") {
      shards = std::stoi(v);
    } else if (k == "epochs") {
      epochs = std::stoi(v);
    } else if (k == "batch_size") {
      bs = std::stoul(v);
    } else if (k == "model_out") {
      model_out = v;
    } else {
      if (k == "V_dim") vdim = v;
      kw.push_back({k, v});
    }
  }
  const char* lr_env = std::getenv("LOCAL_RANK");
  const std::string device = shards < 0 && lr_env ? lr_env : "0";
  std::shared_ptr<GpuDistStore> ds =
      shards > 0 ? GpuDistStore::CreateLoopback(shards, kw) : GpuDistStore::CreateRccl(kw);
  ShardExchange* ex = ds->exchange();
  const int L = ds->nlocal(), N = ex->nranks();
  const size_t n = data.Size();
  size_t nsteps = 0;
  for (int r = 0; r < N; ++r) {
    const size_t rows = (size_t)(r + 1) * n / N - (size_t)r * n / N;
    nsteps = std::max(nsteps, (rows + bs - 1) / bs);
  }
  std::vector<std::unique_ptr<GpuSGDLearner>> learners(L);
  for (int l = 0; l < L; ++l) {
    Store* w = ds->worker(l);
    EXPECT(w->NumWorkers() == N && w->NumServers() == N && w->Rank() == ex->rank(l),
           "worker %d: NumWorkers %d Rank %d", l, w->NumWorkers(), w->Rank());
    // the aliasing shared_ptr keeps the store alive as long as the learner holds its worker
    learners[l].reset(new GpuSGDLearner({{"fused", "0"}, {"V_dim", vdim}, {"device", device}},
                                        std::shared_ptr<Store>(ds, w)));
  }
  for (int ep = 0; ep < epochs; ++ep) {
    std::vector<Progress> prog(L);
    std::vector<std::thread> th;
    for (int l = 0; l < L; ++l) {
      th.emplace_back([&, l]() {
        const int r = ex->rank(l);
        const size_t lo = (size_t)r * n / N, hi = (size_t)(r + 1) * n / N;
        for (size_t t = 0; t < nsteps; ++t) {
          const size_t b = std::min(hi, lo + t * bs), e = std::min(hi, lo + (t + 1) * bs);
          RowSlice s = Slice(data, b, e);
          learners[l]->ProcessBatch(s.blk, GpuSGDLearner::kTraining, ep == 0);
        }
        prog[l] = learners[l]->TakeProgress();
      });
    }
    for (auto& t : th) t.join();
    std::vector<double> sum(3, 0.0);
    for (const Progress& p : prog) {
      sum[0] += p.loss;
      sum[1] += p.auc;
      sum[2] += p.nrows;
    }
    ds->AllReduceSum(&sum);
    if (ex->rank(0) == 0)
      std::printf("epoch %d loss %.9e auc %.9e nrows %.0f\n", ep, sum[0], sum[1], sum[2]);
    std::fflush(stdout);
  }
  if (!model_out.empty())
    for (int l = 0; l < L; ++l)
      DfxCheck(dfx_store_save(ds->shard(l),
                              (model_out + "_part-" + std::to_string(ex->rank(l))).c_str(), 1),
               "dfx_store_save");
  learners.clear();
  std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
  return g_fail ? 1 : 0;
}

// SGDLearner::IterateData (sgd_learner.cc:201-317) restated over the adapters and a Store, with
// its threads: this thread is the reader — it localizes each batch, pushes the batch's counts
// (+ Wait) and issues it; an executor thread pulls with a callback, and the callback (run by the
// store) predicts, evaluates, computes the AUC and the gradient and pushes it, the batch done
// when that push completes; at most two batches in flight (batch_tracker.NumRemains() > 1).
// One deviation: Issue returns once the executor has issued the batch's Pull (the reference's
// AsyncLocalTracker returns at once), so the count push of the next batch always queues after
// that pull and a one-worker run is deterministic.
static Progress IterateDataAsync(Store* store, GpuLocalizer& lc, GpuFMLoss& loss, int V_dim,
                                 const std::vector<RowSlice>& batches, bool push_cnt) {
  struct Job {
    RowBlockContainer<unsigned> data;
    SArray<feaid_t> feaids;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::shared_ptr<Job>> queue;
  int remains = 0;        // issued, not yet complete
  bool issued_pull = false, end = false;
  Progress prog;
  std::thread executor([&]() {
    while (true) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&]() { return !queue.empty() || end; });
        if (queue.empty()) return;
        job = queue.front();
        queue.pop_front();
      }
      auto values = std::make_shared<SArray<real_t>>();
      auto lengths = V_dim > 0 ? std::make_shared<SArray<int>>() : nullptr;
      auto pull_callback = [&, job, values, lengths]() {
        dmlc::RowBlock<unsigned> data = job->data.GetBlock();
        SArray<real_t> pred(data.size);
        SArray<int> w_pos, V_pos;
        if (lengths) GetPos(*lengths, &w_pos, &V_pos);
        std::vector<SArray<char>> inputs = {SArray<char>(*values), SArray<char>(w_pos),
                                            SArray<char>(V_pos)};
        if (data.size) loss.Predict(data, inputs, &pred);
        const double l = data.size ? loss.Evaluate(data.label, pred) : 0.0;
        const double auc = data.size ? loss.AUC(data.label, pred) : 0.0;
        {
          std::lock_guard<std::mutex> lk(mu);
          prog.nrows += data.size;
          prog.loss += l;
          prog.auc += auc;
        }
        SArray<real_t> grads(values->size());
        inputs.push_back(SArray<char>(pred));
        if (data.size) loss.CalcGrad(data, inputs, &grads);
        store->Push(job->feaids, Store::kGradient, grads, lengths ? *lengths : SArray<int>(),
                    [&]() {
                      std::lock_guard<std::mutex> lk(mu);
                      --remains;
                      cv.notify_all();
                    });
      };
      store->Pull(job->feaids, Store::kWeight, values.get(), lengths.get(), pull_callback);
      std::lock_guard<std::mutex> lk(mu);
      issued_pull = true;
      cv.notify_all();
    }
  });
  for (const RowSlice& b : batches) {
    auto job = std::make_shared<Job>();
    auto feaids = std::make_shared<std::vector<feaid_t>>();
    auto feacnt = std::make_shared<std::vector<real_t>>();
    lc.Compact(b.blk, &job->data, feaids.get(), push_cnt ? feacnt.get() : nullptr);
    job->feaids = SArray<feaid_t>(feaids);
    if (push_cnt)
      store->Wait(store->Push(job->feaids, Store::kFeaCount, SArray<real_t>(feacnt), {}));
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&]() { return remains <= 1; });  // while (NumRemains() > 1) sleep
    ++remains;
    issued_pull = false;
    queue.push_back(job);
    cv.notify_all();
    cv.wait(lk, [&]() { return issued_pull; });
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&]() { return remains == 0; });  // batch_tracker.Wait()
    end = true;
    cv.notify_all();
  }
  executor.join();
  return prog;
}

// host_tests dist_async <data> shards=N|-1 epochs=E batch_size=B uneven=0|1 [dfx_ctx kwargs,
// store_sync]: N workers, each running IterateDataAsync (reader + executor threads) over its
// share of the rows: rows [r n / N, (r + 1) n / N), or (uneven=1) r + 1 parts of N (N + 1) / 2,
// so the workers hold different numbers of batches (store_sync=async).  Prints
// "epoch E loss L auc A nrows R" summed over the workers.
static int RunDistAsync(int argc, char** argv) {
  RowBlockContainer<feaid_t> data;
  if (argc < 3 || !ReadLibSVM(argv[2], &data)) return 2;
  int shards = 1, epochs = 1;
  bool uneven = false;
  size_t bs = 10;
  std::string vdim = "0";
  KWArgs kw;
  for (int i = 3; i < argc; ++i) {
    const std::string a = argv[i];
    const size_t eq = a.find('=');
    if (eq == std::string::npos) return 2;
    const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
    if (k == "uneven") uneven = std::stoi(v) != 0;
    else if (k == "shards") shards = std::stoi(v);
    else if (k == "epochs") epochs = std::stoi(v);
    else if (k == "batch_size") bs = std::stoul(v);
    else {
      if (k == "V_dim") vdim = v;
      kw.push_back({k, v});
    }
  }
  const char* lr_env = std::getenv("LOCAL_RANK");
  const int device = shards < 0 && lr_env ? std::atoi(lr_env) : 0;
  std::shared_ptr<GpuDistStore> ds =
      shards > 0 ? GpuDistStore::CreateLoopback(shards, kw) : GpuDistStore::CreateRccl(kw);
  ShardExchange* ex = ds->exchange();
  const int L = ds->nlocal(), N = ex->nranks();
  const size_t n = data.Size(), tri = (size_t)N * (N + 1) / 2;
  const int d = std::stoi(vdim);
  std::vector<std::unique_ptr<GpuLocalizer>> lcs;
  std::vector<std::unique_ptr<GpuFMLoss>> losses;
  for (int l = 0; l < L; ++l) {
    lcs.emplace_back(new GpuLocalizer(std::make_shared<GpuContext>(
        device, KWArgs{{"V_dim", vdim}, {"max_keys", "16"}, {"max_vrows", "1"}})));
    losses.emplace_back(new GpuFMLoss(d == 0));
    losses.back()->Init({{"V_dim", vdim}, {"device", std::to_string(device)}});
  }
  for (int ep = 0; ep < epochs; ++ep) {
    std::vector<Progress> prog(L);
    std::vector<std::thread> th;
    for (int l = 0; l < L; ++l) {
      th.emplace_back([&, l]() {
        const size_t r = (size_t)ex->rank(l);
        const size_t lo = uneven ? n * (r * (r + 1) / 2) / tri : r * n / N;
        const size_t hi = uneven ? n * ((r + 1) * (r + 2) / 2) / tri : (r + 1) * n / N;
        std::vector<RowSlice> batches;
        for (size_t b = lo; b < hi; b += bs) batches.push_back(Slice(data, b, std::min(hi, b + bs)));
        prog[l] = IterateDataAsync(ds->worker(l), *lcs[l], *losses[l], d, batches,
                                   ep == 0 && d > 0);
      });
    }
    for (auto& t : th) t.join();
    std::vector<double> sum(3, 0.0);
    for (const Progress& p : prog) {
      sum[0] += p.loss;
      sum[1] += p.auc;
      sum[2] += p.nrows;
    }
    ds->AllReduceSum(&sum);
    EXPECT(sum[2] == (double)n, "epoch %d nrows %.0f want %zu", ep, sum[2], n);
    if (ex->rank(0) == 0)
      std::printf("epoch %d loss %.9e auc %.9e nrows %.0f\n", ep, sum[0], sum[1], sum[2]);
    std::fflush(stdout);
  }
  losses.clear();
  lcs.clear();
  ds.reset();
  std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
  return g_fail ? 1 : 0;
}

// host_tests split <data> shards=N|-1 epochs=E batch_size=B [model_out=P] [kwargs]: the
// owner-computes split behind GpuSplitLearner (split_learner.h) — IterateData's executor fed
// the raw minibatches of N loopback workers (one thread each) or one RCCL worker per process
// (shards=-1): rows [r n / N, (r + 1) n / N) for worker r in batches of B, the workers stepping
// together (an idle worker gives an empty batch).  Prints "epoch E loss L auc A nrows R" summed
// over the workers; saves every server's model part.
static int RunSplit(int argc, char** argv) {
  RowBlockContainer<feaid_t> data;
  if (argc < 3 || !ReadLibSVM(argv[2], &data)) return 2;
  int shards = 1, epochs = 1;
  size_t bs = 10;
  std::string model_out, vdim = "0";
  KWArgs kw;
  for (int i = 3; i < argc; ++i) {
    const std::string a = argv[i];
    const size_t eq = a.find('=');
    if (eq == std::string::npos) return 2;
    const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
    if (k == "shards") shards = std::stoi(v);
    else if (k == "epochs") epochs = std::stoi(v);
    else if (k == "batch_size") bs = std::stoul(v);
    else if (k == "model_out") model_out = v;
    else {
      if (k == "V_dim") vdim = v;
      kw.push_back({k, v});
    }
  }
  std::shared_ptr<GpuSplitLearner> sl =
      shards > 0 ? GpuSplitLearner::CreateLoopback(shards, kw) : GpuSplitLearner::CreateRccl(kw);
  const int L = sl->nlocal(), N = sl->nranks();
  const size_t n = data.Size();
  size_t nsteps = 0;
  for (int r = 0; r < N; ++r) {
    const size_t rows = (size_t)(r + 1) * n / N - (size_t)r * n / N;
    nsteps = std::max(nsteps, (rows + bs - 1) / bs);
  }
  for (int ep = 0; ep < epochs; ++ep) {
    std::vector<std::thread> th;
    for (int l = 0; l < L; ++l) {
      th.emplace_back([&, l]() {
        const int r = sl->rank(l);
        const size_t lo = (size_t)r * n / N, hi = (size_t)(r + 1) * n / N;
        for (size_t t = 0; t < nsteps; ++t) {
          const size_t b = std::min(hi, lo + t * bs), e = std::min(hi, lo + (t + 1) * bs);
          RowSlice s = Slice(data, b, e);
          sl->ProcessBatch(l, s.blk, GpuSplitLearner::kTraining, ep == 0 && vdim != "0");
        }
      });
    }
    for (auto& t : th) t.join();
    std::vector<double> sum(3, 0.0);
    for (int l = 0; l < L; ++l) {
      const Progress p = sl->TakeProgress(l);
      sum[0] += p.loss;
      sum[1] += p.auc;
      sum[2] += p.nrows;
    }
    sl->AllReduceSum(&sum);
    EXPECT(sum[2] == (double)n, "epoch %d nrows %.0f want %zu", ep, sum[2], n);
    if (sl->rank(0) == 0)
      std::printf("epoch %d loss %.9e auc %.9e nrows %.0f\n", ep, sum[0], sum[1], sum[2]);
    std::fflush(stdout);
  }
  if (!model_out.empty())
    for (int l = 0; l < L; ++l)
      DfxCheck(dfx_store_save(sl->shard(l), (model_out + "_part-" + std::to_string(sl->rank(l))).c_str(),
                              1),
               "dfx_store_save");
  sl.reset();
  std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
  return g_fail ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "split") return RunSplit(argc, argv);
  if (argc >= 2 && std::string(argv[1]) == "dist") return RunDist(argc, argv);
  if (argc >= 2 && std::string(argv[1]) == "dist_async") return RunDistAsync(argc, argv);
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s rcv1_100.libsvm\n", argv[0]);
    return 2;
  }
  RowBlockContainer<feaid_t> data;
  if (!ReadLibSVM(argv[1], &data)) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  std::printf("rcv1-100: %zu rows, %zu nnz\n", data.Size(), data.index.size());
  TestLocalizer(data);
  TestFMLoss(data, 0, 147.4672, 1e-3, 90.5817, 1e-3);
  TestFMLoss(data, 5, 330.628, 1e-3, 1237.8, 0.1);
  TestSGDLearnerBasic(data, false);
  TestSGDLearnerBasic(data, true);
  TestDriversAgree(data);
  std::printf(g_fail ? "FAILED (%d)\n" : "ALL PASSED\n", g_fail);
  return g_fail ? 1 : 0;
}
