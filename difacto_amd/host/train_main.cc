// train_main.cc — dfx_train: the reference's `difacto` executable for the SGD learner
// (src/main.cc + SGDLearner::RunScheduler, src/sgd/sgd_learner.cc:51-117) on one GPU.
//
//   build/dfx_train data_in=FILE [data_val=FILE] [data_format=libsvm|criteo|criteo_test]
//                   [batch_size=100] [shuffle=10] [neg_sampling=1] [max_num_epochs=20]
//                   [num_jobs_per_epoch=10] [stop_rel_objv=1e-5] [model_in=F] [model_out=F]
//                   [load_epoch=-1] [has_aux=0] [task=0|2] [pred_out=F] [pred_prob=1]
//                   [fused=1] [nthreads=8] [V_dim=..] [lr=..] [l1=..] ...  (SGDUpdaterParam)
//
// Sharded store (KVStoreDist over GPUs, dist_host.h): `shards=N` holds N shards on this GPU
// (loopback exchange, for tests); `shards=-1` or a launch with WORLD_SIZE > 1 (RANK / LOCAL_RANK as
// torchrun sets them; DFX_COMM_ID_FILE or /tmp/dfx_comm_<MASTER_PORT> as the node-local
// rendezvous) runs one shard per process over RCCL.  Every epoch is split into
// num_jobs_per_epoch x shards parts; shard r reads parts r, r + shards, ... in order, the shards
// step together (an exhausted shard submits empty batches until all are done), and
// `pipelined=1` (default) selects the 1-step-stale schedule.  Each server saves
// <model_out>_part-<rank>; `model_in_parts=K` loads a model K servers saved into this run's
// shards (each keeps the keys it owns).  `exchange=split` runs the sharded epochs through the
// owner-computes split (GpuSplitLearner, split_learner.h) instead of KVStoreDist's exchanges.
//
// Model files are named like SGDLearner::ModelName (sgd_learner.h:65-69):
// <prefix>[_iter-<epoch>]_part-0, in SGDUpdater::Save's format; task=2 predicts data_val with
// model_in into <pred_out>_part-0, one "label\tprediction" line per row (SavePred,
// sgd_learner.h:72-83).
//
// Each epoch reads data_in in num_jobs_per_epoch parts (the reference's jobs, here run in
// order), minibatched by BatchReader (reader.h) and trained through GpuSGDLearner, i.e. one
// dfx_train_step per batch behind a pinned-staging dfx_feeder.  It prints the reference's
// "Epoch[k] Training: Rows = .., loss = .., AUC = .." line per epoch, plus the rate including
// parsing and PCIe (host ex/s), which is NOT the device-resident rate bench.py reports.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>

#include "dist_host.h"
#include "gpu_adapters.h"
#include "reader.h"
#include "split_learner.h"

using namespace difacto;

namespace {
struct Param {
  std::string data_in, data_val, data_format = "libsvm", model_in, model_out, pred_out;
  size_t batch_size = 100, shuffle = 10;
  float neg_sampling = 1.f;
  int max_num_epochs = 20, num_jobs_per_epoch = 10, nthreads = 8;
  int load_epoch = -1, task = 0;
  int shards = 0;  // > 0: that many loopback shards in this process; -1: one shard, RCCL
  int model_in_parts = 0;  // servers that saved model_in, when not this run's shard count
  bool pipelined = true;
  std::string exchange = "a2a";  // a2a: GpuShardedStore (KVStoreDist); split: GpuSplitLearner
  bool has_aux = false, pred_prob = true;
  double stop_rel_objv = 1e-5;
};

// sgd_learner.h:65-69
std::string ModelNamePart(const std::string& prefix, int iter, int rank) {
  std::string name = prefix;
  if (iter >= 0) name += "_iter-" + std::to_string(iter);
  return name + "_part-" + std::to_string(rank);
}
std::string ModelName(const std::string& prefix, int iter) {  // one server: rank 0
  return ModelNamePart(prefix, iter, 0);
}

double Now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// sgd_utils.h:59-63
std::string Text(const Progress& p) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), "Rows = %.0f, loss = %.9g, AUC = %.9g", p.nrows,
                p.loss / p.nrows, p.auc / p.nrows);
  return buf;
}

Progress RunEpoch(GpuSGDLearner* learner, const Param& P, int epoch, int job_type,
                  FILE* pred_file = nullptr) {
  Progress prog;
  std::vector<real_t> pred;
  const bool train = job_type == GpuSGDLearner::kTraining;
  const std::string& path = train ? P.data_in : P.data_val;
  for (int part = 0; part < P.num_jobs_per_epoch; ++part) {
    if (train) {
      // sgd_learner.cc:273-280
      ThreadedBatchReader reader(path, P.data_format, part, P.num_jobs_per_epoch, P.batch_size,
                                 P.batch_size * P.shuffle, P.neg_sampling, P.nthreads);
      while (reader.Next()) {
        const auto blk = reader.Value().GetBlock();
        learner->ProcessBatch(blk, job_type, epoch == 0);
      }
    } else {
      // sgd_learner.cc:281-286: validation reads whole 256 MB chunks as one batch
      TextReader reader(path, P.data_format, part, P.num_jobs_per_epoch, 256 << 20, P.nthreads);
      while (reader.Next()) {
        const auto& v = reader.Value();
        if (v.Size() == 0) continue;
        learner->ProcessBatch(v.GetBlock(), job_type, false, pred_file ? &pred : nullptr);
        for (size_t i = 0; pred_file && i < pred.size(); ++i)  // SavePred
          std::fprintf(pred_file, "%g\t%g\n", v.label[i],
                       P.pred_prob ? 1.0 / (1.0 + std::exp(-pred[i])) : (double)pred[i]);
      }
    }
    const Progress p = learner->TakeProgress();
    prog.nrows += p.nrows;
    prog.loss += p.loss;
    prog.auc += p.auc;
  }
  return prog;
}
// ---- the sharded store ----------------------------------------------------------------------
// a batch in device memory, uploaded on the context's stream (three per shard in flight)
struct DevBatch {
  dfx_ctx* c = nullptr;
  std::unique_ptr<DevArray<uint64_t>> off, idx;
  std::unique_ptr<DevArray<float>> val, lab, wt;
  dfx_batch b{};
  void Upload(dfx_ctx* ctx, const RowBlockContainer<feaid_t>* blk) {
    if (!off) {
      c = ctx;
      off.reset(new DevArray<uint64_t>(c));
      idx.reset(new DevArray<uint64_t>(c));
      val.reset(new DevArray<float>(c));
      lab.reset(new DevArray<float>(c));
      wt.reset(new DevArray<float>(c));
    }
    const size_t B = blk ? blk->Size() : 0, nnz = blk ? blk->index.size() : 0;
    static const uint64_t zero = 0;
    b = dfx_batch{};
    b.size = (int64_t)B;
    b.nnz = (int64_t)nnz;
    b.offset = blk ? reinterpret_cast<uint64_t*>(off->upload(
                         reinterpret_cast<const uint64_t*>(blk->offset.data()), B + 1))
                   : off->upload(&zero, 1);
    b.index = nnz ? idx->upload(blk->index.data(), nnz) : nullptr;
    b.value = blk && !blk->value.empty() ? val->upload(blk->value.data(), nnz) : nullptr;
    b.label = B ? lab->upload(blk->label.data(), B) : nullptr;
    b.weight = blk && !blk->weight.empty() ? wt->upload(blk->weight.data(), B) : nullptr;
  }
};

std::string KwString(const KWArgs& kw) {
  std::string s;
  for (const auto& p : kw) {
    if (p.first == "fused") continue;
    if (!s.empty()) s += ",";
    s += p.first + "=" + p.second;
  }
  return s;
}

// exchange=split: the owner-computes split behind GpuSplitLearner (split_learner.h): the same
// readers, parts and stop rule, one synchronous reference step per batch index on the
// concatenation of the shards' batches (push_agg=sum); pipelined=1 only overlaps model-free
// work, so the results equal the synchronous schedule
int RunShardedSplit(const Param& P, const KWArgs& rest) {
  const char* ws = std::getenv("WORLD_SIZE");
  const int world = ws ? std::atoi(ws) : 1;
  const bool rccl = world > 1 || P.shards < 0;
  KWArgs kw = rest;
  kw.push_back({"pipelined", P.pipelined ? "1" : "0"});
  std::shared_ptr<GpuSplitLearner> sl =
      rccl ? GpuSplitLearner::CreateRccl(kw) : GpuSplitLearner::CreateLoopback(P.shards, kw);
  const int nlocal = sl->nlocal(), nshards = sl->nranks(), rank = sl->rank(0);
  if (!P.model_in.empty()) {
    const int it = P.load_epoch > 0 ? P.load_epoch : -1;
    for (int l = 0; l < nlocal; ++l) {
      if (P.model_in_parts <= 0 || P.model_in_parts == nshards) {
        DfxCheck(dfx_store_load(sl->shard(l), ModelNamePart(P.model_in, it, sl->rank(l)).c_str()),
                 "dfx_store_load");
      } else {
        for (int r = 0; r < P.model_in_parts; ++r)
          DfxCheck(dfx_store_load_part(sl->shard(l), ModelNamePart(P.model_in, it, r).c_str(),
                                       sl->rank(l), nshards),
                   "dfx_store_load_part");
      }
    }
  }
  static const size_t kZeroOff = 0;
  dmlc::RowBlock<feaid_t> empty;
  empty.size = 0;
  empty.offset = &kZeroOff;
  const double t0 = Now();
  double pre_loss = 0;
  for (int k = std::max(0, P.load_epoch > 0 ? P.load_epoch + 1 : 0); k < P.max_num_epochs; ++k) {
    const double te = Now();
    for (int job = 0; job < P.num_jobs_per_epoch; ++job) {
      const int nparts = P.num_jobs_per_epoch * nshards;
      std::vector<std::unique_ptr<ThreadedBatchReader>> rd(nlocal);
      for (int l = 0; l < nlocal; ++l)
        rd[l].reset(new ThreadedBatchReader(P.data_in, P.data_format,
                                            job * nshards + sl->rank(l), nparts, P.batch_size,
                                            P.batch_size * P.shuffle, P.neg_sampling,
                                            P.nthreads));
      std::vector<bool> more(nlocal, true);
      std::vector<dmlc::RowBlock<feaid_t>> blk(nlocal);
      for (;;) {
        std::vector<double> any(1, 0.0);
        for (int l = 0; l < nlocal; ++l) {
          if (more[l]) more[l] = rd[l]->Next();
          if (more[l]) any[0] += 1;
        }
        sl->AllReduceSum(&any);
        if (any[0] == 0) break;
        std::vector<const dmlc::RowBlock<feaid_t>*> ptrs(nlocal);
        for (int l = 0; l < nlocal; ++l) {
          blk[l] = more[l] ? rd[l]->Value().GetBlock() : empty;
          ptrs[l] = &blk[l];
        }
        sl->ProcessBatches(ptrs, GpuSplitLearner::kTraining, k == 0);
      }
    }
    std::vector<double> pr(3, 0.0);
    for (int l = 0; l < nlocal; ++l) {
      const Progress p = sl->TakeProgress(l);
      pr[0] += p.nrows;
      pr[1] += p.loss;
      pr[2] += p.auc;
    }
    sl->AllReduceSum(&pr);
    Progress tr;
    tr.nrows = pr[0];
    tr.loss = pr[1];
    tr.auc = pr[2];
    const double dt = Now() - te;
    if (rank == 0)
      std::printf("Epoch[%d] Training: %s  (%.0f ex/s incl. parse+PCIe, %d shards, split, %.2f s)\n",
                  k, Text(tr).c_str(), tr.nrows / dt, nshards, Now() - t0);
    std::fflush(stdout);
    const double eps = std::fabs(tr.loss - pre_loss) / pre_loss;
    if (eps < P.stop_rel_objv) break;
    pre_loss = tr.loss;
  }
  sl->Flush();
  if (!P.model_out.empty())
    for (int l = 0; l < nlocal; ++l)
      DfxCheck(dfx_store_save(sl->shard(l), ModelNamePart(P.model_out, -1, sl->rank(l)).c_str(),
                              P.has_aux ? 1 : 0),
               "dfx_store_save");
  return 0;
}

int RunSharded(const Param& P, const KWArgs& rest) {
  if (P.exchange == "split") return RunShardedSplit(P, rest);
  if (P.exchange != "a2a") {
    std::fprintf(stderr, "exchange must be a2a or split\n");
    return 2;
  }
  const char* ws = std::getenv("WORLD_SIZE");
  const int world = ws ? std::atoi(ws) : 1;
  const bool rccl = world > 1 || P.shards < 0;
  const int rank = rccl && std::getenv("RANK") ? std::atoi(std::getenv("RANK")) : 0;
  const int local = std::getenv("LOCAL_RANK") ? std::atoi(std::getenv("LOCAL_RANK")) : 0;
  const int nlocal = rccl ? 1 : P.shards;
  const int nshards = rccl ? world : P.shards;
  if (P.task == 2 || !P.data_val.empty()) {
    std::fprintf(stderr, "sharded store: training only (task=0, no data_val)\n");
    return 2;
  }
  std::vector<dfx_ctx*> ctxs(nlocal, nullptr);
  const std::string kw = KwString(rest);
  for (int l = 0; l < nlocal; ++l)
    DfxCheck(dfx_ctx_create(rccl ? local : 0, kw.c_str(), &ctxs[l]), "dfx_ctx_create");
  std::unique_ptr<ShardExchange> ex;
  if (rccl) {
    std::string id_file;
    if (const char* f = std::getenv("DFX_COMM_ID_FILE")) {
      id_file = f;
    } else {
      const char* port = std::getenv("MASTER_PORT");
      id_file = std::string("/tmp/dfx_comm_") + (port ? port : "0");
    }
    ex = MakeRcclExchange(ctxs[0], rank, world, id_file);
  } else {
    ex = MakeLoopbackExchange(ctxs);
  }
  if (!P.model_in.empty()) {
    const int it = P.load_epoch > 0 ? P.load_epoch : -1;
    for (int l = 0; l < nlocal; ++l) {
      if (P.model_in_parts <= 0 || P.model_in_parts == nshards) {
        DfxCheck(dfx_store_load(ctxs[l], ModelNamePart(P.model_in, it, ex->rank(l)).c_str()),
                 "dfx_store_load");
      } else {  // saved by a different number of servers: keep the keys this shard owns
        for (int r = 0; r < P.model_in_parts; ++r)
          DfxCheck(dfx_store_load_part(ctxs[l], ModelNamePart(P.model_in, it, r).c_str(),
                                       ex->rank(l), nshards),
                   "dfx_store_load_part");
      }
    }
  }
  {
    GpuShardedStore store(ex.get(), P.pipelined);
    std::vector<std::vector<DevBatch>> dev(nlocal);
    for (auto& v : dev) v.resize(3);
    int ring = 0;
    const double t0 = Now();
    double pre_loss = 0;
    for (int k = std::max(0, P.load_epoch > 0 ? P.load_epoch + 1 : 0); k < P.max_num_epochs; ++k) {
      const double te = Now();
      for (int job = 0; job < P.num_jobs_per_epoch; ++job) {
        // shard r reads part job * nshards + r of num_jobs_per_epoch * nshards
        const int nparts = P.num_jobs_per_epoch * nshards;
        std::vector<std::unique_ptr<ThreadedBatchReader>> rd(nlocal);
        for (int l = 0; l < nlocal; ++l)
          rd[l].reset(new ThreadedBatchReader(P.data_in, P.data_format,
                                              job * nshards + ex->rank(l), nparts, P.batch_size,
                                              P.batch_size * P.shuffle, P.neg_sampling,
                                              P.nthreads));
        std::vector<bool> more(nlocal, true);
        for (;;) {
          std::vector<dfx_batch> bs(nlocal);
          std::vector<double> any(1, 0.0);
          for (int l = 0; l < nlocal; ++l) {
            if (more[l]) more[l] = rd[l]->Next();
            if (more[l]) any[0] += 1;
          }
          ex->AllReduceSum(&any);
          bool local_any = false;
          for (int l = 0; l < nlocal; ++l) local_any = local_any || more[l];
          if (any[0] == 0 && !local_any) break;
          for (int l = 0; l < nlocal; ++l) {
            DevBatch& db = dev[l][ring];
            db.Upload(ctxs[l], more[l] ? &rd[l]->Value() : nullptr);
            bs[l] = db.b;
          }
          ring = (ring + 1) % 3;
          store.Submit(bs, GpuSGDLearner::kTraining, k == 0);
        }
      }
      store.Flush();
      std::vector<double> pr(3, 0.0);
      for (int l = 0; l < nlocal; ++l) {
        dfx_progress p;
        DfxCheck(dfx_progress_read(ctxs[l], &p, 1), "dfx_progress_read");
        pr[0] += p.nrows;
        pr[1] += p.loss;
        pr[2] += p.auc;
      }
      ex->AllReduceSum(&pr);
      Progress tr;
      tr.nrows = pr[0];
      tr.loss = pr[1];
      tr.auc = pr[2];
      const double dt = Now() - te;
      if (rank == 0)
        std::printf("Epoch[%d] Training: %s  (%.0f ex/s incl. parse+PCIe, %d shards, %.2f s)\n", k,
                    Text(tr).c_str(), tr.nrows / dt, nshards, Now() - t0);
      std::fflush(stdout);
      const double eps = std::fabs(tr.loss - pre_loss) / pre_loss;
      if (eps < P.stop_rel_objv) break;
      pre_loss = tr.loss;
    }
  }
  if (!P.model_out.empty())
    for (int l = 0; l < nlocal; ++l)
      DfxCheck(dfx_store_save(ctxs[l], ModelNamePart(P.model_out, -1, ex->rank(l)).c_str(),
                              P.has_aux ? 1 : 0),
               "dfx_store_save");
  ex.reset();
  for (auto c : ctxs) dfx_ctx_destroy(c);
  return 0;
}
}  // namespace

int main(int argc, char** argv) {
  Param P;
  KWArgs rest;
  bool fused_given = false;
  for (int i = 1; i < argc; ++i) {
    const char* eq = std::strchr(argv[i], '=');
    if (!eq) {
      std::fprintf(stderr, "argument '%s' is not key=value\n", argv[i]);
      return 2;
    }
    const std::string k(argv[i], eq - argv[i]), v(eq + 1);
    if (k == "data_in") P.data_in = v;
    else if (k == "data_val") P.data_val = v;
    else if (k == "data_format") P.data_format = v;
    else if (k == "model_in") P.model_in = v;
    else if (k == "model_out") P.model_out = v;
    else if (k == "batch_size") P.batch_size = std::stoul(v);
    else if (k == "shuffle") P.shuffle = std::stoul(v);
    else if (k == "neg_sampling") P.neg_sampling = std::stof(v);
    else if (k == "max_num_epochs") P.max_num_epochs = std::stoi(v);
    else if (k == "num_jobs_per_epoch") P.num_jobs_per_epoch = std::stoi(v);
    else if (k == "stop_rel_objv") P.stop_rel_objv = std::stod(v);
    else if (k == "nthreads") P.nthreads = std::stoi(v);
    else if (k == "load_epoch") P.load_epoch = std::stoi(v);
    else if (k == "task") P.task = std::stoi(v);
    else if (k == "pred_out") P.pred_out = v;
    else if (k == "pred_prob") P.pred_prob = std::stoi(v) != 0;
    else if (k == "has_aux") P.has_aux = std::stoi(v) != 0;
    else if (k == "shards") P.shards = std::stoi(v);
    else if (k == "pipelined") P.pipelined = std::stoi(v) != 0;
    else if (k == "exchange") P.exchange = v;
    else if (k == "model_in_parts") P.model_in_parts = std::stoi(v);
    else {
      fused_given = fused_given || k == "fused";
      rest.push_back({k, v});
    }
  }
  if (P.data_in.empty() && P.task != 2) {
    std::fprintf(stderr, "usage: %s data_in=FILE [key=value ...]\n", argv[0]);
    return 2;
  }
  const char* ws = std::getenv("WORLD_SIZE");
  if (P.shards != 0 || (ws && std::atoi(ws) > 1)) return RunSharded(P, rest);
  if (!fused_given) rest.push_back({"fused", "1"});
  GpuSGDLearner learner(rest);
  int k0 = 0;
  if (!P.model_in.empty()) {  // sgd_learner.cc:58-67
    FileStream fi(ModelName(P.model_in, P.load_epoch > 0 ? P.load_epoch : -1).c_str(), "rb");
    learner.updater()->Load(&fi);
    if (P.load_epoch > 0) k0 = P.load_epoch + 1;
  }
  if (P.task == 2) {  // prediction, sgd_learner.cc:69-77
    if (P.model_in.empty() || P.data_val.empty()) {
      std::fprintf(stderr, "prediction needs model_in and data_val\n");
      return 2;
    }
    FILE* pf = nullptr;
    if (!P.pred_out.empty()) {
      pf = std::fopen((P.pred_out + "_part-0").c_str(), "w");
      if (!pf) {
        std::fprintf(stderr, "cannot open %s_part-0\n", P.pred_out.c_str());
        return 1;
      }
    }
    const Progress pr = RunEpoch(&learner, P, k0, GpuSGDLearner::kPrediction, pf);
    if (pf) std::fclose(pf);
    std::printf("Prediction: %s\n", Text(pr).c_str());
    return 0;
  }
  const double t0 = Now();
  double pre_loss = 0, pre_val_auc = 0;  // sgd_learner.cc:52
  for (int k = k0; k < P.max_num_epochs; ++k) {
    const double te = Now();
    const Progress tr = RunEpoch(&learner, P, k, GpuSGDLearner::kTraining);
    const double dt = Now() - te;
    std::printf("Epoch[%d] Training: %s  (%.0f ex/s incl. parse+PCIe, %.2f s)\n", k,
                Text(tr).c_str(), tr.nrows / dt, Now() - t0);
    Progress va;
    if (!P.data_val.empty()) {
      va = RunEpoch(&learner, P, k, GpuSGDLearner::kValidation);
      std::printf("Epoch[%d] Validation: %s\n", k, Text(va).c_str());
    }
    std::fflush(stdout);
    // stop criteria, sgd_learner.cc:89-108
    double eps = std::fabs(tr.loss - pre_loss) / pre_loss;
    if (eps < P.stop_rel_objv) {
      std::printf("Change of loss [%g] < stop_rel_objv [%g]\n", eps, P.stop_rel_objv);
      break;
    }
    if (va.auc > 0) {
      eps = (va.auc - pre_val_auc) / va.nrows;
      if (eps < 1e-5) break;
    }
    pre_loss = tr.loss;
    pre_val_auc = va.auc;
  }
  if (!P.model_out.empty()) {  // sgd_learner.cc:116-120
    FileStream fo(ModelName(P.model_out, -1).c_str(), "wb");
    learner.updater()->Save(P.has_aux, &fo);
  }
  return 0;
}
