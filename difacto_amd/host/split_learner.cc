// split_learner.cc — see split_learner.h.  Host code over the C-ABIs (libdifacto_amd.so's
// contexts and feeders, libdfx_dist.so's split driver); no HIP headers.
#include "split_learner.h"

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>

#include "../../include/difacto_amd_dist.h"
#include "dist_host.h"

namespace difacto {

namespace {

void DistCheck(int status, const char* what) {
  DFX_HOST_CHECK(status == DFX_OK, std::string(what) + ": " + dfx_dist_last_error());
}

}  // namespace

struct GpuSplitLearner::Impl {
  std::vector<dfx_ctx*> ctxs;  // owned
  dfx_split_store* store = nullptr;
  int N = 1, L = 1, rank0 = 0;
  bool pipelined = true;
  std::vector<dfx_feeder*> feeders;
  int64_t cap_rows = 0, cap_nnz = 0;
  int64_t submits = 0;
  bool queued = false;  // a pipelined step is waiting for the next submit (or Flush)

  // the step being assembled from the local workers' calls
  std::mutex mu;
  std::condition_variable cv;
  std::vector<const dmlc::RowBlock<feaid_t>*> pend;
  std::vector<int> pend_job, pend_cnt;
  int arrived = 0;
  int64_t gen = 0;
  std::string failure;

  ~Impl() {
    if (store) (void)dfx_split_store_destroy(store);  // flushes and syncs the contexts
    for (dfx_feeder* f : feeders)
      if (f) (void)dfx_feeder_destroy(f);
    for (dfx_ctx* c : ctxs) (void)dfx_ctx_destroy(c);
  }

  // feeders with room for every pending batch (3 staging slots: a pipelined step reads its
  // batch until the submit after it)
  void Feeders() {
    int64_t rows = 0, nnz = 0;
    for (const auto* b : pend) {
      rows = std::max<int64_t>(rows, (int64_t)b->size);
      nnz = std::max<int64_t>(nnz, b->size ? (int64_t)b->offset[b->size] : 0);
    }
    if (!feeders.empty() && rows <= cap_rows && nnz <= cap_nnz) return;
    // grow: every queued step must be done with the old staging buffers first (the store's
    // sync also frees the step buffers it outgrew)
    if (store) DistCheck(dfx_split_store_sync(store), "dfx_split_store_sync");
    queued = false;
    for (dfx_ctx* c : ctxs) DfxCheck(dfx_sync(c), "dfx_sync");
    for (dfx_feeder* f : feeders) DfxCheck(dfx_feeder_destroy(f), "dfx_feeder_destroy");
    feeders.assign(L, nullptr);
    cap_rows = std::max<int64_t>(std::max<int64_t>(rows, 1), cap_rows + cap_rows / 2);
    cap_nnz = std::max<int64_t>(std::max<int64_t>(nnz, 1), cap_nnz + cap_nnz / 2);
    for (int l = 0; l < L; ++l)
      DfxCheck(dfx_feeder_create_slots(ctxs[l], cap_rows, cap_nnz, 3, &feeders[l]),
               "dfx_feeder_create_slots");
  }

  // the last local worker's call: every pending batch uploaded, one step submitted
  void Submit(int job, bool push_cnt) {
    Feeders();
    std::vector<dfx_batch> b(L);
    for (int l = 0; l < L; ++l) {
      const dmlc::RowBlock<feaid_t>& x = *pend[l];
      const int64_t B = (int64_t)x.size, nnz = B ? (int64_t)x.offset[B] : 0;
      DFX_HOST_CHECK(B == 0 || x.offset[0] == 0, "split learner: offset[0] must be 0");
      dfx_host_batch hb;
      DfxCheck(dfx_feeder_slot(feeders[l], &hb), "dfx_feeder_slot");
      static_assert(sizeof(size_t) == sizeof(uint64_t), "size_t offsets");
      if (B) {
        std::memcpy(hb.offset, x.offset, (B + 1) * 8);
      } else {
        hb.offset[0] = 0;
      }
      if (nnz) std::memcpy(hb.index, x.index, nnz * 8);
      if (nnz && x.value) std::memcpy(hb.value, x.value, nnz * 4);
      if (B) std::memcpy(hb.label, x.label, B * 4);
      if (B && x.weight) std::memcpy(hb.weight, x.weight, B * 4);
      DfxCheck(dfx_feeder_submit(feeders[l], B, nnz, x.value != nullptr && nnz > 0,
                                 x.weight != nullptr && B > 0, &b[l]),
               "dfx_feeder_submit");
    }
    DistCheck(dfx_split_store_submit(store, b.data(), job, push_cnt ? 1 : 0, nullptr),
              "dfx_split_store_submit");
    // a pipelined submit queued the previous step, the last reader of the previous batch
    for (int l = 0; l < L; ++l)
      DfxCheck(pipelined ? (queued ? dfx_feeder_consumed_back(feeders[l], 1) : DFX_OK)
                         : dfx_feeder_consumed(feeders[l]),
               "dfx_feeder_consumed");
    queued = pipelined;
    ++submits;
  }
};

namespace {

std::string CtxKw(const KWArgs& kw) {
  std::string s;
  for (const auto& p : kw) {
    if (!s.empty()) s += ",";
    s += p.first + "=" + p.second;
  }
  return s;
}

// the learner's own keys out of kwargs; the rest are every shard's context kwargs
std::unique_ptr<GpuSplitLearner::Impl> Parse(const KWArgs& kwargs, int* slices,
                                             std::string* ctx_kw) {
  std::unique_ptr<GpuSplitLearner::Impl> m(new GpuSplitLearner::Impl());
  KWArgs rest;
  std::string loss = "fm";
  *slices = 0;
  for (const auto& p : kwargs) {
    if (p.first == "pipelined") {
      m->pipelined = std::stoi(p.second) != 0;
    } else if (p.first == "slices") {
      *slices = std::stoi(p.second);
    } else if (p.first == "loss") {
      loss = p.second;
    } else if (p.first == "push_agg") {
      DFX_HOST_CHECK(p.second == "sum", "the split step is push_agg=sum (one Update per key)");
    } else {
      rest.push_back(p);
    }
  }
  DFX_HOST_CHECK(loss == "fm" || loss == "logit", "unknown loss type " + loss);
  if (loss == "logit") rest.push_back({"loss", "logit"});
  rest.push_back({"push_agg", "sum"});
  *ctx_kw = CtxKw(rest);
  return m;
}

}  // namespace

std::shared_ptr<GpuSplitLearner> GpuSplitLearner::CreateLoopback(int nshards,
                                                                  const KWArgs& kwargs) {
  DFX_HOST_CHECK(nshards >= 1, "GpuSplitLearner: nshards >= 1");
  int slices = 0;
  std::string kw;
  std::unique_ptr<Impl> m = Parse(kwargs, &slices, &kw);
  m->N = m->L = nshards;
  m->ctxs.assign(nshards, nullptr);
  for (auto& c : m->ctxs) DfxCheck(dfx_ctx_create(0, kw.c_str(), &c), "dfx_ctx_create");
  DistCheck(dfx_split_store_create_loopback(m->ctxs.data(), nshards, m->pipelined ? 1 : 0,
                                            std::numeric_limits<uint64_t>::max(), &m->store),
            "dfx_split_store_create_loopback");
  if (slices) DistCheck(dfx_split_store_set_slices(m->store, slices), "set_slices");
  return std::shared_ptr<GpuSplitLearner>(new GpuSplitLearner(std::move(m)));
}

std::shared_ptr<GpuSplitLearner> GpuSplitLearner::CreateRccl(const KWArgs& kwargs) {
  const char* ws = std::getenv("WORLD_SIZE");
  const int world = ws ? std::atoi(ws) : 1;
  const int rank = std::getenv("RANK") ? std::atoi(std::getenv("RANK")) : 0;
  const int local = std::getenv("LOCAL_RANK") ? std::atoi(std::getenv("LOCAL_RANK")) : 0;
  int slices = 0;
  std::string kw;
  std::unique_ptr<Impl> m = Parse(kwargs, &slices, &kw);
  m->N = world;
  m->L = 1;
  m->rank0 = rank;
  m->ctxs.assign(1, nullptr);
  DfxCheck(dfx_ctx_create(local, kw.c_str(), &m->ctxs[0]), "dfx_ctx_create");
  // communicator ids: made by rank 0, handed over through the node-local id file
  const int nid = dfx_dist_rccl_comms();
  std::vector<char> ids((size_t)nid * dfx_dist_rccl_id_bytes());
  if (rank == 0) DistCheck(dfx_dist_rccl_ids(nid, ids.data()), "dfx_dist_rccl_ids");
  const std::string id_file = CommIdFile();
  ShareIdsThroughFile(rank, ids.data(), ids.size(), id_file);
  DistCheck(dfx_split_store_create_rccl(m->ctxs[0], rank, world, ids.data(), 0,
                                        m->pipelined ? 1 : 0,
                                        std::numeric_limits<uint64_t>::max(), &m->store),
            "dfx_split_store_create_rccl");
  // every rank holds its communicators now: the id file can go
  double one = 1;
  DistCheck(dfx_split_store_allreduce_sum(m->store, &one, 1), "allreduce");
  if (rank == 0) std::remove(id_file.c_str());
  if (slices) DistCheck(dfx_split_store_set_slices(m->store, slices), "set_slices");
  return std::shared_ptr<GpuSplitLearner>(new GpuSplitLearner(std::move(m)));
}

GpuSplitLearner::GpuSplitLearner(std::unique_ptr<Impl> impl) : impl_(std::move(impl)) {
  impl_->pend.assign(impl_->L, nullptr);
  impl_->pend_job.assign(impl_->L, 0);
  impl_->pend_cnt.assign(impl_->L, 0);
}

GpuSplitLearner::~GpuSplitLearner() {}

int GpuSplitLearner::nlocal() const { return impl_->L; }
int GpuSplitLearner::nranks() const { return impl_->N; }
int GpuSplitLearner::rank(int local) const { return impl_->rank0 + local; }
dfx_ctx* GpuSplitLearner::shard(int local) const { return impl_->ctxs.at(local); }

void GpuSplitLearner::ProcessBatch(int local, const dmlc::RowBlock<feaid_t>& batch, int job_type,
                                   bool push_cnt) {
  Impl& m = *impl_;
  DFX_HOST_CHECK(local >= 0 && local < m.L, "GpuSplitLearner: bad local worker");
  DFX_HOST_CHECK(job_type == kTraining || job_type == kValidation || job_type == kPrediction,
                 "GpuSplitLearner: bad job type");
  push_cnt = push_cnt && job_type == kTraining;
  std::unique_lock<std::mutex> lk(m.mu);
  DFX_HOST_CHECK(m.failure.empty(), "GpuSplitLearner: " + m.failure);
  DFX_HOST_CHECK(m.pend[local] == nullptr, "GpuSplitLearner: two batches of one worker in a step");
  m.pend[local] = &batch;
  m.pend_job[local] = job_type;
  m.pend_cnt[local] = push_cnt ? 1 : 0;
  const int64_t my_gen = m.gen;
  if (++m.arrived < m.L) {
    // the other local workers' batches complete the step; the last one submits it
    m.cv.wait(lk, [&]() { return m.gen != my_gen || !m.failure.empty(); });
    DFX_HOST_CHECK(m.failure.empty(), "GpuSplitLearner: " + m.failure);
    return;
  }
  for (int l = 0; l < m.L; ++l)
    if (m.pend_job[l] != job_type || m.pend_cnt[l] != (push_cnt ? 1 : 0))
      m.failure = "the local workers' calls of one step differ in job type or count push";
  if (m.failure.empty()) m.Submit(job_type, push_cnt);
  m.arrived = 0;
  for (auto& p : m.pend) p = nullptr;
  ++m.gen;
  m.cv.notify_all();
  DFX_HOST_CHECK(m.failure.empty(), "GpuSplitLearner: " + m.failure);
}

void GpuSplitLearner::ProcessBatches(const std::vector<const dmlc::RowBlock<feaid_t>*>& batches,
                                     int job_type, bool push_cnt) {
  Impl& m = *impl_;
  DFX_HOST_CHECK((int)batches.size() == m.L, "GpuSplitLearner: one batch per local worker");
  DFX_HOST_CHECK(job_type == kTraining || job_type == kValidation || job_type == kPrediction,
                 "GpuSplitLearner: bad job type");
  std::lock_guard<std::mutex> lk(m.mu);
  DFX_HOST_CHECK(m.arrived == 0, "GpuSplitLearner: ProcessBatches beside ProcessBatch calls");
  for (int l = 0; l < m.L; ++l) m.pend[l] = batches[l];
  m.Submit(job_type, push_cnt && job_type == kTraining);
  for (auto& p : m.pend) p = nullptr;
}

void GpuSplitLearner::Flush() {
  Impl& m = *impl_;
  std::lock_guard<std::mutex> lk(m.mu);
  if (!m.queued) return;
  DistCheck(dfx_split_store_flush(m.store), "dfx_split_store_flush");
  for (dfx_feeder* f : m.feeders) DfxCheck(dfx_feeder_consumed(f), "dfx_feeder_consumed");
  m.queued = false;
}

Progress GpuSplitLearner::TakeProgress(int local) {
  Flush();
  dfx_progress p;
  DfxCheck(dfx_progress_read(shard(local), &p, 1), "dfx_progress_read");
  Progress out;
  out.nrows = p.nrows;
  out.loss = p.loss;
  out.auc = p.auc;
  return out;
}

void GpuSplitLearner::AllReduceSum(std::vector<double>* v) {
  DistCheck(dfx_split_store_allreduce_sum(impl_->store, v->data(), (int)v->size()),
            "dfx_split_store_allreduce_sum");
}

}  // namespace difacto
