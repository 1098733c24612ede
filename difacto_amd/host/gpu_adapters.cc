// gpu_adapters.cc — see gpu_adapters.h.
#include "gpu_adapters.h"

#include <cstdlib>

#include <iterator>

#include "reader.h"

#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <set>
#include <sstream>
#include <thread>

namespace difacto {

void DfxCheck(int status, const char* what) {
  if (status == DFX_OK) return;
  std::fprintf(stderr, "[FATAL] %s failed (status %d): %s\n", what, status, dfx_last_error());
  std::abort();
}

static std::string KwString(const KWArgs& kw) {
  std::string s;
  for (const auto& p : kw) {
    if (!s.empty()) s += ",";
    s += p.first + "=" + p.second;
  }
  return s;
}

/** split kwargs into (known, rest) — dmlc::Parameter::InitAllowUnknown's contract */
static KWArgs Consume(const KWArgs& kw, const std::set<std::string>& known, KWArgs* mine) {
  KWArgs rest;
  for (const auto& p : kw) {
    if (known.count(p.first)) {
      mine->push_back(p);
    } else {
      rest.push_back(p);
    }
  }
  return rest;
}

GpuContext::GpuContext(int device, const KWArgs& kwargs) {
  DfxCheck(dfx_ctx_create(device, KwString(kwargs).c_str(), &h_), "dfx_ctx_create");
}

GpuContext::~GpuContext() {
  if (h_) dfx_ctx_destroy(h_);
}

// ---- Localizer ---------------------------------------------------------------------------
void GpuLocalizer::Compact(const dmlc::RowBlock<feaid_t>& blk,
                           RowBlockContainer<unsigned>* compacted,
                           std::vector<feaid_t>* uniq_idx, std::vector<real_t>* idx_frq) {
  dfx_ctx* c = ctx_->h();
  const size_t B = blk.size;
  const size_t nnz = B ? blk.offset[B] - blk.offset[0] : 0;
  DFX_HOST_CHECK(B == 0 || blk.offset[0] == 0, "Compact: offset[0] must be 0");
  if (B == 0) {
    if (uniq_idx) uniq_idx->clear();
    if (idx_frq) idx_frq->clear();
    *compacted = RowBlockContainer<unsigned>();
    return;
  }
  DevArray<uint64_t> offs(c), idx(c), uniq(c);
  DevArray<float> cnt(c);
  DevArray<uint32_t> col(c);
  offs.upload(reinterpret_cast<const uint64_t*>(blk.offset), B + 1);
  idx.upload(blk.index, nnz);
  uniq.ensure(nnz);
  col.ensure(nnz);
  if (idx_frq) cnt.ensure(nnz);
  int64_t U = 0;
  DfxCheck(dfx_localize(c, (int64_t)B, (int64_t)nnz, offs.get(), idx.get(), max_index_,
                        uniq.get(), idx_frq ? cnt.get() : nullptr, col.get(), &U),
           "dfx_localize");
  if (uniq_idx) {
    uniq_idx->resize(U);
    uniq.download(uniq_idx->data(), U);
  }
  if (idx_frq) {
    idx_frq->resize(U);
    cnt.download(idx_frq->data(), U);
  }
  // RemapIndex (localizer.cc:53-107): every index stays, only its column changes
  compacted->offset.assign(blk.offset, blk.offset + B + 1);
  compacted->label.assign(blk.label, blk.label ? blk.label + B : blk.label);
  compacted->weight.assign(blk.weight, blk.weight ? blk.weight + B : blk.weight);
  compacted->value.assign(blk.value, blk.value ? blk.value + nnz : blk.value);
  compacted->index.resize(nnz);
  col.download(compacted->index.data(), nnz);
  compacted->max_index = U ? (unsigned)(U - 1) : 0;
}

// ---- FMLoss ------------------------------------------------------------------------------
struct GpuFMLoss::Dev {
  explicit Dev(dfx_ctx* c)
      : offs(c), col(c), val(c), label(c), weight(c), W(c), pred(c), grad(c), wpos(c), vpos(c) {}
  DevArray<uint64_t> offs;
  DevArray<uint32_t> col;
  DevArray<float> val, label, weight, W, pred, grad;
  DevArray<int32_t> wpos, vpos;
  int64_t B = 0, nnz = 0, ncols = 0;
  const float* d_val = nullptr;
  const float* d_weight = nullptr;
  const int32_t* d_wpos = nullptr;
  const int32_t* d_vpos = nullptr;
};

KWArgs GpuFMLoss::Init(const KWArgs& kwargs) {
  KWArgs mine;
  // FMLossParam (fm_loss.h:19-27), plus the device this loss runs on
  KWArgs rest = Consume(kwargs, {"V_dim", "device"}, &mine);
  int device = 0;
  for (const auto& p : mine) {
    if (p.first == "V_dim") V_dim_ = std::stoi(p.second);
    if (p.first == "device") device = std::stoi(p.second);
  }
  if (logit_) V_dim_ = 0;
  DFX_HOST_CHECK(V_dim_ >= 0 && V_dim_ <= 1024, "V_dim out of range");
  // the loss needs a stream and scratch only: keep its (unused) model table tiny
  ctx_ = std::make_shared<GpuContext>(
      device, KWArgs{{"V_dim", std::to_string(V_dim_)}, {"max_keys", "16"}, {"max_vrows", "1"}});
  dev_ = std::make_shared<Dev>(ctx_->h());
  return rest;
}

void GpuFMLoss::Upload(const dmlc::RowBlock<unsigned>& data,
                       const std::vector<SArray<char>>& param) {
  DFX_HOST_CHECK(dev_ != nullptr, "GpuFMLoss: Init first");
  Dev& d = *dev_;
  d.B = (int64_t)data.size;
  d.nnz = d.B ? (int64_t)(data.offset[data.size] - data.offset[0]) : 0;
  DFX_HOST_CHECK(d.B == 0 || data.offset[0] == 0, "offset[0] must be 0");
  d.offs.upload(reinterpret_cast<const uint64_t*>(data.offset), d.B + 1);
  d.col.upload(data.index, d.nnz);
  d.d_val = d.val.upload(data.value, d.nnz);
  d.label.upload(data.label, d.B);
  d.d_weight = d.weight.upload(data.weight, d.B);
  SArray<real_t> W(param[0]);
  d.W.upload(W.data(), W.size());
  d.d_wpos = d.d_vpos = nullptr;
  d.ncols = (int64_t)W.size();
  if (param.size() > 1 && !param[1].empty()) {
    SArray<int> wp(param[1]);
    d.d_wpos = d.wpos.upload(wp.data(), wp.size());
    d.ncols = (int64_t)wp.size();
  }
  if (param.size() > 2 && !param[2].empty()) {
    SArray<int> vp(param[2]);
    d.d_vpos = d.vpos.upload(vp.data(), vp.size());
  }
  DFX_HOST_CHECK(V_dim_ == 0 || (d.d_wpos && d.d_vpos), "V_dim > 0 needs w_pos and V_pos");
}

void GpuFMLoss::Predict(const dmlc::RowBlock<unsigned>& data,
                        const std::vector<SArray<char>>& param, SArray<real_t>* pred) {
  DFX_HOST_CHECK(param.size() >= 1, "Predict: param = {weights, w_pos, V_pos}");
  DFX_HOST_CHECK(pred->size() == data.size, "Predict: pred must have one entry per row");
  Upload(data, param);
  Dev& d = *dev_;
  d.pred.upload(pred->data(), d.B);
  DfxCheck(dfx_fm_predict(ctx_->h(), d.B, d.nnz, d.offs.get(), d.col.get(), d.d_val, d.W.get(),
                          d.d_wpos, d.d_vpos, d.ncols, V_dim_, d.pred.get()),
           "dfx_fm_predict");
  d.pred.download(pred->data(), d.B);
}

real_t GpuFMLoss::Evaluate(dmlc::real_t const* label, const SArray<real_t>& pred) const {
  Dev& d = *dev_;
  d.label.upload(label, pred.size());
  d.pred.upload(pred.data(), pred.size());
  double objv = 0;
  DfxCheck(dfx_evaluate(ctx_->h(), (int64_t)pred.size(), d.label.get(), d.pred.get(), &objv),
           "dfx_evaluate");
  return (real_t)objv;
}

real_t GpuFMLoss::AUC(dmlc::real_t const* label, const SArray<real_t>& pred) const {
  Dev& d = *dev_;
  d.label.upload(label, pred.size());
  d.pred.upload(pred.data(), pred.size());
  double auc = 0;
  DfxCheck(dfx_auc(ctx_->h(), (int64_t)pred.size(), d.label.get(), d.pred.get(), &auc),
           "dfx_auc");
  return (real_t)auc;
}

void GpuFMLoss::CalcGrad(const dmlc::RowBlock<unsigned>& data,
                         const std::vector<SArray<char>>& param, SArray<real_t>* grad) {
  DFX_HOST_CHECK(param.size() == 4, "CalcGrad: param = {weights, w_pos, V_pos, pred}");
  Upload(data, param);
  Dev& d = *dev_;
  SArray<real_t> pred(param[3]);
  DFX_HOST_CHECK(pred.size() == data.size, "CalcGrad: pred size");
  d.pred.upload(pred.data(), d.B);
  d.grad.upload(grad->data(), grad->size());
  DfxCheck(dfx_fm_calcgrad(ctx_->h(), d.B, d.nnz, d.offs.get(), d.col.get(), d.d_val,
                           d.label.get(), d.d_weight, d.W.get(), d.d_wpos, d.d_vpos, d.ncols,
                           V_dim_, d.pred.get(), d.grad.get()),
           "dfx_fm_calcgrad");
  d.grad.download(grad->data(), grad->size());
}

// ---- SGDUpdater --------------------------------------------------------------------------
KWArgs GpuSGDUpdater::Init(const KWArgs& kwargs) {
  // SGDUpdaterParam (sgd_param.h:79-123) + the device store's sizing
  static const std::set<std::string> known = {
      "l1", "l2", "V_l2", "lr", "lr_beta", "V_lr", "V_lr_beta", "V_init_scale", "V_threshold",
      "V_dim", "l1_shrk", "seed", "max_keys", "max_vrows"};
  KWArgs mine;
  KWArgs rest = Consume(kwargs, known, &mine);
  ctx_ = std::make_shared<GpuContext>(0, mine);
  V_dim_ = ctx_->V_dim();
  return rest;
}

void GpuSGDUpdater::Get(const SArray<feaid_t>& fea_ids, int data_type, SArray<real_t>* data,
                        SArray<int>* data_offset) {
  DFX_HOST_CHECK(data_type == Store::kWeight, "Get: only kWeight");
  dfx_ctx* c = ctx_->h();
  const size_t n = fea_ids.size();
  DevArray<uint64_t> keys(c);
  DevArray<float> vals(c);
  DevArray<int32_t> lens(c);
  keys.upload(fea_ids.data(), n);
  vals.ensure(n * (1 + V_dim_));
  if (V_dim_ > 0) lens.ensure(n);
  int64_t nv = 0;
  DfxCheck(dfx_store_pull(c, keys.get(), (int64_t)n, vals.get(), V_dim_ > 0 ? lens.get() : nullptr,
                          &nv),
           "dfx_store_pull");
  data->resize(nv);
  vals.download(data->data(), nv);
  if (data_offset) {
    if (V_dim_ > 0) {
      data_offset->resize(n);
      lens.download(data_offset->data(), n);
    } else {
      data_offset->clear();
    }
  }
}

void GpuSGDUpdater::Update(const SArray<feaid_t>& fea_ids, int data_type,
                           const SArray<real_t>& data, const SArray<int>& data_offset) {
  dfx_ctx* c = ctx_->h();
  const size_t n = fea_ids.size();
  DevArray<uint64_t> keys(c);
  DevArray<float> vals(c);
  DevArray<int32_t> lens(c);
  keys.upload(fea_ids.data(), n);
  vals.upload(data.data(), data.size());
  const int32_t* dl = data_offset.empty() ? nullptr : lens.upload(data_offset.data(), n);
  DfxCheck(dfx_store_push(c, keys.get(), (int64_t)n, data_type, vals.get(),
                          (int64_t)data.size(), dl),
           "dfx_store_push");
  DfxCheck(dfx_sync(c), "dfx_sync");
}

std::string GpuSGDUpdater::Get_report() {
  int64_t nk = 0, nv = 0;
  double new_w = 0;
  uint32_t seed = 0;
  DfxCheck(dfx_store_stats(ctx_->h(), &nk, &nv, &new_w, &seed), "dfx_store_stats");
  std::ostringstream os;
  os << "new_w " << (new_w - last_new_w_);
  last_new_w_ = new_w;
  return os.str();
}

void GpuSGDUpdater::Evaluate(double* penalty, int64_t* nnz_w) const {
  DfxCheck(dfx_store_evaluate(ctx_->h(), penalty, nnz_w), "dfx_store_evaluate");
}

// The C-ABI writes / reads the reference's model formats by path; a Stream is bridged
// through a private temporary file.
void GpuSGDUpdater::CopyThroughFile(bool save, bool aux, bool reverse, Stream* s) const {
  char path[] = "/tmp/difacto_amd_modelXXXXXX";
  int fd = mkstemp(path);
  DFX_HOST_CHECK(fd >= 0, "mkstemp");
  close(fd);
  if (save) {
    if (reverse) {
      DfxCheck(dfx_store_dump(ctx_->h(), path, aux, 1), "dfx_store_dump");
    } else {
      DfxCheck(dfx_store_save(ctx_->h(), path, aux), "dfx_store_save");
    }
    std::ifstream in(path, std::ios::binary);
    std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    if (!buf.empty()) s->Write(buf.data(), buf.size());
  } else {
    std::ofstream out(path, std::ios::binary);
    char buf[1 << 16];
    size_t n;
    while ((n = s->Read(buf, sizeof(buf))) > 0) out.write(buf, (std::streamsize)n);
    out.close();
    DfxCheck(dfx_store_load(ctx_->h(), path), "dfx_store_load");
  }
  unlink(path);
}

void GpuSGDUpdater::Load(Stream* fi) { CopyThroughFile(false, false, false, fi); }

void GpuSGDUpdater::Save(bool save_aux, Stream* fo) const {
  CopyThroughFile(true, save_aux, false, fo);
}

void GpuSGDUpdater::Dump(bool dump_aux, bool need_reverse, Stream* fo) const {
  // dfx_store_dump takes need_reverse itself; route through the dump branch
  char path[] = "/tmp/difacto_amd_dumpXXXXXX";
  int fd = mkstemp(path);
  DFX_HOST_CHECK(fd >= 0, "mkstemp");
  close(fd);
  DfxCheck(dfx_store_dump(ctx_->h(), path, dump_aux, need_reverse), "dfx_store_dump");
  std::ifstream in(path, std::ios::binary);
  std::vector<char> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (!buf.empty()) fo->Write(buf.data(), buf.size());
  unlink(path);
}

// ---- Store -------------------------------------------------------------------------------
int StoreGPU::Push(const SArray<feaid_t>& fea_ids, int val_type, const SArray<real_t>& vals,
                   const SArray<int>& lens, const std::function<void()>& on_complete) {
  DFX_HOST_CHECK(updater_ != nullptr, "StoreGPU: SetUpdater first");
  updater_->Update(fea_ids, val_type, vals, lens);
  if (on_complete) on_complete();
  return time_++;
}

int StoreGPU::Pull(const SArray<feaid_t>& fea_ids, int val_type, SArray<real_t>* vals,
                   SArray<int>* lens, const std::function<void()>& on_complete) {
  DFX_HOST_CHECK(updater_ != nullptr, "StoreGPU: SetUpdater first");
  updater_->Get(fea_ids, val_type, vals, lens);
  if (on_complete) on_complete();
  return time_++;
}

// ---- learner -----------------------------------------------------------------------------
void GetPos(const SArray<int>& len, SArray<int>* w_pos, SArray<int>* V_pos) {
  const size_t n = len.size();
  w_pos->resize(n);
  V_pos->resize(n);
  int run = 0;
  for (size_t i = 0; i < n; ++i) {
    const int l = len[i];
    (*w_pos)[i] = l == 0 ? -1 : run;
    (*V_pos)[i] = l > 1 ? run + 1 : -1;
    run += l;
  }
}

// large host copies into pinned staging, split over a few threads (one thread's memcpy bandwidth
// would bound the host-side batch rate)
static void ParallelCopy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kSplit = 4 << 20;
  const int T = (int)std::min<size_t>(8, bytes / kSplit);
  if (T < 2) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    const size_t a = bytes * t / T, b = bytes * (t + 1) / T;
    th.emplace_back([=]() {
      std::memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, b - a);
    });
  }
  for (auto& x : th) x.join();
}

GpuSGDLearner::GpuSGDLearner(const KWArgs& kwargs, std::shared_ptr<Store> store) {
  KWArgs mine;
  KWArgs rest = Consume(kwargs, {"fused", "loss", "device"}, &mine);
  std::string loss = "fm";
  int device = -1;
  for (const auto& p : mine) {
    if (p.first == "fused") fused_ = std::stoi(p.second) != 0;
    if (p.first == "loss") loss = p.second;
    if (p.first == "device") device = std::stoi(p.second);
  }
  if (device < 0) {
    // under a distributed launch the store's shard is on LOCAL_RANK (CreateStore /
    // GpuDistStore::CreateRccl): the learner's Localizer and loss default to the same GPU
    const char* lr = std::getenv("LOCAL_RANK");
    device = (store && lr) ? std::atoi(lr) : 0;
  }
  DFX_HOST_CHECK(loss == "fm" || loss == "logit", "unknown loss type " + loss);
  if (store) {
    // a given Store (a GpuDistStore worker) holds the model on its servers: this worker runs
    // the interface path with a context of its own for the Localizer
    DFX_HOST_CHECK(!fused_, "a given Store runs the interface path (fused=0)");
    for (const auto& p : rest)
      if (p.first == "V_dim") V_dim_ = std::stoi(p.second);
    if (loss == "logit") V_dim_ = 0;
    store_ = store;
    loss_.reset(new GpuFMLoss(loss == "logit"));
    loss_->Init({{"V_dim", std::to_string(V_dim_)}, {"device", std::to_string(device)}});
    localizer_.reset(new GpuLocalizer(std::make_shared<GpuContext>(
        device, KWArgs{{"V_dim", std::to_string(V_dim_)}, {"max_keys", "16"},
                       {"max_vrows", "1"}})));
    return;
  }
  if (loss == "logit") rest.push_back({"loss", "logit"});
  updater_ = std::make_shared<GpuSGDUpdater>();
  rest = updater_->Init(rest);
  V_dim_ = updater_->V_dim();
  store_ = std::make_shared<StoreGPU>();
  store_->SetUpdater(updater_);
  if (!fused_) {
    // V_dim is forwarded to the loss (sgd_learner.cc:37)
    loss_.reset(new GpuFMLoss(loss == "logit"));
    loss_->Init({{"V_dim", std::to_string(V_dim_)}});
    localizer_.reset(new GpuLocalizer(updater_->context()));
  }
}

GpuSGDLearner::~GpuSGDLearner() {
  if (feeder_) dfx_feeder_destroy(feeder_);
}

void GpuSGDLearner::ProcessBatch(const dmlc::RowBlock<feaid_t>& batch, int job_type,
                                 bool push_cnt, std::vector<real_t>* pred_out) {
  push_cnt = push_cnt && job_type == kTraining && V_dim_ > 0;
  if (fused_) {
    const int64_t B = (int64_t)batch.size, nnz = B ? (int64_t)batch.offset[B] : 0;
    dfx_ctx* c = updater_->context()->h();
    if (!feeder_ || B > feed_rows_ || nnz > feed_nnz_) {
      if (feeder_) {
        DfxCheck(dfx_sync(c), "dfx_sync");
        dfx_feeder_destroy(feeder_);
      }
      feed_rows_ = std::max<int64_t>(B, feed_rows_);
      feed_nnz_ = std::max<int64_t>(nnz, feed_nnz_);
      DfxCheck(dfx_feeder_create(c, feed_rows_, feed_nnz_, &feeder_), "dfx_feeder_create");
    }
    dfx_host_batch hb;
    DfxCheck(dfx_feeder_slot(feeder_, &hb), "dfx_feeder_slot");
    static_assert(sizeof(size_t) == sizeof(uint64_t), "size_t offsets");
    std::memcpy(hb.offset, batch.offset, (B + 1) * 8);
    ParallelCopy(hb.index, batch.index, nnz * 8);
    if (batch.value) ParallelCopy(hb.value, batch.value, nnz * 4);
    std::memcpy(hb.label, batch.label, B * 4);
    if (batch.weight) std::memcpy(hb.weight, batch.weight, B * 4);
    dfx_batch b;
    DfxCheck(dfx_feeder_submit(feeder_, B, nnz, batch.value != nullptr, batch.weight != nullptr,
                               &b),
             "dfx_feeder_submit");
    float* dp = nullptr;
    if (pred_out) {
      if (!dpred_) dpred_.reset(new DevArray<float>(c));
      dpred_->ensure(B);
      dp = dpred_->get();
    }
    DfxCheck(dfx_train_step(c, &b, job_type, push_cnt ? 1 : 0,
                            std::numeric_limits<uint64_t>::max(), dp),
             "dfx_train_step");
    DfxCheck(dfx_feeder_consumed(feeder_), "dfx_feeder_consumed");
    if (pred_out) {
      pred_out->resize(B);
      dpred_->download(pred_out->data(), B);
    }
    return;
  }
  // the executor lambda of IterateData, through the plugin interfaces
  RowBlockContainer<unsigned> data;
  auto feaids = std::make_shared<std::vector<feaid_t>>();
  auto feacnt = std::make_shared<std::vector<real_t>>();
  localizer_->Compact(batch, &data, feaids.get(), push_cnt ? feacnt.get() : nullptr);
  SArray<feaid_t> keys(feaids);
  if (push_cnt) store_->Wait(store_->Push(keys, Store::kFeaCount, SArray<real_t>(feacnt), {}));
  SArray<real_t> values;
  SArray<int> lengths;
  // (a StoreGPU pull completes inline; a GpuDistStore pull when its round has run)
  store_->Wait(store_->Pull(keys, Store::kWeight, &values, V_dim_ > 0 ? &lengths : nullptr));
  dmlc::RowBlock<unsigned> blk = data.GetBlock();
  if (blk.size == 0) {
    // a worker with no rows this round (the sharded store's workers call in step): it takes
    // part in the exchanges with no keys
    if (job_type == kTraining)
      store_->Wait(store_->Push(keys, Store::kGradient, SArray<real_t>(), SArray<int>()));
    return;
  }
  prog_.nrows += blk.size;
  SArray<real_t> pred(blk.size);
  SArray<int> w_pos, V_pos;
  if (V_dim_ > 0) GetPos(lengths, &w_pos, &V_pos);
  std::vector<SArray<char>> inputs = {SArray<char>(values), SArray<char>(w_pos),
                                      SArray<char>(V_pos)};
  loss_->Predict(blk, inputs, &pred);
  if (pred_out) pred_out->assign(pred.data(), pred.data() + pred.size());
  prog_.loss += loss_->Evaluate(blk.label, pred);
  prog_.auc += loss_->AUC(blk.label, pred);
  if (job_type == kTraining) {
    SArray<real_t> grads(values.size());
    inputs.push_back(SArray<char>(pred));
    loss_->CalcGrad(blk, inputs, &grads);
    // the batch is done once its update is applied (sgd_learner.cc:255-259, on_complete): a
    // caller may read the store's shards (save, progress) right after ProcessBatch returns
    store_->Wait(store_->Push(keys, Store::kGradient, grads, V_dim_ > 0 ? lengths : SArray<int>()));
  }
}

Progress GpuSGDLearner::TakeProgress() {
  Progress out = prog_;
  prog_ = Progress();
  if (fused_) {
    dfx_progress p;
    DfxCheck(dfx_progress_read(updater_->context()->h(), &p, 1), "dfx_progress_read");
    out.nrows += p.nrows;
    out.loss += p.loss;
    out.auc += p.auc;
  }
  return out;
}

// ---- reader ------------------------------------------------------------------------------
bool ReadLibSVM(const std::string& path, RowBlockContainer<feaid_t>* out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return false;
  const std::string text((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  *out = RowBlockContainer<feaid_t>();
  ParseLibSVM(text.data(), text.data() + text.size(), out);
  bool all_one = true;
  for (float v : out->value) all_one = all_one && v == 1.f;
  if (all_one) out->value.clear();  // binary data (batch_reader.cc:71-73)
  return true;
}

RowSlice Slice(const RowBlockContainer<feaid_t>& c, size_t begin, size_t end) {
  RowSlice s;
  const size_t o0 = c.offset[begin];
  for (size_t i = begin; i <= end; ++i) s.offs.push_back(c.offset[i] - o0);
  s.blk.size = end - begin;
  s.blk.offset = s.offs.data();
  s.blk.label = c.label.data() + begin;
  s.blk.weight = c.weight.empty() ? nullptr : c.weight.data() + begin;
  s.blk.index = c.index.data() + o0;
  s.blk.value = c.value.empty() ? nullptr : c.value.data() + o0;
  return s;
}

}  // namespace difacto
