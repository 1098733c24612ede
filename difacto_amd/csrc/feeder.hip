// Batch feeder: host RowBlocks -> device batches through pinned staging buffers and a loader
// stream, double-buffered (or more slots: dfx_feeder_create_slots).  The reader fills a slot's pinned arrays (parsing straight into
// them), dfx_feeder_submit enqueues the host->device copies on the loader stream, which is the
// context's input stream, so the Localizer lane of dfx_train_step waits only for the copy of
// its own batch — batch t+1's upload runs while the GPU trains on batch t.  A slot is reused
// only after the context stream passed the step that consumed it (dfx_feeder_consumed).
// This is the host side of SGDLearner::IterateData's producer loop (sgd_learner.cc:289-314).
#include <vector>

#include "internal.h"

struct dfx_feeder {
  dfx_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  int64_t max_rows = 0, max_nnz = 0;
  struct Slot {
    uint64_t *h_off = nullptr, *h_idx = nullptr;
    float *h_val = nullptr, *h_lab = nullptr, *h_wt = nullptr;
    uint64_t *d_off = nullptr, *d_idx = nullptr;
    float *d_val = nullptr, *d_lab = nullptr, *d_wt = nullptr;
    hipEvent_t consumed = nullptr;
  };
  std::vector<Slot> slot;
  int cur = -1;
};

using namespace dfx;

extern "C" int dfx_feeder_destroy(dfx_feeder* f) {
  if (!f) return DFX_OK;
  if (f->stream) (void)hipStreamSynchronize(f->stream);
  (void)hipDeviceSynchronize();
  for (auto& s : f->slot) {
    for (void* p : {(void*)s.h_off, (void*)s.h_idx, (void*)s.h_val, (void*)s.h_lab,
                    (void*)s.h_wt})
      if (p) (void)hipHostFree(p);
    for (void* p : {(void*)s.d_off, (void*)s.d_idx, (void*)s.d_val, (void*)s.d_lab,
                    (void*)s.d_wt})
      if (p) (void)hipFree(p);
    if (s.consumed) (void)hipEventDestroy(s.consumed);
  }
  if (f->ctx) (void)dfx_ctx_set_input_stream(f->ctx, nullptr);
  if (f->stream) (void)hipStreamDestroy(f->stream);
  delete f;
  return DFX_OK;
}

extern "C" int dfx_feeder_create_slots(dfx_ctx* ctx, int64_t max_rows, int64_t max_nnz,
                                       int nslots, dfx_feeder** out) {
  DFX_CHECK_ARG(ctx && out && max_rows > 0 && max_nnz >= 0 && nslots >= 2 && nslots <= 8,
                "feeder_create: bad argument");
  dfx_feeder* f = new dfx_feeder();
  f->slot.resize((size_t)nslots);
  f->ctx = ctx;
  f->max_rows = max_rows;
  f->max_nnz = max_nnz > 0 ? max_nnz : 1;
  auto fail = [&](const char* what) {
    set_error(std::string("feeder_create: ") + what);
    dfx_feeder_destroy(f);
    return DFX_ERR_HIP;
  };
  if (hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) != hipSuccess)
    return fail("stream");
  const size_t R = (size_t)max_rows, N = (size_t)f->max_nnz;
  for (auto& s : f->slot) {
    if (hipHostMalloc(&s.h_off, (R + 1) * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_idx, N * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_val, N * 4, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_lab, R * 4, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&s.h_wt, R * 4, hipHostMallocDefault) != hipSuccess)
      return fail("pinned host memory");
    if (hipMalloc(&s.d_off, (R + 1) * 8) != hipSuccess || hipMalloc(&s.d_idx, N * 8) != hipSuccess ||
        hipMalloc(&s.d_val, N * 4) != hipSuccess || hipMalloc(&s.d_lab, R * 4) != hipSuccess ||
        hipMalloc(&s.d_wt, R * 4) != hipSuccess)
      return fail("device memory");
    if (hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming) != hipSuccess)
      return fail("event");
  }
  int rc = dfx_ctx_set_input_stream(ctx, f->stream);
  if (rc != DFX_OK) {
    dfx_feeder_destroy(f);
    return rc;
  }
  *out = f;
  return DFX_OK;
}

extern "C" int dfx_feeder_create(dfx_ctx* ctx, int64_t max_rows, int64_t max_nnz,
                                 dfx_feeder** out) {
  return dfx_feeder_create_slots(ctx, max_rows, max_nnz, 2, out);
}

extern "C" int dfx_feeder_slot(dfx_feeder* f, dfx_host_batch* hb) {
  DFX_CHECK_ARG(f && hb, "feeder_slot: null argument");
  f->cur = (f->cur + 1) % (int)f->slot.size();
  auto& s = f->slot[f->cur];
  // the step that consumed this slot a round of slots ago must be past the device
  DFX_HIP(hipEventSynchronize(s.consumed));
  hb->offset = s.h_off;
  hb->index = s.h_idx;
  hb->value = s.h_val;
  hb->label = s.h_lab;
  hb->weight = s.h_wt;
  hb->max_rows = f->max_rows;
  hb->max_nnz = f->max_nnz;
  return DFX_OK;
}

extern "C" int dfx_feeder_submit(dfx_feeder* f, int64_t B, int64_t nnz, int has_value,
                                 int has_weight, dfx_batch* out) {
  DFX_CHECK_ARG(f && out, "feeder_submit: null argument");
  DFX_CHECK_ARG(B >= 0 && B <= f->max_rows && nnz >= 0 && nnz <= f->max_nnz,
                "feeder_submit: batch larger than the feeder's capacity");
  auto& s = f->slot[f->cur];
  DFX_CHECK_ARG(B == 0 || s.h_off[0] == 0, "feeder_submit: offset[0] must be 0");
  DFX_CHECK_ARG(B == 0 || (int64_t)s.h_off[B] == nnz, "feeder_submit: offset[B] != nnz");
  DFX_HIP(hipMemcpyAsync(s.d_off, s.h_off, (B + 1) * 8, hipMemcpyHostToDevice, f->stream));
  if (nnz) DFX_HIP(hipMemcpyAsync(s.d_idx, s.h_idx, nnz * 8, hipMemcpyHostToDevice, f->stream));
  if (has_value && nnz)
    DFX_HIP(hipMemcpyAsync(s.d_val, s.h_val, nnz * 4, hipMemcpyHostToDevice, f->stream));
  if (B) DFX_HIP(hipMemcpyAsync(s.d_lab, s.h_lab, B * 4, hipMemcpyHostToDevice, f->stream));
  if (has_weight && B)
    DFX_HIP(hipMemcpyAsync(s.d_wt, s.h_wt, B * 4, hipMemcpyHostToDevice, f->stream));
  out->size = B;
  out->nnz = nnz;
  out->offset = s.d_off;
  out->index = s.d_idx;
  out->value = has_value ? s.d_val : nullptr;
  out->label = s.d_lab;
  out->weight = has_weight ? s.d_wt : nullptr;
  return DFX_OK;
}

extern "C" int dfx_feeder_consumed(dfx_feeder* f) { return dfx_feeder_consumed_back(f, 0); }

extern "C" int dfx_feeder_consumed_back(dfx_feeder* f, int back) {
  const int n = f ? (int)f->slot.size() : 0;
  DFX_CHECK_ARG(f && back >= 0 && back < n && f->cur >= 0, "feeder_consumed: bad argument");
  DFX_HIP(hipEventRecord(f->slot[(f->cur - back + n) % n].consumed, f->ctx->c.stream));
  return DFX_OK;
}
