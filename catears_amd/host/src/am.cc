// am.cc -- AcousticModel on the GPU (reference src/am.cc:26-164).
#include "am.h"

#include <assert.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>

namespace pocketkaldi {

using catears::host::Check;
using catears::host::Runtime;

// Leader/follower batching of ready chunks across Instances: whoever finds
// no batch in progress leads -- waits for up to `max_blocks` requests or
// `wait`, runs them as one device call, marks them done; a request left
// behind by a finished batch makes its owner the next leader.
struct AcousticModel::Batcher {
  struct Req {
    Req(const float *r, int n_, int d, Matrix<float> *o) : rows(r), n(n_), dim(d), out(o), done(false) {}
    const float *rows;
    int n, dim;
    Matrix<float> *out;
    bool done;
    std::exception_ptr error;  // the batch's failure, rethrown by the request's owner
  };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Req *> pending;
  bool leader_active = false;
  int max_blocks = 1;
  std::chrono::microseconds wait{200};
  int64_t calls = 0, blocks = 0;
};

AcousticModel::AcousticModel() {}

AcousticModel::~AcousticModel() {
  if (model_) ce_gpu_model_destroy(model_);
}

void AcousticModel::batch_stats(int64_t *calls, int64_t *blocks) const {
  if (!batcher_) {
    *calls = *blocks = 0;
    return;
  }
  std::lock_guard<std::mutex> lk(batcher_->mu);
  *calls = batcher_->calls;
  *blocks = batcher_->blocks;
}

Status AcousticModel::Read(const Configuration &conf) {
  // Same key order and error paths as src/am.cc:26-64.
  std::string nnet_file, prior_file, tid2pdf_file;
  PK_CHECK_STATUS(conf.GetPath("nnet", &nnet_file));
  Nnet nnet;
  {
    util::ReadableFile fd;
    PK_CHECK_STATUS(fd.Open(nnet_file));
    PK_CHECK_STATUS(nnet.Read(&fd));
  }
  Vector<float> prior;
  PK_CHECK_STATUS(conf.GetPath("prior", &prior_file));
  {
    util::ReadableFile fd;
    PK_CHECK_STATUS(fd.Open(prior_file));
    PK_CHECK_STATUS(prior.Read(&fd));
  }
  PK_CHECK_STATUS(conf.GetInteger("left_context", &left_context_));
  PK_CHECK_STATUS(conf.GetInteger("right_context", &right_context_));
  PK_CHECK_STATUS(conf.GetInteger("chunk_size", &chunk_size_));
  PK_CHECK_STATUS(conf.GetInteger("num_pdfs", &num_pdfs_));
  PK_CHECK_STATUS(conf.GetPath("tid2pdf", &tid2pdf_file));
  {
    util::ReadableFile fd;
    PK_CHECK_STATUS(fd.Open(tid2pdf_file));
    PK_CHECK_STATUS(tid2pdf_.Read(&fd));
  }

  // Upload the network + log prior as one fused device program.  The
  // config's context must be the network's (the reference would assert on
  // the first batch otherwise, src/am.cc:104).
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  if (model_) ce_gpu_model_destroy(model_);
  model_ = nullptr;
  const int rc = ce_gpu_model_load_mem(rt.ctx(), nnet.image().data(), (int64_t)nnet.image().size(), prior.Data(),
                                       prior.Dim(), left_context_, right_context_, &model_);
  if (rc == CE_GPU_ENOTSUP)
    return Status::NotImplemented(util::Format("{}: {}", nnet_file, ce_gpu_last_error()));
  if (rc != CE_GPU_OK) return Status::Corruption(util::Format("{}: {}", nnet_file, ce_gpu_last_error()));
  int pdfs = 0;
  ce_gpu_model_info(model_, nullptr, nullptr, &feat_dim_, &pdfs, nullptr, nullptr);
  // streaming chunks are small row blocks: latency mode (split-K GEMMs,
  // ce_gpu_ctx_set_latency) unless the config turns it off.  The flag is this
  // model's: RunBlocks sets it on the shared context for each of its calls,
  // so models loaded later with another setting do not change it.
  latency_ = conf.GetIntegerOrElse("gpu_latency_mode", 1) ? 1 : 0;
  batcher_.reset(new Batcher());
  batcher_->max_blocks = conf.GetIntegerOrElse("gpu_batch_streams", 1);
  batcher_->wait = std::chrono::microseconds(conf.GetIntegerOrElse("gpu_batch_wait_us", 200));
  return Status::OK();
}

void AcousticModel::Append(Instance *inst, const float *frame, int dim) const {
  assert((inst->dim == 0 || inst->dim == dim) && "AcousticModel: feature width changed");
  inst->dim = dim;
  if (inst->head > 0 && inst->head * 2 >= inst->rows.size() / dim) {  // compact the consumed prefix
    inst->rows.erase(inst->rows.begin(), inst->rows.begin() + inst->head * dim);
    inst->head = 0;
  }
  inst->rows.insert(inst->rows.end(), frame, frame + dim);
}

void AcousticModel::ComputeBatch(Instance *inst, int batch_size, Matrix<float> *log_prob) const {
  const int L = left_context_, R = right_context_;
  if (batch_size == kBatchSizeAll) {
    batch_size = (int)inst->size() - L - R;
    assert(batch_size > 0 && "ComputeBatch: insufficient data");
  }
  if (batch_size == 0) {
    log_prob->Resize(0, log_prob->NumCols());
    return;
  }
  const int rows_in = batch_size + L + R;
  assert((int)inst->size() >= rows_in && "ComputeBatch: insufficient data");
  const int dim = inst->dim;
  if (dim != feat_dim_) throw catears::host::DeviceError("AcousticModel: feature width differs from the nnet input");
  const float *rows = inst->rows.data() + inst->head * dim;
  if (batcher_ && batcher_->max_blocks > 1) {
    Batcher &b = *batcher_;
    Batcher::Req req(rows, rows_in, dim, log_prob);
    std::unique_lock<std::mutex> lk(b.mu);
    b.pending.push_back(&req);
    b.cv.notify_all();
    while (!req.done) {
      if (!b.leader_active) {
        b.leader_active = true;
        b.cv.wait_for(lk, b.wait, [&] { return (int)b.pending.size() >= b.max_blocks; });
        std::vector<Batcher::Req *> batch;
        batch.swap(b.pending);
        lk.unlock();
        std::vector<const float *> ptrs;
        std::vector<int32_t> ns;
        std::vector<Matrix<float> *> outs;
        for (Batcher::Req *q : batch) ptrs.push_back(q->rows), ns.push_back(q->n), outs.push_back(q->out);
        // A device failure must still release the followers: every request
        // of the batch is finished with the error, which its owner rethrows.
        std::exception_ptr error;
        try {
          RunBlocks(ptrs, ns, dim, outs);
        } catch (...) {
          error = std::current_exception();
        }
        lk.lock();
        for (Batcher::Req *q : batch) q->done = true, q->error = error;
        b.calls += 1;
        b.blocks += (int64_t)batch.size();
        b.leader_active = false;
        b.cv.notify_all();
      } else {
        b.cv.wait(lk, [&] { return req.done || !b.leader_active; });
      }
    }
    if (req.error) std::rethrow_exception(req.error);
    return;
  }
  RunBlocks({rows}, {rows_in}, dim, {log_prob});
  if (batcher_) {
    std::lock_guard<std::mutex> lk(batcher_->mu);
    batcher_->calls += 1;
    batcher_->blocks += 1;
  }
}

// Uploads the blocks back to back, scores them in one device call
// (Nnet::Propagate + row -= log_prior, src/am.cc:104-112), hands each block's
// rows - L - R output rows to its matrix.
void AcousticModel::RunBlocks(const std::vector<const float *> &rows, const std::vector<int32_t> &n, int dim,
                              const std::vector<Matrix<float> *> &out) const {
  int pdfs = 0;
  ce_gpu_model_info(model_, nullptr, nullptr, nullptr, &pdfs, nullptr, nullptr);
  const int ctx_rows = left_context_ + right_context_;
  size_t in_rows = 0, out_rows = 0;
  for (int32_t k : n) in_rows += k, out_rows += k - ctx_rows;
  // a lane of its own: calls from other threads run on other lanes
  Runtime::Lease lane = Runtime::Get().Acquire();
  float *d_in = static_cast<float *>(lane.scratch(0).Reserve(sizeof(float) * in_rows * dim));
  float *d_out = static_cast<float *>(lane.scratch(1).Reserve(sizeof(float) * out_rows * pdfs));
  size_t at = 0;
  for (size_t b = 0; b < rows.size(); ++b) {
    lane.Upload(d_in + at * dim, dim, rows[b], dim, sizeof(float), n[b], dim);
    at += n[b];
  }
  Check(ce_gpu_ctx_set_latency(lane.ctx(), latency_), "AcousticModel::ComputeBatch");
  if (rows.size() == 1)
    Check(ce_gpu_nnet_propagate(lane.ctx(), model_, d_in, n[0], dim, 1, d_out), "AcousticModel::ComputeBatch");
  else
    Check(ce_gpu_nnet_propagate_blocks(lane.ctx(), model_, d_in, dim, n.data(), (int)n.size(), 1, d_out),
          "AcousticModel::ComputeBatch");
  at = 0;
  for (size_t b = 0; b < rows.size(); ++b) {
    const int m = n[b] - ctx_rows;
    out[b]->Resize(m, pdfs, Matrix<float>::kUndefined);
    lane.Download(out[b]->Data(), out[b]->Stride(), d_out + at * pdfs, pdfs, sizeof(float), m, pdfs);
    at += m;
  }
}

void AcousticModel::Process(Instance *inst, const VectorBase<float> &frame_feat, Matrix<float> *log_prob) const {
  if (!inst->started) {  // L copies of the first frame (src/am.cc:118-124)
    for (int i = 0; i < left_context_; ++i) Append(inst, frame_feat.Data(), frame_feat.Dim());
    inst->started = true;
  }
  Append(inst, frame_feat.Data(), frame_feat.Dim());
  if ((int)inst->size() < left_context_ + right_context_ + chunk_size_) {
    log_prob->Resize(0, 0);
    return;
  }
  ComputeBatch(inst, chunk_size_, log_prob);
  inst->head += chunk_size_;
}

void AcousticModel::EndOfStream(Instance *inst, Matrix<float> *log_prob) const {
  if (inst->size() == 0) {
    log_prob->Resize(0, 0);
    return;
  }
  // R copies of the last frame (src/am.cc:151-155)
  std::vector<float> last(inst->rows.end() - inst->dim, inst->rows.end());
  for (int i = 0; i < right_context_; ++i) Append(inst, last.data(), inst->dim);
  if ((int)inst->size() <= left_context_ + right_context_) {
    log_prob->Resize(0, 0);
    return;
  }
  ComputeBatch(inst, kBatchSizeAll, log_prob);
}

}  // namespace pocketkaldi
