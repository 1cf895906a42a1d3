// am.cc -- AcousticModel on the GPU (reference src/am.cc:26-164).
#include "am.h"

#include <assert.h>
#include <string.h>

#include <memory>

namespace pocketkaldi {

using catears::host::Check;
using catears::host::Runtime;

AcousticModel::AcousticModel() {}

AcousticModel::~AcousticModel() {
  if (model_) ce_gpu_model_destroy(model_);
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
  int pdfs = 0;
  ce_gpu_model_info(model_, nullptr, nullptr, nullptr, &pdfs, nullptr, nullptr);
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  float *d_in = static_cast<float *>(rt.scratch(0).Reserve(sizeof(float) * (size_t)rows_in * dim));
  float *d_out = static_cast<float *>(rt.scratch(1).Reserve(sizeof(float) * (size_t)batch_size * pdfs));
  rt.Upload(d_in, dim, inst->rows.data() + inst->head * dim, dim, sizeof(float), rows_in, dim);
  // Nnet::Propagate + row -= log_prior (src/am.cc:104-112), fused
  Check(ce_gpu_nnet_propagate(rt.ctx(), model_, d_in, rows_in, dim, 1, d_out), "AcousticModel::ComputeBatch");
  log_prob->Resize(batch_size, pdfs, Matrix<float>::kUndefined);
  rt.Download(log_prob->Data(), log_prob->Stride(), d_out, pdfs, sizeof(float), batch_size, pdfs);
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
