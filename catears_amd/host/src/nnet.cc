// nnet.cc -- the pocketkaldi layer stack on the GPU (reference
// src/nnet.cc:22-307).  Host side: NN02 parsing with the reference's error
// strings and an NN02 image of what was read.  Device side: a fused program
// (ce_gpu_nnet_propagate) for converter-shaped networks, single-layer ops
// (ce_gpu_linear / ce_gpu_splice / ce_gpu_rowwise / D2D copies) otherwise.
#include "nnet.h"

#include <assert.h>
#include <string.h>

namespace pocketkaldi {

using catears::host::Check;
using catears::host::DeviceMatrix;
using catears::host::Runtime;

namespace {

// ---- NN02 image writer (the byte layout Nnet::Read consumes) ----
void put_bytes(std::string *s, const void *p, size_t n) { s->append(static_cast<const char *>(p), n); }
void put_i32(std::string *s, int32_t v) { put_bytes(s, &v, 4); }
void put_vec(std::string *s, const float *v, int n) {  // VEC0, src/vector.cc:267-300
  put_bytes(s, "VEC0", 4);
  put_i32(s, 4 * n + 4);
  put_i32(s, n);
  put_bytes(s, v, sizeof(float) * (size_t)n);
}
void put_layer_head(std::string *s, int id) {
  put_bytes(s, PK_NNET_LAYER_SECTION, 4);
  put_i32(s, id);
}

template <typename V>
void to_std(const VectorBase<float> &v, V *out) {
  out->assign(v.Data(), v.Data() + v.Dim());
}

// Parameter vectors are uploaded back to back into one buffer on first use.
void upload_once(bool *done, catears::host::DeviceBuffer *buf, const std::vector<const std::vector<float> *> &parts) {
  if (*done) return;
  size_t total = 0;
  for (auto *p : parts) total += p->size();
  float *d = static_cast<float *>(buf->Reserve(sizeof(float) * (total ? total : 1)));
  Runtime &rt = Runtime::Get();
  for (auto *p : parts) {
    rt.Upload(d, p->size(), p->data(), p->size(), sizeof(float), 1, p->size());
    d += p->size();
  }
  rt.Sync();  // host vectors are not pinned; finish before they can change
  *done = true;
}

}  // namespace

// ------------------------------------------------------------------ Layer --

void Layer::Propagate(const MatrixBase<float> &in, Matrix<float> *out) const {
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  DeviceMatrix x, y;
  x.Resize(in.NumRows(), in.NumCols());
  rt.Upload(x.data, x.cols, in.Data(), in.Stride(), sizeof(float), x.rows, x.cols);
  PropagateDevice(x, &y);
  out->Resize(y.rows, y.cols, Matrix<float>::kUndefined);
  rt.Download(out->Data(), out->Stride(), y.data, y.cols, sizeof(float), y.rows, y.cols);
}

// ---------------------------------------------------------------- Linear --

LinearLayer::LinearLayer() {}

LinearLayer::LinearLayer(const MatrixBase<float> &W, const VectorBase<float> &b)
    : in_(W.NumRows()), out_(W.NumCols()) {
  w_.resize((size_t)in_ * out_);
  for (int r = 0; r < in_; ++r) memcpy(&w_[(size_t)r * out_], W.Data() + (size_t)r * W.Stride(), 4 * (size_t)out_);
  to_std(b, &b_);
}

Status LinearLayer::Read(util::ReadableFile *fd) {  // src/nnet.cc:38-43: W (MAT0) then b (VEC0)
  Matrix<float> W;
  Vector<float> b;
  PK_CHECK_STATUS(W.Read(fd));
  PK_CHECK_STATUS(b.Read(fd));
  in_ = W.NumRows();
  out_ = W.NumCols();
  w_.resize((size_t)in_ * out_);
  for (int r = 0; r < in_; ++r) memcpy(&w_[(size_t)r * out_], W.Data() + (size_t)r * W.Stride(), 4 * (size_t)out_);
  to_std(b, &b_);
  uploaded_ = false;
  return Status::OK();
}

void LinearLayer::PropagateDevice(const DeviceMatrix &in, DeviceMatrix *out) const {
  assert(in.cols == in_ && (int)b_.size() == out_ && "LinearLayer: shape mismatch");
  upload_once(&uploaded_, &d_params_, {&w_, &b_});  // W (in x out) then b
  out->Resize(in.rows, out_);
  const float *w = d_params_.as<float>();
  Check(ce_gpu_linear(Runtime::Get().ctx(), in.rows, in_, out_, in.data, in.cols, w, out_, w + w_.size(),
                      out->data, out_),
        "LinearLayer::Propagate");
}

void LinearLayer::AppendImage(std::string *s) const {
  put_layer_head(s, kLinear);
  put_bytes(s, PK_MATRIX_SECTION, 4);
  put_i32(s, 8 + in_ * (12 + 4 * out_));  // section size (not checked by readers)
  put_i32(s, in_);
  put_i32(s, out_);
  for (int r = 0; r < in_; ++r) put_vec(s, &w_[(size_t)r * out_], out_);
  put_vec(s, b_.data(), (int)b_.size());
}

// ---------------------------------------------------------------- Splice --

SpliceLayer::SpliceLayer() {}
SpliceLayer::SpliceLayer(const std::vector<int> &indices) : indices_(indices) {}

Status SpliceLayer::Read(util::ReadableFile *fd) {  // src/nnet.cc:77-95
  indices_.clear();
  int32_t n = 0;
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&n));
  if (n < 0) return Status::Corruption("SpliceLayer: unexpected num_indcies");
  for (int i = 0; i < n; ++i) {
    int32_t v = 0;
    PK_CHECK_STATUS(fd->ReadValue<int32_t>(&v));
    indices_.push_back(v);
  }
  return Status::OK();
}

void SpliceLayer::PropagateDevice(const DeviceMatrix &in, DeviceMatrix *out) const {
  assert(!indices_.empty() && "SpliceLayer is not initialized");
  const int n = (int)indices_.size();
  out->Resize(in.rows, in.cols * n);
  if (in.rows == 0 || in.cols == 0) return;
  std::vector<int32_t> idx(indices_.begin(), indices_.end());
  Check(ce_gpu_splice(Runtime::Get().ctx(), in.rows, in.cols, in.data, in.cols, idx.data(), n, out->data),
        "SpliceLayer::Propagate");
}

void SpliceLayer::AppendImage(std::string *s) const {
  put_layer_head(s, kSplice);
  put_i32(s, (int32_t)indices_.size());
  for (int v : indices_) put_i32(s, v);
}

// ------------------------------------------------------------- BatchNorm --

BatchNormLayer::BatchNormLayer() {}
BatchNormLayer::BatchNormLayer(const VectorBase<float> &scale, const VectorBase<float> &offset) {
  to_std(scale, &scale_);
  to_std(offset, &offset_);
}

Status BatchNormLayer::Read(util::ReadableFile *fd) {  // src/nnet.cc:119-123
  Vector<float> scale, offset;
  PK_CHECK_STATUS(scale.Read(fd));
  PK_CHECK_STATUS(offset.Read(fd));
  to_std(scale, &scale_);
  to_std(offset, &offset_);
  uploaded_ = false;
  return Status::OK();
}

void BatchNormLayer::PropagateDevice(const DeviceMatrix &in, DeviceMatrix *out) const {
  assert(!scale_.empty() && (int)scale_.size() == in.cols && "BatchNormLayer: shape mismatch");
  upload_once(&uploaded_, &d_params_, {&scale_, &offset_});
  Runtime &rt = Runtime::Get();
  out->Resize(in.rows, in.cols);
  rt.CopyDevice(out->data, out->cols, in.data, in.cols, sizeof(float), in.rows, in.cols);
  const float *p = d_params_.as<float>();
  Check(ce_gpu_rowwise(rt.ctx(), CE_GPU_ROW_BATCHNORM, in.rows, in.cols, out->data, out->cols, p,
                       p + scale_.size()),
        "BatchNormLayer::Propagate");
}

void BatchNormLayer::AppendImage(std::string *s) const {
  put_layer_head(s, kBatchNorm);
  put_vec(s, scale_.data(), (int)scale_.size());
  put_vec(s, offset_.data(), (int)offset_.size());
}

// ------------------------------------------------------ per-row layers --

void RowLayer::PropagateDevice(const DeviceMatrix &in, DeviceMatrix *out) const {
  Runtime &rt = Runtime::Get();
  out->Resize(in.rows, in.cols);
  rt.CopyDevice(out->data, out->cols, in.data, in.cols, sizeof(float), in.rows, in.cols);
  Check(ce_gpu_rowwise(rt.ctx(), op_, in.rows, in.cols, out->data, out->cols, nullptr, nullptr),
        "Layer::Propagate");
}

void RowLayer::AppendImage(std::string *s) const { put_layer_head(s, id_); }

SoftmaxLayer::SoftmaxLayer() : RowLayer(kSoftmax, CE_GPU_ROW_SOFTMAX) {}
LogSoftmaxLayer::LogSoftmaxLayer() : RowLayer(kLogSoftmax, CE_GPU_ROW_LOGSOFTMAX) {}
ReLULayer::ReLULayer() : RowLayer(kReLU, CE_GPU_ROW_RELU) {}
NormalizeLayer::NormalizeLayer() : RowLayer(kNormalize, CE_GPU_ROW_NORMALIZE) {}

// ---------------------------------------------------------------- Narrow --

NarrowLayer::NarrowLayer() {}
NarrowLayer::NarrowLayer(int narrow_left, int narrow_right) : left_(narrow_left), right_(narrow_right) {}

Status NarrowLayer::Read(util::ReadableFile *fd) {  // src/nnet.cc:205-215
  int32_t l = 0, r = 0;
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&l));
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&r));
  left_ = l;
  right_ = r;
  return Status::OK();
}

void NarrowLayer::PropagateDevice(const DeviceMatrix &in, DeviceMatrix *out) const {
  assert(left_ >= 0 && "NarrowLayer is not initialized");
  // blocks too short to narrow pass through unchanged (src/nnet.cc:186-189)
  const bool pass = in.rows <= left_ + right_;
  const int first = pass ? 0 : left_;
  const int rows = pass ? in.rows : in.rows - left_ - right_;
  out->Resize(rows, in.cols);
  Runtime::Get().CopyDevice(out->data, out->cols, in.data + (size_t)first * in.cols, in.cols, sizeof(float), rows,
                            in.cols);
}

void NarrowLayer::AppendImage(std::string *s) const {
  put_layer_head(s, kNarrow);
  put_i32(s, left_);
  put_i32(s, right_);
}

// ------------------------------------------------------------------ Nnet --

Nnet::Nnet() {}

Nnet::~Nnet() {
  if (program_) ce_gpu_model_destroy(program_);
}

Status Nnet::ReadLayer(util::ReadableFile *fd) {  // src/nnet.cc:221-271
  PK_CHECK_STATUS(fd->ReadAndVerifyString(PK_NNET_LAYER_SECTION));
  int32_t type = 0;
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&type));
  std::unique_ptr<Layer> layer;
  switch (type) {
    case Layer::kLinear: layer.reset(new LinearLayer()); break;
    case Layer::kReLU: layer.reset(new ReLULayer()); break;
    case Layer::kNormalize: layer.reset(new NormalizeLayer()); break;
    case Layer::kSoftmax: layer.reset(new SoftmaxLayer()); break;
    case Layer::kSplice: layer.reset(new SpliceLayer()); break;
    case Layer::kBatchNorm: layer.reset(new BatchNormLayer()); break;
    case Layer::kLogSoftmax: layer.reset(new LogSoftmaxLayer()); break;
    case Layer::kNarrow: layer.reset(new NarrowLayer()); break;
    default:
      return Status::Corruption(util::Format("read_layer: unexpected layer type: {} ({})", type, fd->filename()));
  }
  PK_CHECK_STATUS(layer->Read(fd));
  layer->AppendImage(&image_);
  layers_.emplace_back(std::move(layer));
  return Status::OK();
}

Status Nnet::Read(util::ReadableFile *fd) {  // src/nnet.cc:273-293
  PK_CHECK_STATUS(fd->ReadAndVerifyString(PK_NNET_SECTION));
  int32_t l = 0, r = 0, n = 0;
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&l));
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&r));
  left_context_ = l;
  right_context_ = r;
  PK_CHECK_STATUS(fd->ReadValue<int32_t>(&n));
  image_.clear();
  put_bytes(&image_, PK_NNET_SECTION, 4);
  put_i32(&image_, l);
  put_i32(&image_, r);
  put_i32(&image_, n);
  for (int i = 0; i < n; ++i) PK_CHECK_STATUS(ReadLayer(fd));
  if (program_) ce_gpu_model_destroy(program_);
  program_ = nullptr;
  program_tried_ = false;
  return Status::OK();
}

void Nnet::Propagate(const MatrixBase<float> &in, Matrix<float> *out) const {
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  if (!program_tried_) {
    program_tried_ = true;
    // A network the fused program does not take (e.g. a lone layer) runs
    // layer by layer below; both paths are device code.
    if (ce_gpu_model_load_mem(rt.ctx(), image_.data(), (int64_t)image_.size(), nullptr, 0, -1, -1, &program_) !=
        CE_GPU_OK)
      program_ = nullptr;
    if (program_) ce_gpu_model_info(program_, &program_left_, &program_right_, nullptr, nullptr, nullptr, nullptr);
  }
  DeviceMatrix x;
  x.Resize(in.NumRows(), in.NumCols());
  rt.Upload(x.data, x.cols, in.Data(), in.Stride(), sizeof(float), x.rows, x.cols);
  int input_dim = 0, pdfs = 0;
  if (program_) ce_gpu_model_info(program_, nullptr, nullptr, &input_dim, &pdfs, nullptr, nullptr);
  if (program_ && in.NumCols() == input_dim && in.NumRows() > program_left_ + program_right_) {
    const int rows = in.NumRows() - program_left_ - program_right_;
    DeviceMatrix y;
    y.Resize(rows, pdfs);
    Check(ce_gpu_nnet_propagate(rt.ctx(), program_, x.data, x.rows, x.cols, 0, y.data), "Nnet::Propagate");
    out->Resize(rows, pdfs, Matrix<float>::kUndefined);
    rt.Download(out->Data(), out->Stride(), y.data, pdfs, sizeof(float), rows, pdfs);
    return;
  }
  DeviceMatrix y;
  for (const std::unique_ptr<Layer> &layer : layers_) {
    layer->PropagateDevice(x, &y);
    std::swap(x, y);
  }
  out->Resize(x.rows, x.cols, Matrix<float>::kUndefined);
  rt.Download(out->Data(), out->Stride(), x.data, x.cols, sizeof(float), x.rows, x.cols);
}

}  // namespace pocketkaldi
