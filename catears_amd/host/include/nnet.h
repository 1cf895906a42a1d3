// nnet.h -- drop-in replacement for pocketkaldi's nnet.h (reference
// src/nnet.h:18-260): the same Layer / Nnet classes and signatures, with
// Propagate running on the MI355X through the catears_gpu C-ABI.
//
//   Nnet::Read       parses NN02 on the host (src/nnet.cc:221-293) and keeps
//                    the image; the first Propagate uploads it as a fused
//                    device program (ce_gpu_model_load_mem).
//   Nnet::Propagate  one ce_gpu_nnet_propagate call when the network has the
//                    converter's shape (every Splice followed by its Narrow
//                    and a Linear, tool/convert_am.py:272-285) and the block
//                    covers its context; otherwise layer by layer on the
//                    device, each Layer keeping the reference semantics
//                    (Splice clamps, Narrow passes short blocks through).
//   Layer::Propagate upload -> one device op -> download.
#ifndef CATEARS_PK_NNET_H_
#define CATEARS_PK_NNET_H_

#include <memory>
#include <string>
#include <vector>

#include "catears_runtime.h"
#include "matrix.h"
#include "util.h"

#define PK_NNET_SECTION "NN02"
#define PK_NNET_LAYER_SECTION "LAY0"

namespace pocketkaldi {

class Layer {
 public:
  // Type ids as stored after LAY0 (src/nnet.h:21-30).
  enum { kLinear = 0, kReLU = 1, kNormalize = 2, kSoftmax = 3, kSplice = 6, kBatchNorm = 7, kLogSoftmax = 8,
         kNarrow = 9 };

  // in (rows x d) -> out, resized by the layer.
  virtual void Propagate(const MatrixBase<float> &in, Matrix<float> *out) const;
  virtual Status Read(util::ReadableFile *fd) = 0;
  virtual std::string Type() const = 0;
  virtual ~Layer() {}

  // Device form of Propagate (HBM in, HBM out); caller holds the runtime lock.
  virtual void PropagateDevice(const catears::host::DeviceMatrix &in, catears::host::DeviceMatrix *out) const = 0;
  // Appends this layer's LAY0 record (id + payload) to an NN02 image.
  virtual void AppendImage(std::string *image) const = 0;
};

class LinearLayer : public Layer {
 public:
  LinearLayer();
  LinearLayer(const MatrixBase<float> &W, const VectorBase<float> &b);
  Status Read(util::ReadableFile *fd) override;
  std::string Type() const override { return "Linear"; }
  void PropagateDevice(const catears::host::DeviceMatrix &in, catears::host::DeviceMatrix *out) const override;
  void AppendImage(std::string *image) const override;

 private:
  std::vector<float> w_;  // in x out, MAT0 order
  std::vector<float> b_;
  int in_ = 0, out_ = 0;
  mutable catears::host::DeviceBuffer d_params_;  // W then b
  mutable bool uploaded_ = false;
};

class SpliceLayer : public Layer {
 public:
  SpliceLayer();
  explicit SpliceLayer(const std::vector<int> &indices);
  Status Read(util::ReadableFile *fd) override;
  std::string Type() const override { return "Splice"; }
  void PropagateDevice(const catears::host::DeviceMatrix &in, catears::host::DeviceMatrix *out) const override;
  void AppendImage(std::string *image) const override;

 private:
  std::vector<int> indices_;
};

class BatchNormLayer : public Layer {
 public:
  BatchNormLayer();
  BatchNormLayer(const VectorBase<float> &scale, const VectorBase<float> &offset);
  Status Read(util::ReadableFile *fd) override;
  std::string Type() const override { return "BatchNorm"; }
  void PropagateDevice(const catears::host::DeviceMatrix &in, catears::host::DeviceMatrix *out) const override;
  void AppendImage(std::string *image) const override;

 private:
  std::vector<float> scale_, offset_;
  mutable catears::host::DeviceBuffer d_params_;  // scale then offset
  mutable bool uploaded_ = false;
};

// Parameter-free per-row layers share one implementation.
class RowLayer : public Layer {
 public:
  Status Read(util::ReadableFile *) override { return Status::OK(); }
  void PropagateDevice(const catears::host::DeviceMatrix &in, catears::host::DeviceMatrix *out) const override;
  void AppendImage(std::string *image) const override;

 protected:
  RowLayer(int id, int op) : id_(id), op_(op) {}

 private:
  int id_, op_;
};

class SoftmaxLayer : public RowLayer {
 public:
  SoftmaxLayer();
  std::string Type() const override { return "Softmax"; }
};

class LogSoftmaxLayer : public RowLayer {
 public:
  LogSoftmaxLayer();
  std::string Type() const override { return "LogSoftmax"; }
};

class ReLULayer : public RowLayer {
 public:
  ReLULayer();
  std::string Type() const override { return "ReLU"; }
};

class NormalizeLayer : public RowLayer {
 public:
  NormalizeLayer();
  std::string Type() const override { return "Normalize"; }
};

class NarrowLayer : public Layer {
 public:
  NarrowLayer();
  NarrowLayer(int narrow_left, int narrow_right);
  Status Read(util::ReadableFile *fd) override;
  std::string Type() const override { return "NarrowLayer"; }
  void PropagateDevice(const catears::host::DeviceMatrix &in, catears::host::DeviceMatrix *out) const override;
  void AppendImage(std::string *image) const override;

 private:
  int left_ = -1, right_ = -1;
};

class Nnet {
 public:
  Nnet();
  ~Nnet();

  Status Read(util::ReadableFile *fd);
  void Propagate(const MatrixBase<float> &in, Matrix<float> *out) const;

  int left_context() const { return left_context_; }
  int right_context() const { return right_context_; }

  // The NN02 image this network was read from (re-serialised), for loaders
  // that build their own device program (AcousticModel).
  const std::string &image() const { return image_; }

 private:
  std::vector<std::unique_ptr<Layer>> layers_;
  int left_context_ = 0, right_context_ = 0;
  std::string image_;
  // device program: built on first Propagate; fused == false -> layerwise
  mutable ce_gpu_model *program_ = nullptr;
  mutable bool program_tried_ = false;
  mutable int program_left_ = 0, program_right_ = 0;

  Status ReadLayer(util::ReadableFile *fd);
  Nnet(const Nnet &) = delete;
  Nnet &operator=(const Nnet &) = delete;
};

}  // namespace pocketkaldi

#endif  // CATEARS_PK_NNET_H_
