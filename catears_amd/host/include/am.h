// am.h -- drop-in replacement for pocketkaldi's am.h (reference
// src/am.h:22-86): AcousticModel with the same Read / Process / EndOfStream /
// TransitionPdfIdMap / num_pdfs API.  Process keeps the reference's chunking
// (L copies of the first frame, a batch of L + R + chunk_size rows whenever
// that many frames are buffered, R copies of the last frame at the end,
// src/am.cc:115-164); each batch runs as one fused device call
// (ce_gpu_nnet_propagate with the log prior subtracted, src/am.cc:82-113).
// Because every Splice is followed by its Narrow, a batch's rows do not
// depend on where chunks start, so a larger chunk_size in the config only
// changes how many rows one device call carries.
//
// Serving many streams: with the optional config key
// gpu_batch_streams = N > 1, chunks that become ready on different Instances
// (threads) at about the same time are scored in ONE device call
// (ce_gpu_nnet_propagate_blocks): the first caller waits up to
// gpu_batch_wait_us (default 200) for up to N-1 others, runs the batch, and
// every caller gets exactly the rows it would have got alone.
#ifndef CATEARS_PK_AM_H_
#define CATEARS_PK_AM_H_

#include <memory>
#include <vector>

#include "catears_runtime.h"
#include "configuration.h"
#include "nnet.h"
#include "util.h"

#define PK_AM_SECTION "AM~0"

namespace pocketkaldi {

class AcousticModel {
 public:
  class Instance;

  static constexpr int kBatchSizeAll = -1;

  AcousticModel();
  ~AcousticModel();

  // Keys nnet, prior, left_context, right_context, chunk_size, num_pdfs,
  // tid2pdf (src/am.cc:26-64).
  Status Read(const Configuration &conf);

  const Vector<int32_t> &TransitionPdfIdMap() const { return tid2pdf_; }

  // One feature frame in; 0 or chunk_size rows of log-likelihoods out.
  void Process(Instance *inst, const VectorBase<float> &frame_feat, Matrix<float> *log_prob) const;

  // Flushes the buffered frames (right padding applied).
  void EndOfStream(Instance *inst, Matrix<float> *log_prob) const;

  int num_pdfs() const { return num_pdfs_; }

  // Device program (for batch scorers built on the same model).
  const ce_gpu_model *device_model() const { return model_; }

  // Device calls made so far / blocks they carried (batching statistics).
  void batch_stats(int64_t *calls, int64_t *blocks) const;

 private:
  struct Batcher;
  ce_gpu_model *model_ = nullptr;
  int left_context_ = 0;
  int right_context_ = 0;
  int chunk_size_ = 0;
  int num_pdfs_ = 0;
  int feat_dim_ = 0;
  int latency_ = 1;  // gpu_latency_mode: applied to the shared context per call
  Vector<int32_t> tid2pdf_;
  std::unique_ptr<Batcher> batcher_;

  void Append(Instance *inst, const float *frame, int dim) const;
  void ComputeBatch(Instance *inst, int batch_size, Matrix<float> *log_prob) const;
  void RunBlocks(const std::vector<const float *> &rows, const std::vector<int32_t> &n, int dim,
                 const std::vector<Matrix<float> *> &out) const;
  AcousticModel(const AcousticModel &) = delete;
  AcousticModel &operator=(const AcousticModel &) = delete;
};

class AcousticModel::Instance {
 public:
  Instance() = default;

 private:
  friend class AcousticModel;
  bool started = false;
  int dim = 0;
  size_t head = 0;             // first live row in `rows`
  std::vector<float> rows;     // buffered feature rows, dim floats each
  size_t size() const { return dim ? rows.size() / dim - head : 0; }
  Instance(const Instance &) = delete;
  Instance &operator=(const Instance &) = delete;
};

}  // namespace pocketkaldi

#endif  // CATEARS_PK_AM_H_
