// catears_runtime.h -- the device side shared by the drop-in pocketkaldi
// classes (fbank.h, cmvn.h, nnet.h, am.h, linalg).  Not part of the
// reference's API; the classes reach the GPU only through include/catears_gpu.h.
//
// ce_gpu contexts on device $CATEARS_DEVICE (default 0), each with its own
// HIP stream (a "lane").  The reference's hot-path methods are const and may
// be called from many threads (SURVEY.md 8(b) Threading): every drop-in call
// holds one lane for its upload -> kernels -> download sequence and returns
// with its results on the host, like the CPU code it replaces; calls from
// different threads run on different lanes concurrently.
// Device failures throw DeviceError (the reference would have crashed on an
// assert or bad_alloc); there is no CPU fallback.
#ifndef CATEARS_RUNTIME_H_
#define CATEARS_RUNTIME_H_

#include <stddef.h>

#include <mutex>
#include <utility>
#include <stdexcept>
#include <string>

#include "catears_gpu.h"

namespace catears {
namespace host {

class DeviceError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// Throws DeviceError("<what>: <ce_gpu_last_error()>") unless rc == CE_GPU_OK.
void Check(int rc, const char *what);

// Grow-only device allocation.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  ~DeviceBuffer();
  DeviceBuffer(DeviceBuffer &&o) noexcept;
  DeviceBuffer &operator=(DeviceBuffer &&o) noexcept;
  DeviceBuffer(const DeviceBuffer &) = delete;
  DeviceBuffer &operator=(const DeviceBuffer &) = delete;

  void *Reserve(size_t bytes);
  template <typename T>
  T *as() const {
    return static_cast<T *>(ptr_);
  }
  size_t capacity() const { return cap_; }

 private:
  void *ptr_ = nullptr;
  size_t cap_ = 0;
};

// Dense row-major fp32 matrix in HBM (ld = cols).
struct DeviceMatrix {
  DeviceBuffer buf;
  float *data = nullptr;
  int rows = 0, cols = 0;
  void Resize(int r, int c) {
    data = static_cast<float *>(buf.Reserve(sizeof(float) * (size_t)(r > 0 ? r : 1) * (size_t)(c > 0 ? c : 1)));
    rows = r;
    cols = c;
  }
};

class Runtime {
 public:
  // Creates the context on first use.  Throws DeviceError if the HIP
  // library or the device is unusable.
  static Runtime &Get();

  // Streaming calls from many threads (AcousticModel, Fbank, CMVN) lease a
  // lane: a context with its own HIP stream and scratch, held exclusively for
  // one upload -> kernels -> download sequence, so concurrent Instances
  // overlap their copies and kernels instead of queueing on one mutex.
  // Lanes are created on demand up to $CATEARS_LANES (default 4, 1..16); a
  // caller finding every lane busy waits for one.  Device models (weights)
  // are shared by all lanes of the device.
  class Lane;
  class Lease {
   public:
    Lease(Lane *lane, std::unique_lock<std::mutex> lock) : lane_(lane), lock_(std::move(lock)) {}
    ce_gpu_ctx *ctx() const;
    DeviceBuffer &scratch(int slot);
    // as Runtime::Upload / Download, on the lane's stream
    void Upload(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows, size_t cols);
    void Download(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows, size_t cols);
    int index() const;

   private:
    Lane *lane_;
    std::unique_lock<std::mutex> lock_;
  };
  Lease Acquire();
  int lanes_created() const;

  // Lane 0, for the layer-level paths (Nnet / Layer::Propagate, MatMat,
  // model loading) which take mutex() for their whole sequence.
  ce_gpu_ctx *ctx() const;
  void *stream() const;
  std::mutex &mutex();

  // Strided 2-D copies on lane 0's stream (element size `elem` bytes,
  // leading dimensions in elements).  Upload/CopyDevice are asynchronous;
  // Download waits for the stream.
  void Upload(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows, size_t cols);
  void Download(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows, size_t cols);
  void CopyDevice(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                  size_t cols);
  void Sync();

  // Per-call scratch of lane 0 (use only while holding mutex()).
  DeviceBuffer &scratch(int slot);
  static constexpr int kScratchSlots = 6;

 private:
  Runtime();
  ~Runtime();
  Lane *NewLane();
  int device_ = 0;
  int max_lanes_ = 4;
  int fbank_mode_ = 0;  // CE_GPU_FBANK_EXACT, or _FAST from CATEARS_FBANK
  mutable std::mutex pool_mu_;
  Lane *lanes_[16] = {nullptr};
  int n_lanes_ = 0;
  unsigned next_ = 0;
};

}  // namespace host
}  // namespace catears

#endif  // CATEARS_RUNTIME_H_
