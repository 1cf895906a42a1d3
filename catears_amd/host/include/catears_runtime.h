// catears_runtime.h -- the device side shared by the drop-in pocketkaldi
// classes (fbank.h, cmvn.h, nnet.h, am.h, linalg).  Not part of the
// reference's API; the classes reach the GPU only through include/catears_gpu.h.
//
// One ce_gpu context per process on device $CATEARS_DEVICE (default 0) with
// its own HIP stream.  The reference's hot-path methods are const and may be
// called from many threads (SURVEY.md 8(b) Threading), so every drop-in call
// takes Runtime::mutex() for its upload -> kernels -> download sequence and
// returns with its results on the host, like the CPU code it replaces.
// Device failures throw DeviceError (the reference would have crashed on an
// assert or bad_alloc); there is no CPU fallback.
#ifndef CATEARS_RUNTIME_H_
#define CATEARS_RUNTIME_H_

#include <stddef.h>

#include <mutex>
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

// Test support: the next `n` Check() calls throw DeviceError as if their
// device call had failed (exercises the error paths, e.g. the AcousticModel
// batcher releasing its followers).  Process-wide, thread-safe.
void InjectDeviceFailures(int n);

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

  ce_gpu_ctx *ctx() const { return ctx_; }
  void *stream() const { return stream_; }
  std::mutex &mutex() { return mu_; }

  // Strided 2-D copies on the runtime's stream (element size `elem` bytes,
  // leading dimensions in elements).  Upload/CopyDevice are asynchronous;
  // Download waits for the stream.
  void Upload(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows, size_t cols);
  void Download(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows, size_t cols);
  void CopyDevice(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                  size_t cols);
  void Sync();

  // Per-call scratch (use only while holding mutex()).
  DeviceBuffer &scratch(int slot) { return scratch_[slot]; }
  static constexpr int kScratchSlots = 6;

 private:
  Runtime();
  ~Runtime();
  ce_gpu_ctx *ctx_ = nullptr;
  void *stream_ = nullptr;
  int device_ = 0;
  std::mutex mu_;
  DeviceBuffer scratch_[kScratchSlots];
};

}  // namespace host
}  // namespace catears

#endif  // CATEARS_RUNTIME_H_
