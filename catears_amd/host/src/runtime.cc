// runtime.cc -- process-wide device context for the drop-in classes
// (catears_runtime.h).  HIP is used here only for memory and copies; every
// kernel is reached through the catears_gpu C-ABI.
#include "catears_runtime.h"

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <atomic>

namespace catears {
namespace host {

static void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw DeviceError(std::string(what) + ": " + hipGetErrorString(e));
}

static std::atomic<int> g_injected_failures{0};

void InjectDeviceFailures(int n) { g_injected_failures.store(n); }

void Check(int rc, const char *what) {
  if (rc != CE_GPU_OK) throw DeviceError(std::string(what) + ": " + ce_gpu_last_error());
  int left = g_injected_failures.load();
  while (left > 0 && !g_injected_failures.compare_exchange_weak(left, left - 1)) {
  }
  if (left > 0) throw DeviceError(std::string(what) + ": injected device failure");
}

DeviceBuffer::~DeviceBuffer() {
  if (ptr_) (void)hipFree(ptr_);
}

DeviceBuffer::DeviceBuffer(DeviceBuffer &&o) noexcept : ptr_(o.ptr_), cap_(o.cap_) {
  o.ptr_ = nullptr;
  o.cap_ = 0;
}

DeviceBuffer &DeviceBuffer::operator=(DeviceBuffer &&o) noexcept {
  if (this != &o) {
    if (ptr_) (void)hipFree(ptr_);
    ptr_ = o.ptr_;
    cap_ = o.cap_;
    o.ptr_ = nullptr;
    o.cap_ = 0;
  }
  return *this;
}

void *DeviceBuffer::Reserve(size_t bytes) {
  if (bytes <= cap_ && ptr_) return ptr_;
  if (ptr_) {
    // a buffer being replaced may still be read by queued work
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipFree(ptr_), "hipFree");
    ptr_ = nullptr;
    cap_ = 0;
  }
  const size_t want = bytes < 256 ? 256 : bytes;
  hip_check(hipMalloc(&ptr_, want), "hipMalloc");
  cap_ = want;
  return ptr_;
}

Runtime::Runtime() {
  const char *dev = getenv("CATEARS_DEVICE");
  device_ = dev ? atoi(dev) : 0;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hipStream_t s = nullptr;
  hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
  Check(ce_gpu_ctx_create(device_, stream_, &ctx_), "ce_gpu_ctx_create");
}

Runtime::~Runtime() {}

Runtime &Runtime::Get() {
  // Deliberately leaked: HIP objects must not be torn down from static
  // destructors after the runtime itself has shut down.
  static Runtime *rt = new Runtime();
  return *rt;
}

void Runtime::Upload(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                     size_t cols) {
  if (!rows || !cols) return;
  hip_check(hipMemcpy2DAsync(dst, dst_ld * elem, src, src_ld * elem, cols * elem, rows, hipMemcpyHostToDevice,
                             static_cast<hipStream_t>(stream_)),
            "hipMemcpy2DAsync(H2D)");
}

void Runtime::Download(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                       size_t cols) {
  if (rows && cols)
    hip_check(hipMemcpy2DAsync(dst, dst_ld * elem, src, src_ld * elem, cols * elem, rows, hipMemcpyDeviceToHost,
                               static_cast<hipStream_t>(stream_)),
              "hipMemcpy2DAsync(D2H)");
  Sync();
}

void Runtime::CopyDevice(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                         size_t cols) {
  if (!rows || !cols) return;
  hip_check(hipMemcpy2DAsync(dst, dst_ld * elem, src, src_ld * elem, cols * elem, rows,
                             hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream_)),
            "hipMemcpy2DAsync(D2D)");
}

void Runtime::Sync() {
  hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream_)), "hipStreamSynchronize");
}

}  // namespace host
}  // namespace catears
