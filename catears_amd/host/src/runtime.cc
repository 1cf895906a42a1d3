// runtime.cc -- process-wide device context for the drop-in classes
// (catears_runtime.h).  HIP is used here only for memory and copies; every
// kernel is reached through the catears_gpu C-ABI.
#include "catears_runtime.h"

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <memory>
#include <string>

namespace catears {
namespace host {

static void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw DeviceError(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace host
}  // namespace catears

// Test-only failure injection: a weak reference that only the test driver
// (tests/native/pk_dropin.cc, linked -rdynamic) defines.  In every product
// binary it resolves to null, so Check() carries no test state and costs one
// pointer test on its error-free path.
extern "C" __attribute__((weak)) int catears_test_inject_failure(void);

namespace catears {
namespace host {

void Check(int rc, const char *what) {
  if (rc != CE_GPU_OK) throw DeviceError(std::string(what) + ": " + ce_gpu_last_error());
  if (catears_test_inject_failure && catears_test_inject_failure())
    throw DeviceError(std::string(what) + ": injected device failure");
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

struct Runtime::Lane {
  int index = 0;
  ce_gpu_ctx *ctx = nullptr;
  void *stream = nullptr;
  std::mutex mu;
  DeviceBuffer scratch[kScratchSlots];
};

static void copy2d(void *stream, hipMemcpyKind kind, void *dst, size_t dst_ld, const void *src, size_t src_ld,
                   size_t elem, size_t rows, size_t cols, const char *what) {
  if (!rows || !cols) return;
  hip_check(hipMemcpy2DAsync(dst, dst_ld * elem, src, src_ld * elem, cols * elem, rows, kind,
                             static_cast<hipStream_t>(stream)),
            what);
}

Runtime::Lane *Runtime::NewLane() {
  // caller holds pool_mu_ (or is the constructor)
  // nothing leaks when a step throws: the lane, its stream and its context
  // are released on the way out, and the pool is unchanged
  std::unique_ptr<Lane> l(new Lane());
  l->index = n_lanes_;
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hipStream_t s = nullptr;
  hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  l->stream = s;
  try {
    Check(ce_gpu_ctx_create(device_, l->stream, &l->ctx), "ce_gpu_ctx_create");
    Check(ce_gpu_ctx_set_fbank(l->ctx, fbank_mode_), "ce_gpu_ctx_set_fbank");
  } catch (...) {
    if (l->ctx) ce_gpu_ctx_destroy(l->ctx);
    hipStreamDestroy(s);
    throw;
  }
  lanes_[n_lanes_++] = l.get();
  return l.release();
}

Runtime::Runtime() {
  const char *dev = getenv("CATEARS_DEVICE");
  device_ = dev ? atoi(dev) : 0;
  if (const char *e = getenv("CATEARS_LANES")) {
    const int v = atoi(e);
    if (v < 1 || v > 16) throw DeviceError("CATEARS_LANES must be 1..16");
    max_lanes_ = v;
  }
  // CATEARS_FBANK=fast: every lane's fbank launches take the fast kernel
  // (the exact lane program with FMA contraction, ce_gpu_ctx_set_fbank);
  // "exact" (the default) keeps the reference's operation order
  if (const char *e = getenv("CATEARS_FBANK")) {
    const std::string v(e);
    if (v == "fast")
      fbank_mode_ = CE_GPU_FBANK_FAST;
    else if (v != "exact")
      throw DeviceError("CATEARS_FBANK must be \"exact\" or \"fast\"");
  }
  NewLane();  // lane 0: the layer-level paths and model loading
}

Runtime::~Runtime() {}

Runtime &Runtime::Get() {
  // Deliberately leaked: HIP objects must not be torn down from static
  // destructors after the runtime itself has shut down.
  static Runtime *rt = new Runtime();
  return *rt;
}

Runtime::Lease Runtime::Acquire() {
  Lane *wait_on = nullptr;
  {
    std::lock_guard<std::mutex> pool(pool_mu_);
    for (int t = 0; t < n_lanes_; ++t) {
      Lane *l = lanes_[(next_ + t) % n_lanes_];
      std::unique_lock<std::mutex> lk(l->mu, std::try_to_lock);
      if (lk.owns_lock()) {
        next_ = (unsigned)(l->index + 1);
        return Lease(l, std::move(lk));
      }
    }
    if (n_lanes_ < max_lanes_) {
      Lane *l = NewLane();
      return Lease(l, std::unique_lock<std::mutex>(l->mu));
    }
    wait_on = lanes_[next_++ % n_lanes_];
  }
  return Lease(wait_on, std::unique_lock<std::mutex>(wait_on->mu));
}

int Runtime::lanes_created() const {
  std::lock_guard<std::mutex> pool(pool_mu_);
  return n_lanes_;
}

ce_gpu_ctx *Runtime::Lease::ctx() const { return lane_->ctx; }
DeviceBuffer &Runtime::Lease::scratch(int slot) { return lane_->scratch[slot]; }
int Runtime::Lease::index() const { return lane_->index; }

void Runtime::Lease::Upload(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                            size_t cols) {
  copy2d(lane_->stream, hipMemcpyHostToDevice, dst, dst_ld, src, src_ld, elem, rows, cols, "hipMemcpy2DAsync(H2D)");
}

void Runtime::Lease::Download(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                              size_t cols) {
  copy2d(lane_->stream, hipMemcpyDeviceToHost, dst, dst_ld, src, src_ld, elem, rows, cols, "hipMemcpy2DAsync(D2H)");
  hip_check(hipStreamSynchronize(static_cast<hipStream_t>(lane_->stream)), "hipStreamSynchronize");
}

ce_gpu_ctx *Runtime::ctx() const { return lanes_[0]->ctx; }
void *Runtime::stream() const { return lanes_[0]->stream; }
std::mutex &Runtime::mutex() { return lanes_[0]->mu; }
DeviceBuffer &Runtime::scratch(int slot) { return lanes_[0]->scratch[slot]; }

void Runtime::Upload(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                     size_t cols) {
  copy2d(stream(), hipMemcpyHostToDevice, dst, dst_ld, src, src_ld, elem, rows, cols, "hipMemcpy2DAsync(H2D)");
}

void Runtime::Download(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                       size_t cols) {
  copy2d(stream(), hipMemcpyDeviceToHost, dst, dst_ld, src, src_ld, elem, rows, cols, "hipMemcpy2DAsync(D2H)");
  Sync();
}

void Runtime::CopyDevice(void *dst, size_t dst_ld, const void *src, size_t src_ld, size_t elem, size_t rows,
                         size_t cols) {
  copy2d(stream(), hipMemcpyDeviceToDevice, dst, dst_ld, src, src_ld, elem, rows, cols, "hipMemcpy2DAsync(D2D)");
}

void Runtime::Sync() {
  hip_check(hipStreamSynchronize(static_cast<hipStream_t>(stream())), "hipStreamSynchronize");
}

}  // namespace host
}  // namespace catears
