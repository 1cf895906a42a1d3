// vector.h -- stand-in for pocketkaldi's vector containers (reference
// src/vector.h:43-258, src/vector.cc) for builds outside the reference tree.
// VectorBase is a (data, dim) view; Vector owns 32-byte aligned storage;
// SubVector borrows.  Arithmetic follows the reference's sequential float
// order where it matters to callers (ApplyLogSoftMax: no max shift,
// src/vector.cc:109-122).
#ifndef CATEARS_COMPAT_VECTOR_H_
#define CATEARS_COMPAT_VECTOR_H_

#include <assert.h>
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "status.h"
#include "util.h"

#define PK_VECTOR_SECTION "VEC0"

namespace pocketkaldi {

template <typename Real>
class SubVector;

template <typename Real>
class VectorBase {
 public:
  int Dim() const { return dim_; }
  Real *Data() { return data_; }
  const Real *Data() const { return data_; }

  Real operator()(int i) const {
    assert(i < dim_);
    return data_[i];
  }
  Real &operator()(int i) {
    assert(i < dim_);
    return data_[i];
  }

  SubVector<Real> Range(int o, int l) { return SubVector<Real>(*this, o, l); }
  const SubVector<Real> Range(int o, int l) const { return SubVector<Real>(*this, o, l); }

  void SetZero() {
    if (dim_) memset(data_, 0, sizeof(Real) * dim_);
  }
  void Set(Real f) { std::fill(data_, data_ + dim_, f); }
  bool IsZero(Real cutoff = 1.0e-06) const {
    for (int i = 0; i < dim_; ++i)
      if (fabs((double)data_[i]) > cutoff) return false;
    return true;
  }

  template <typename Other>
  void CopyFromVec(const VectorBase<Other> &v) {
    assert(v.Dim() == dim_);
    for (int i = 0; i < dim_; ++i) data_[i] = static_cast<Real>(v.Data()[i]);
  }

  template <typename Other>
  void AddVec(const Real alpha, const VectorBase<Other> &v) {
    assert(v.Dim() == dim_);
    for (int i = 0; i < dim_; ++i) data_[i] += alpha * v.Data()[i];
  }

  Real VecVec(const VectorBase<Real> &v) const {
    assert(v.Dim() == dim_);
    Real s = 0;
    for (int i = 0; i < dim_; ++i) s += data_[i] * v.data_[i];
    return s;
  }
  void MulElements(const VectorBase<Real> &v) {
    assert(v.Dim() == dim_);
    for (int i = 0; i < dim_; ++i) data_[i] *= v.data_[i];
  }
  void Scale(Real a) {
    for (int i = 0; i < dim_; ++i) data_[i] *= a;
  }
  void Add(Real c) {
    for (int i = 0; i < dim_; ++i) data_[i] += c;
  }
  void ApplyLog() {
    for (int i = 0; i < dim_; ++i) data_[i] = log(data_[i]);
  }
  int ApplyFloor(Real floor_val) {
    int n = 0;
    for (int i = 0; i < dim_; ++i)
      if (data_[i] < floor_val) data_[i] = floor_val, ++n;
    return n;
  }
  void ApplyPow(Real p) {
    for (int i = 0; i < dim_; ++i) data_[i] = pow(data_[i], p);
  }
  void ApplySoftMax() {
    Real s = 0;
    for (int i = 0; i < dim_; ++i) s += exp(data_[i]);
    for (int i = 0; i < dim_; ++i) data_[i] = exp(data_[i]) / s;
  }
  void ApplyLogSoftMax() {
    Real s = 0;
    for (int i = 0; i < dim_; ++i) s += exp(data_[i]);
    const Real ls = log(s);
    for (int i = 0; i < dim_; ++i) data_[i] -= ls;
  }

 protected:
  VectorBase() = default;
  ~VectorBase() = default;
  Real *data_ = nullptr;
  int dim_ = 0;
  template <typename>
  friend class VectorBase;
};

template <typename Real>
class Vector : public VectorBase<Real> {
 public:
  enum { kSetZero, kUndefined, kCopyData };

  Vector() = default;
  explicit Vector(int n, int resize_type = kSetZero) { Resize(n, resize_type); }
  Vector(Vector<Real> &&o) noexcept { Swap(&o); }
  Vector<Real> &operator=(Vector<Real> &&o) noexcept {
    Swap(&o);
    return *this;
  }
  ~Vector() { free(this->data_); }

  void Resize(int n, int resize_type = kSetZero) {
    assert(n >= 0);
    if (n == this->dim_ && resize_type != kSetZero) return;
    Real *fresh = nullptr;
    if (n > 0) {
      const size_t bytes = (sizeof(Real) * (size_t)n + 31) / 32 * 32;
      if (posix_memalign(reinterpret_cast<void **>(&fresh), 32, bytes) != 0) abort();
      if (resize_type == kSetZero) memset(fresh, 0, bytes);
      if (resize_type == kCopyData && this->dim_)
        memcpy(fresh, this->data_, sizeof(Real) * std::min(n, this->dim_));
      if (resize_type == kCopyData && n > this->dim_)
        memset(fresh + this->dim_, 0, sizeof(Real) * (n - this->dim_));
    }
    free(this->data_);
    this->data_ = fresh;
    this->dim_ = n;
  }

  void Swap(Vector<Real> *o) {
    std::swap(this->data_, o->data_);
    std::swap(this->dim_, o->dim_);
  }

  // VEC0 section (src/vector.cc:267-300): "VEC0", i32 4*dim+4, i32 dim, data.
  Status Read(util::ReadableFile *fd) {
    PK_CHECK_STATUS(fd->ReadAndVerifyString(PK_VECTOR_SECTION));
    int32_t section = 0, dim = 0;
    PK_CHECK_STATUS(fd->ReadValue<int32_t>(&section));
    PK_CHECK_STATUS(fd->ReadValue<int32_t>(&dim));
    if (dim < 0 || (int64_t)dim * (int64_t)sizeof(Real) + 4 != section)
      return Status::Corruption(util::Format("section_size = {} * {} + 4 expected, but {} found: {}", dim,
                                             sizeof(Real), section, fd->filename()));
    PK_CHECK_STATUS(fd->Need((int64_t)dim * (int64_t)sizeof(Real)));
    Resize(dim, kUndefined);
    if (dim) PK_CHECK_STATUS(fd->Read(this->data_, (int)(dim * sizeof(Real))));
    return Status::OK();
  }

 private:
  Vector(const Vector<Real> &) = delete;
  void operator=(const Vector<Real> &) = delete;
};

template <typename Real>
class SubVector : public VectorBase<Real> {
 public:
  SubVector(const VectorBase<Real> &t, int origin, int length) {
    assert(origin >= 0 && length >= 0 && origin + length <= t.Dim());
    this->data_ = const_cast<Real *>(t.Data()) + origin;
    this->dim_ = length;
  }
  SubVector(Real *data, int length) {
    this->data_ = data;
    this->dim_ = length;
  }
  SubVector(const SubVector<Real> &o) {
    this->data_ = o.data_;
    this->dim_ = o.dim_;
  }
};

}  // namespace pocketkaldi

#endif  // CATEARS_COMPAT_VECTOR_H_
