// matrix.h -- stand-in for pocketkaldi's matrix containers and BLAS entry
// points (reference src/matrix.h:25-260) for builds outside the reference
// tree.  Row-major storage, stride = NumCols (kStrideEqualNumCols, the
// reference default, src/matrix.cc:90-91).  MatMat / Quantize /
// MatMat_U8U8F32 are declared here and defined by the drop-in (src/linalg.cc)
// on the GPU, exactly as a reference build would take them from it.
#ifndef CATEARS_COMPAT_MATRIX_H_
#define CATEARS_COMPAT_MATRIX_H_

#include <assert.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "util.h"
#include "vector.h"

#define PK_MATRIX_SECTION "MAT0"

namespace pocketkaldi {

template <typename Real>
class SubMatrix;

template <typename Real>
class MatrixBase {
 public:
  enum { kTrans, kNoTrans };

  int NumRows() const { return num_rows_; }
  int NumCols() const { return num_cols_; }
  int Stride() const { return stride_; }
  Real *Data() { return data_; }
  const Real *Data() const { return data_; }

  Real &operator()(int r, int c) {
    assert(r < num_rows_ && c < num_cols_);
    return data_[(size_t)r * stride_ + c];
  }
  const Real operator()(int r, int c) const {
    assert(r < num_rows_ && c < num_cols_);
    return data_[(size_t)r * stride_ + c];
  }

  SubVector<Real> Row(int i) {
    assert(i < num_rows_);
    return SubVector<Real>(data_ + (size_t)i * stride_, num_cols_);
  }
  const SubVector<Real> Row(int i) const {
    assert(i < num_rows_);
    return SubVector<Real>(data_ + (size_t)i * stride_, num_cols_);
  }

  SubMatrix<Real> Range(int row_offset, int rows, int col_offset, int cols) const {
    return SubMatrix<Real>(*this, row_offset, rows, col_offset, cols);
  }

  void SetZero() {
    for (int r = 0; r < num_rows_; ++r) memset(data_ + (size_t)r * stride_, 0, sizeof(Real) * num_cols_);
  }
  void Scale(Real a) {
    for (int r = 0; r < num_rows_; ++r)
      for (int c = 0; c < num_cols_; ++c) data_[(size_t)r * stride_ + c] *= a;
  }
  void CopyFromMat(const MatrixBase<Real> &m, int trans = kNoTrans) {
    if (trans == kNoTrans) {
      assert(m.num_rows_ == num_rows_ && m.num_cols_ == num_cols_);
      for (int r = 0; r < num_rows_; ++r)
        if (num_cols_) memcpy(data_ + (size_t)r * stride_, m.data_ + (size_t)r * m.stride_, sizeof(Real) * num_cols_);
    } else {
      assert(m.num_rows_ == num_cols_ && m.num_cols_ == num_rows_);
      for (int r = 0; r < num_rows_; ++r)
        for (int c = 0; c < num_cols_; ++c) (*this)(r, c) = m(c, r);
    }
  }

 protected:
  MatrixBase() = default;
  MatrixBase(Real *data, int cols, int rows, int stride)
      : data_(data), num_cols_(cols), num_rows_(rows), stride_(stride) {}
  ~MatrixBase() = default;
  Real *data_ = nullptr;
  int num_cols_ = 0;
  int num_rows_ = 0;
  int stride_ = 0;
  friend class SubMatrix<Real>;
};

template <typename Real>
class Matrix : public MatrixBase<Real> {
 public:
  enum { kSetZero, kUndefined, kCopyData };
  enum { kDefaultStride, kStrideEqualNumCols };

  Matrix() = default;
  Matrix(int r, int c, int resize_type = kSetZero, int stride_type = kStrideEqualNumCols) {
    Resize(r, c, resize_type, stride_type);
  }
  Matrix(Matrix<Real> &&o) noexcept { Swap(&o); }
  Matrix<Real> &operator=(Matrix<Real> &&o) noexcept {
    Swap(&o);
    return *this;
  }
  ~Matrix() { free(this->data_); }

  void Resize(int r, int c, int resize_type = kSetZero, int stride_type = kStrideEqualNumCols) {
    (void)stride_type;
    assert(r >= 0 && c >= 0);
    Real *fresh = nullptr;
    const size_t n = (size_t)r * c;
    if (n) {
      const size_t bytes = (sizeof(Real) * n + 31) / 32 * 32;
      if (posix_memalign(reinterpret_cast<void **>(&fresh), 32, bytes) != 0) abort();
      if (resize_type != kUndefined) memset(fresh, 0, bytes);
      if (resize_type == kCopyData)
        for (int i = 0; i < std::min(r, this->num_rows_); ++i)
          memcpy(fresh + (size_t)i * c, this->data_ + (size_t)i * this->stride_,
                 sizeof(Real) * std::min(c, this->num_cols_));
    }
    free(this->data_);
    this->data_ = fresh;
    this->num_rows_ = r;
    this->num_cols_ = c;
    this->stride_ = c;
  }

  void Swap(Matrix<Real> *o) {
    std::swap(this->data_, o->data_);
    std::swap(this->num_rows_, o->num_rows_);
    std::swap(this->num_cols_, o->num_cols_);
    std::swap(this->stride_, o->stride_);
  }

  // MAT0 section (src/matrix.cc:159-191): "MAT0", i32 section (unchecked),
  // i32 rows, i32 cols, then `rows` VEC0 rows.
  Status Read(util::ReadableFile *fd) {
    PK_CHECK_STATUS(fd->ReadAndVerifyString(PK_MATRIX_SECTION));
    int32_t section = 0, rows = 0, cols = 0;
    PK_CHECK_STATUS(fd->ReadValue<int32_t>(&section));
    PK_CHECK_STATUS(fd->ReadValue<int32_t>(&rows));
    PK_CHECK_STATUS(fd->ReadValue<int32_t>(&cols));
    if (rows < 0 || cols < 0) return Status::Corruption("negative matrix shape in " + fd->filename());
    // The rows are collected as they are read and the matrix sized after the
    // last one, so storage never outgrows the file (a corrupt shape in the
    // billions fails as the truncated file it is, where the reference would
    // abort in posix_memalign) and every error is the reference's for the
    // same bytes.
    std::vector<Real> rows_read;
    Vector<Real> row;
    for (int r = 0; r < rows; ++r) {
      PK_CHECK_STATUS(row.Read(fd));
      if (row.Dim() != cols)
        return Status::Corruption(util::Format("Matrix::Read: row_read.Dim() == {} expected, but {} found: {}",
                                               cols, row.Dim(), fd->filename()));
      rows_read.insert(rows_read.end(), row.Data(), row.Data() + cols);
    }
    Resize(rows, cols, kUndefined);
    for (int r = 0; r < rows; ++r)
      if (cols) memcpy(this->Row(r).Data(), rows_read.data() + (size_t)r * cols, sizeof(Real) * cols);
    return Status::OK();
  }

 private:
  Matrix(const Matrix<Real> &) = delete;
  void operator=(const Matrix<Real> &) = delete;
};

template <typename Real>
class SubMatrix : public MatrixBase<Real> {
 public:
  SubMatrix(const MatrixBase<Real> &m, int ro, int r, int co, int c)
      : MatrixBase<Real>(const_cast<Real *>(m.Data()) + (size_t)ro * m.Stride() + co, c, r, m.Stride()) {
    assert(ro >= 0 && co >= 0 && ro + r <= m.NumRows() && co + c <= m.NumCols());
  }
  SubMatrix(Real *data, int rows, int cols, int stride) : MatrixBase<Real>(data, cols, rows, stride) {}
};

struct QuantizationParams {
  float scale;
  int32_t zero_point;
};

// Defined by the drop-in (GPU) -- src/linalg.cc.
void Quantize(const MatrixBase<float> &src, Matrix<uint8_t> *dest, QuantizationParams *params);
void MatMat(const MatrixBase<float> &A, const MatrixBase<float> &B, MatrixBase<float> *C);
void MatMat_U8U8F32(const MatrixBase<uint8_t> &A, const QuantizationParams &quant_params_A,
                    const MatrixBase<uint8_t> &B, const QuantizationParams &quant_params_B,
                    MatrixBase<float> *C);

// Naive triple loop (test helper, src/matrix.h:242-246).
template <typename Real>
void SimpleMatMat(const MatrixBase<Real> &A, const MatrixBase<Real> &B, MatrixBase<Real> *C) {
  assert(A.NumCols() == B.NumRows() && C->NumRows() == A.NumRows() && C->NumCols() == B.NumCols());
  for (int i = 0; i < A.NumRows(); ++i)
    for (int j = 0; j < B.NumCols(); ++j) {
      Real s = 0;
      for (int k = 0; k < A.NumCols(); ++k) s += A(i, k) * B(k, j);
      (*C)(i, j) = s;
    }
}

}  // namespace pocketkaldi

#endif  // CATEARS_COMPAT_MATRIX_H_
