// linalg.cc -- MatMat / Quantize / MatMat_U8U8F32 (reference
// src/matrix.cc:300-420) on the GPU.  A reference build takes these three
// definitions from here instead of matrix.cc.
#include <assert.h>

#include "catears_runtime.h"
#include "matrix.h"

namespace pocketkaldi {

using catears::host::Check;
using catears::host::Runtime;

static_assert(sizeof(QuantizationParams) == 8, "QuantizationParams must match the device record {float, int32}");

// C = A * B (cblas_sgemm RowMajor NoTrans NoTrans, alpha 1, beta 0).
void MatMat(const MatrixBase<float> &A, const MatrixBase<float> &B, MatrixBase<float> *C) {
  assert(A.NumCols() == B.NumRows() && A.NumRows() == C->NumRows() && B.NumCols() == C->NumCols());
  const int m = A.NumRows(), n = B.NumCols(), k = A.NumCols();
  if (m == 0 || n == 0) return;
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  float *da = static_cast<float *>(rt.scratch(0).Reserve(sizeof(float) * (size_t)m * (k ? k : 1)));
  float *db = static_cast<float *>(rt.scratch(1).Reserve(sizeof(float) * (size_t)(k ? k : 1) * n));
  float *dc = static_cast<float *>(rt.scratch(2).Reserve(sizeof(float) * (size_t)m * n));
  rt.Upload(da, k, A.Data(), A.Stride(), sizeof(float), m, k);
  rt.Upload(db, n, B.Data(), B.Stride(), sizeof(float), k, n);
  Check(ce_gpu_sgemm(rt.ctx(), m, n, k, da, k ? k : 1, db, n, dc, n), "MatMat");
  rt.Download(C->Data(), C->Stride(), dc, n, sizeof(float), m, n);
}

// Per-tensor asymmetric uint8 (src/matrix.cc:329-387); src is dense.
void Quantize(const MatrixBase<float> &src, Matrix<uint8_t> *dest, QuantizationParams *params) {
  assert(src.Stride() == src.NumCols());
  assert(src.NumCols() != 0 && src.NumRows() != 0);
  const size_t count = (size_t)src.NumRows() * src.NumCols();
  if (dest->NumCols() != src.NumCols() || dest->NumRows() != src.NumRows())
    dest->Resize(src.NumRows(), src.NumCols(), Matrix<uint8_t>::kUndefined);
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  float *dx = static_cast<float *>(rt.scratch(0).Reserve(sizeof(float) * count));
  uint8_t *dq = static_cast<uint8_t *>(rt.scratch(1).Reserve(count));
  void *dp = rt.scratch(2).Reserve(sizeof(QuantizationParams));
  rt.Upload(dx, count, src.Data(), count, sizeof(float), 1, count);
  Check(ce_gpu_quantize(rt.ctx(), dx, (int64_t)count, dq, dp), "Quantize");
  rt.Download(params, 1, dp, 1, sizeof(QuantizationParams), 1, 1);
  rt.Download(dest->Data(), dest->Stride(), dq, src.NumCols(), 1, src.NumRows(), src.NumCols());
}

// C = (sA*sB) * sum_k (A - zpA)(B - zpB), int32 exact (gemmlowp
// EightBitIntGemm, src/matrix.cc:389-420).  Like the reference, operands are
// addressed as dense (lda = K, ldb = ldc = N whatever their Stride()).
void MatMat_U8U8F32(const MatrixBase<uint8_t> &A, const QuantizationParams &quant_params_A,
                    const MatrixBase<uint8_t> &B, const QuantizationParams &quant_params_B,
                    MatrixBase<float> *C) {
  assert(A.NumCols() == B.NumRows() && A.NumRows() == C->NumRows() && B.NumCols() == C->NumCols());
  assert(A.NumCols() * A.NumRows() > 1 && B.NumCols() * B.NumRows() > 1);
  const int m = A.NumRows(), n = B.NumCols(), k = A.NumCols();
  Runtime &rt = Runtime::Get();
  std::lock_guard<std::mutex> lock(rt.mutex());
  uint8_t *da = static_cast<uint8_t *>(rt.scratch(0).Reserve((size_t)m * k));
  uint8_t *db = static_cast<uint8_t *>(rt.scratch(1).Reserve((size_t)k * n));
  float *dc = static_cast<float *>(rt.scratch(2).Reserve(sizeof(float) * (size_t)m * n));
  QuantizationParams *dp = static_cast<QuantizationParams *>(rt.scratch(3).Reserve(2 * sizeof(QuantizationParams)));
  const QuantizationParams both[2] = {quant_params_A, quant_params_B};
  rt.Upload(da, k, A.Data(), k, 1, m, k);
  rt.Upload(db, n, B.Data(), n, 1, k, n);
  rt.Upload(dp, 2, both, 2, sizeof(QuantizationParams), 1, 2);
  Check(ce_gpu_gemm_u8u8f32(rt.ctx(), m, n, k, da, dp, db, dp + 1, dc), "MatMat_U8U8F32");
  rt.Download(C->Data(), n, dc, n, sizeof(float), m, n);
}

}  // namespace pocketkaldi
