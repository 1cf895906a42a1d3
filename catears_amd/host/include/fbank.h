// fbank.h -- drop-in replacement for pocketkaldi's fbank.h (reference
// src/fbank.h:17-123): same Fbank / Fbank::Instance API, features computed on
// the MI355X by the fused framing + split-radix FFT + mel kernel
// (ce_gpu_fbank).  Streaming contract kept: samples not yet covered by a
// whole frame stay in the Instance until the next call (src/fbank.cc:265-314).
#ifndef CATEARS_PK_FBANK_H_
#define CATEARS_PK_FBANK_H_

#define PK_SAMPLERATE 16000
#define PK_FRAMESHIFT_MS 10.0
#define PK_FRAMELENGTH_MS 25.0
#define PK_FBANK_DIM 40
#define PK_FBANK_LOWFREQ 20
#define PK_FBANK_HIGHFREQ (PK_SAMPLERATE / 2)
#define PK_PREEMPH_COEFF 0.97

#include <vector>

#include "catears_runtime.h"
#include "matrix.h"
#include "vector.h"

namespace pocketkaldi {

class Fbank {
 public:
  class Instance;

  Fbank();
  ~Fbank();

  // Appends `wave` (16 kHz samples at raw int16 scale) to the stream and
  // writes every frame that is now complete to fbank_feature (T x 40).
  // Empty wave -> 0 x 40; fewer than 400 buffered samples -> 0 x 0.
  void Process(Instance *inst, const VectorBase<float> &wave, Matrix<float> *fbank_feature) const;

 private:
  Fbank(const Fbank &) = delete;
  Fbank &operator=(const Fbank &) = delete;
};

class Fbank::Instance {
 public:
  Instance() = default;

 private:
  friend class Fbank;
  std::vector<float> pending_;  // samples from the first incomplete frame on
};

}  // namespace pocketkaldi

#endif  // CATEARS_PK_FBANK_H_
