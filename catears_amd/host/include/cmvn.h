// cmvn.h -- drop-in replacement for pocketkaldi's cmvn.h (reference
// src/cmvn.h:17-43): online CMVN with a 600-frame window smoothed by 200
// global frames.  The constructor normalises every frame of the utterance in
// one device pass (ce_gpu_cmvn, one lane per (utterance, dim) chain, bit-exact
// with src/cmvn.cc:35-110); GetFrame hands them out in the reference's
// sequential order.
#ifndef CATEARS_PK_CMVN_H_
#define CATEARS_PK_CMVN_H_

#include <stdint.h>

#include <vector>

#include "catears_runtime.h"
#include "matrix.h"
#include "util.h"

#define PK_ONLINECMVN_WINDOW 600
#define PK_ONLINECMVN_GLOBALFRAMES 200

namespace pocketkaldi {

class CMVN {
 public:
  // global_stats: 41 values (40 sums + frame count, cmvn_stats.bin);
  // raw_feats: T x 40 fbank features.  Both are copied.
  CMVN(const Vector<float> &global_stats, const Matrix<float> &raw_feats);
  ~CMVN();

  // Normalised frame `frame`; frames must be requested 0, 1, 2, ... as the
  // reference requires (src/cmvn.cc:38).
  void GetFrame(int frame, VectorBase<float> *feats);

 private:
  std::vector<float> normalized_;  // T x 40
  int num_frames_ = 0;
  int next_frame_ = 0;
  CMVN(const CMVN &) = delete;
  CMVN &operator=(const CMVN &) = delete;
};

}  // namespace pocketkaldi

#endif  // CATEARS_PK_CMVN_H_
