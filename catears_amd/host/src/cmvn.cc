// cmvn.cc -- online CMVN (reference src/cmvn.cc:35-119), all frames of the
// utterance normalised by one device pass at construction.
#include "cmvn.h"

#include <assert.h>
#include <string.h>

#include <memory>
#include <stdexcept>

#include "fbank.h"

namespace pocketkaldi {

using catears::host::Check;
using catears::host::Runtime;

CMVN::CMVN(const Vector<float> &global_stats, const Matrix<float> &raw_feats) {
  if (global_stats.Dim() != PK_FBANK_DIM + 1 || (raw_feats.NumRows() > 0 && raw_feats.NumCols() != PK_FBANK_DIM))
    throw std::invalid_argument("CMVN: expects 41 global stats and 40-dim features");
  num_frames_ = raw_feats.NumRows();
  normalized_.resize((size_t)num_frames_ * PK_FBANK_DIM);
  if (num_frames_ == 0) return;
  // a one-utterance plan whose frame count is num_frames_
  const int64_t samples = CE_GPU_FRAME_LENGTH + (int64_t)CE_GPU_FRAME_SHIFT * (num_frames_ - 1);
  Runtime::Lease lane = Runtime::Get().Acquire();
  ce_gpu_plan *raw = nullptr;
  Check(ce_gpu_plan_create(lane.ctx(), nullptr, &samples, 1, 0, &raw), "CMVN");
  std::unique_ptr<ce_gpu_plan, int (*)(ce_gpu_plan *)> plan(raw, ce_gpu_plan_destroy);
  const size_t n = (size_t)num_frames_ * PK_FBANK_DIM;
  float *d_in = static_cast<float *>(lane.scratch(0).Reserve(sizeof(float) * n));
  float *d_out = static_cast<float *>(lane.scratch(1).Reserve(sizeof(float) * n));
  float *d_stats = static_cast<float *>(lane.scratch(2).Reserve(sizeof(float) * (PK_FBANK_DIM + 1)));
  lane.Upload(d_in, PK_FBANK_DIM, raw_feats.Data(), raw_feats.Stride(), sizeof(float), num_frames_, PK_FBANK_DIM);
  lane.Upload(d_stats, PK_FBANK_DIM + 1, global_stats.Data(), PK_FBANK_DIM + 1, sizeof(float), 1, PK_FBANK_DIM + 1);
  Check(ce_gpu_cmvn(lane.ctx(), plan.get(), d_stats, d_in, d_out), "CMVN");
  lane.Download(normalized_.data(), PK_FBANK_DIM, d_out, PK_FBANK_DIM, sizeof(float), num_frames_, PK_FBANK_DIM);
}

CMVN::~CMVN() {}

void CMVN::GetFrame(int frame, VectorBase<float> *feats) {
  assert(frame == next_frame_ && "CMVN::GetFrame: frames must be requested in order");
  assert(frame >= 0 && frame < num_frames_ && feats->Dim() == PK_FBANK_DIM);
  memcpy(feats->Data(), normalized_.data() + (size_t)frame * PK_FBANK_DIM, sizeof(float) * PK_FBANK_DIM);
  next_frame_ = frame + 1;
}

}  // namespace pocketkaldi
