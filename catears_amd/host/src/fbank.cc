// fbank.cc -- Fbank::Process on the GPU (reference src/fbank.cc:265-314).
#include "fbank.h"

#include <memory>

namespace pocketkaldi {

using catears::host::Check;
using catears::host::Runtime;

Fbank::Fbank() {}
Fbank::~Fbank() {}

void Fbank::Process(Instance *inst, const VectorBase<float> &wave, Matrix<float> *fbank_feature) const {
  if (wave.Dim() == 0) {  // src/fbank.cc:269-273
    fbank_feature->Resize(0, PK_FBANK_DIM);
    return;
  }
  std::vector<float> &buf = inst->pending_;
  buf.insert(buf.end(), wave.Data(), wave.Data() + wave.Dim());
  const int64_t samples = (int64_t)buf.size();
  const int64_t frames = ce_gpu_fbank_num_frames(samples);
  if (frames == 0) {  // src/fbank.cc:283-287
    fbank_feature->Resize(0, 0);
    return;
  }
  fbank_feature->Resize((int)frames, PK_FBANK_DIM, Matrix<float>::kUndefined);
  {
    Runtime::Lease lane = Runtime::Get().Acquire();
    ce_gpu_plan *raw = nullptr;
    Check(ce_gpu_plan_create(lane.ctx(), nullptr, &samples, 1, 0, &raw), "Fbank::Process");
    std::unique_ptr<ce_gpu_plan, int (*)(ce_gpu_plan *)> plan(raw, ce_gpu_plan_destroy);
    float *d_pcm = static_cast<float *>(lane.scratch(0).Reserve(sizeof(float) * samples));
    float *d_feat = static_cast<float *>(lane.scratch(1).Reserve(sizeof(float) * frames * PK_FBANK_DIM));
    lane.Upload(d_pcm, samples, buf.data(), samples, sizeof(float), 1, samples);
    Check(ce_gpu_fbank(lane.ctx(), plan.get(), d_pcm, d_feat, nullptr), "Fbank::Process");
    lane.Download(fbank_feature->Data(), fbank_feature->Stride(), d_feat, PK_FBANK_DIM, sizeof(float), frames,
                  PK_FBANK_DIM);
  }
  // keep the samples from the first frame not emitted (src/fbank.cc:305-313)
  buf.erase(buf.begin(), buf.begin() + frames * CE_GPU_FRAME_SHIFT);
}

}  // namespace pocketkaldi
