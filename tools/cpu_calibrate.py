#!/usr/bin/env python3
"""Calibrate the CPU baseline port against reference code compiled here
(TEST / MEASUREMENT INFRASTRUCTURE; runs in the build container, where
/root/reference exists -- the GPU box has no reference, so the result is
committed as profiles/cpu_calibration.json and bench.py quotes it beside its
cpu_baseline).

The reference's hot path cannot be built here whole (matrix.cc needs
<cblas.h>).  What can be compared on one core, on the same
10 s synthetic utterance:
  * the real FFT: the reference's SRFFT::Compute (src/srfft.cc:370-459,
    compiled by oracle/Makefile into oracle/_ref/libref.so) against the
    oracle's restatement, on the utterance's 998 windowed frames;
  * the share of the port's per-utterance time that each stage takes
    (fbank, CMVN, nnet), so the FFT ratio can be weighed;
  * the nnet GEMM: the port's single-threaded sgemm (numpy / OpenBLAS, one
    thread) -- the reference's cblas_sgemm (src/matrix.cc:300-323) is the
    same BLAS call, so its rate is the library's, reported as GFLOP/s.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def best_of(fn, reps=5):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    from threadpoolctl import threadpool_limits

    from catears_amd import formats, synth
    from oracle import pyoracle
    ref = pyoracle.ref_lib()
    if ref is None:
        sys.exit("oracle/_ref/libref.so missing: run `make -C oracle` here (needs /root/reference)")
    conf = synth.write_model(os.path.join("/tmp", "catears_calib"), "tdnn-s")
    am = formats.read_am(conf)
    gstats = synth.cmvn_stats_synthetic()
    wave = synth.pcm(900000, 160000)
    frames = pyoracle.Fbank.num_frames(len(wave))
    # the windowed frames both FFTs see (any 512-float inputs time the same)
    rng = np.random.default_rng(1)
    wins = rng.standard_normal((frames, 512)).astype(np.float32) * 1000

    L = pyoracle.lib()
    oh = L.orc_srfft_new(512)
    rh = ref.ref_srfft_new(512)
    tmp = np.zeros(512, np.float32)
    work = wins.copy()

    import ctypes
    f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    L.orc_srfft_forward_n.argtypes = [ctypes.c_void_p, f32p, ctypes.c_int, f32p]
    ref.ref_srfft_forward_n.argtypes = [ctypes.c_void_p, f32p, ctypes.c_int, ctypes.c_int, f32p]

    def fft_port():
        L.orc_srfft_forward_n(oh, work, frames, tmp)

    def fft_ref():
        ref.ref_srfft_forward_n(rh, work, frames, 512, tmp)

    with threadpool_limits(limits=1):
        t_port, t_ref = best_of(fft_port), best_of(fft_ref)
        fb = pyoracle.Fbank()
        t_fbank = best_of(lambda: fb.compute(wave))
        feats = fb.compute(wave)
        t_cmvn = best_of(lambda: pyoracle.cmvn(gstats, feats))
        norm = pyoracle.cmvn(gstats, feats)
        t_nnet = best_of(lambda: pyoracle.am_whole(am, norm, gemm=lambda a, b: a @ b), reps=3)
        a = rng.standard_normal((1018, 3072)).astype(np.float32)
        w = rng.standard_normal((3072, 1024)).astype(np.float32)
        t_g = best_of(lambda: a @ w)
    L.orc_srfft_free(oh)
    ref.ref_srfft_free(rh)
    total = t_fbank + t_cmvn + t_nnet
    out = {
        "utterance": "10 s synthetic 16 kHz, 998 frames, TDNN-S, one core",
        "fft_port_us_per_frame": round(t_port / frames * 1e6, 3),
        "fft_reference_us_per_frame": round(t_ref / frames * 1e6, 3),
        "fft_port_over_reference_time": round(t_port / t_ref, 3),
        "port_stage_seconds": {"fbank": round(t_fbank, 4), "cmvn": round(t_cmvn, 4), "nnet": round(t_nnet, 4)},
        "port_stage_share": {"fbank": round(t_fbank / total, 4), "cmvn": round(t_cmvn / total, 4),
                             "nnet": round(t_nnet / total, 4)},
        "port_frames_per_s_one_core": round(frames / total, 1),
        "sgemm_gflops_one_thread": round(2 * 1018 * 3072 * 1024 / t_g / 1e9, 1),
        "reference_per_core_BASELINE_md": {"fbank_frames_per_s": "190-200 k (BASELINE.md:35)",
                                           "nnet_whole_utterance_frames_per_s": "2.5 k (BASELINE.md:37)"},
        "port_fbank_frames_per_s_one_core": round(frames / t_fbank, 1),
        "port_nnet_frames_per_s_one_core": round(frames / t_nnet, 1),
        "note": "FFT: both transforms looped in C over the same frames.  The nnet is the same cblas_sgemm "
                "call the reference makes (matrix.cc:300-323), through numpy's single-threaded OpenBLAS; "
                "the reference figures are the survey's, measured in this container",
    }
    path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
