/*
 * catears_gpu.h -- C-ABI boundary of the MI355X acoustic-scoring path.
 *
 * The reference (ishine/CatEars, a.k.a. pocketkaldi) computes
 *   PCM -> Fbank::Process -> CMVN::GetFrame -> AcousticModel::Process/EndOfStream
 *       -> Nnet::Propagate -> (- log prior) -> log-likelihood rows
 * on one CPU core, one frame at a time.  This header is the thin extern "C"
 * FFI under which the same path runs as hand-written gfx950 HIP kernels, on
 * whole utterances batched together.  Plain pointers, sizes and opaque
 * handles only; every entry point returns an int status (CE_GPU_OK == 0) and
 * never throws across the ABI.  The message of the last failure on the
 * calling thread is returned by ce_gpu_last_error().
 *
 * Pointers named d_* are device (HBM) pointers; h_* are host pointers.  All
 * device work is enqueued on the context's stream (asynchronous) unless a
 * function says otherwise.
 *
 * Reference interfaces replaced (all paths relative to the reference root):
 *   Fbank::Process            src/fbank.h:57-59,  src/fbank.cc:265-314
 *   CMVN::CMVN / GetFrame     src/cmvn.h:22-26,   src/cmvn.cc:100-119
 *   AcousticModel::Read       src/am.h:34-35,     src/am.cc:26-64
 *   AcousticModel::Process /
 *   EndOfStream / ComputeBatch src/am.h:41-47,    src/am.cc:82-164
 *   Nnet::Read / Propagate    src/nnet.h:229-232, src/nnet.cc:273-307
 *   MatMat (cblas_sgemm)      src/matrix.h:248-251, src/matrix.cc:300-323
 *   Quantize                  src/matrix.h:238-240, src/matrix.cc:366-387
 *   MatMat_U8U8F32            src/matrix.h:254-260, src/matrix.cc:389-420
 *   ce_stt_last_error         src/ce_stt.h:74-76 (per-thread here, not global)
 */
#ifndef CATEARS_GPU_H_
#define CATEARS_GPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CE_GPU_OK 0
#define CE_GPU_EINVAL (-2)    /* bad argument / shape (reference: assert)        */
#define CE_GPU_EHIP (-3)      /* HIP runtime error                                */
#define CE_GPU_EIO (-4)       /* cannot open / read a file (Status::IOError)      */
#define CE_GPU_ECORRUPT (-5)  /* malformed model/config (Status::Corruption)      */
#define CE_GPU_ENOTSUP (-6)   /* model topology this path does not run            */
#define CE_GPU_ENOMEM (-7)    /* device allocation failed (std::bad_alloc)        */

/* Feature geometry fixed at compile time in the reference (src/fbank.h:7-13). */
#define CE_GPU_FBANK_DIM 40
#define CE_GPU_FRAME_SHIFT 160
#define CE_GPU_FRAME_LENGTH 400

typedef struct ce_gpu_ctx ce_gpu_ctx;     /* device + stream + workspaces + fbank tables */
typedef struct ce_gpu_model ce_gpu_model; /* device-resident nnet, log prior, contexts   */
typedef struct ce_gpu_plan ce_gpu_plan;   /* geometry of one batch of utterances         */

/* Message of the last failure on this thread ("" if none). */
const char *ce_gpu_last_error(void);

/* Library version string, "catears-mi355x <abi> (gfx950)".  ABI history
 * (INTEGRATION.md §5): 0.1 round 1; 0.2 ce_gpu_loglik_gather gained `dim`
 * (argument 5) -- a caller built against 0.1 must be rebuilt; 0.3 adds the
 * int16 PCM entry points (ce_gpu_fbank_s16, ce_gpu_score_s16) and the fast
 * fbank mode (ce_gpu_ctx_set_fbank). */
const char *ce_gpu_version(void);

/* ------------------------------------------------------------ context --- */

/* Create a context on `device` that enqueues on `stream` (a hipStream_t; NULL
 * = the legacy default stream).  Builds the fbank tables on the host with the
 * reference's formulas (Hamming window src/fbank.cc:248-255, mel banks
 * src/fbank.cc:103-163, split-radix tables src/srfft.cc:74-122) and uploads
 * them once. */
int ce_gpu_ctx_create(int device, void *stream, ce_gpu_ctx **out);
int ce_gpu_ctx_destroy(ce_gpu_ctx *ctx);
/* Later calls enqueue on `stream`.  The switch is ordered: `stream` waits
 * (device-side, no host block) for everything already queued on the old
 * stream, which may still be using the context's workspaces -- so the old
 * stream must still be alive when this is called (switch first, destroy the
 * old stream afterwards; destroying a stream the context still uses is
 * undefined, as for any HIP call on a destroyed stream). */
int ce_gpu_ctx_set_stream(ce_gpu_ctx *ctx, void *stream);
/* Block the host until all work enqueued through ctx has finished. */
int ce_gpu_ctx_synchronize(ce_gpu_ctx *ctx);
/* Synchronizes ctx's stream, returns in *overflow whether an f16x3 GEMM
 * (CE_GPU_GEMM_F16X3) met an activation outside its range since the last
 * call, and clears the word.  When set, the log-likelihoods computed through
 * ctx since the last call are not fp32-accurate. */
int ce_gpu_ctx_overflow(ce_gpu_ctx *ctx, int *overflow);
/* Latency mode (on = 1) for callers that score small batches one at a time
 * -- the streaming AcousticModel::Process path (src/am.cc:115-142, a
 * chunk_size + left + right row block per call) or one utterance per call.
 * The fp32 nnet GEMMs of ctx (default bf16x6 mode) then split their K
 * dimension into slices -- at most 256 blocks of 64 output units per row
 * tile, at most 8 K-tiles of 32 per slice: TDNN-S 16 slices for its
 * 3072 x 1024 and 1024 x 1024 layers, 4 for 1024 x 3456 -- each slice loading
 * all its weights at once, and a second kernel sums the slices' partials in
 * slice order (for the last layer, inside the finalize launch).  The slice
 * count depends on K and N only, so results do not depend on the row count
 * and propagate_blocks still returns each block exactly the rows it gets
 * alone.  Results differ from the default mode's only by fp32 summation
 * order.  Measured on MI355X (TDNN-S, one stream): 92 us per 70-row chunk
 * (761 us in the default mode), 390 us per 1018-row utterance (780 us);
 * past ~2000 rows the default mode is faster.  Off (0, the default) is the
 * throughput mode for full 4096-row batches. */
int ce_gpu_ctx_set_latency(ce_gpu_ctx *ctx, int on);

/* Tile shape of ctx's throughput-mode bf16x6 GEMMs (round 5): on (1), every
 * layer runs the direct-weight kernel on 128 x 128 tiles -- twice the blocks
 * of the 256 x 128 default, so a hidden layer of a 4072-row batch fills all
 * 256 CUs (140 vs 202 us alone) at 38 % more CU time.  For a batch scored
 * while no other is in flight (a pipeline's first and last, or one batch on
 * an idle GPU); the default suits batches that share the chip.  Same bits
 * either way (tests/test_gpu_x6_variants.py).  Replaces nothing in the
 * reference (a scheduling choice of this implementation). */
int ce_gpu_ctx_set_wide_tiles(ce_gpu_ctx *ctx, int on);

/* Fbank kernel of ctx's ce_gpu_fbank / ce_gpu_fbank_s16 / ce_gpu_score*:
 *   CE_GPU_FBANK_EXACT (default) the reference's operation order
 *       (src/fbank.cc:44-245, src/srfft.cc:124-459): pre-log mel energies
 *       bit-identical to Fbank::Process, log-mel within 1e-5;
 *   CE_GPU_FBANK_FAST  the exact kernel's lane program built with FMA
 *       contraction and a single-precision pre-emphasis (23 % fewer
 *       instructions; C2 2.53 vs 2.26 G frames/s on one MI355X): log-mel within
 *       1e-4 of the reference on speech (and of its Kaldi dump), and as close
 *       to the exact float64 result as the reference's own fp32 order is
 *       (max 1.03e-4 vs the reference's 1.07e-4, p99.9 2.7e-5;
 *       tests/test_gpu_fbank_fast.py).  Deterministic: a frame's features
 *       do not depend on the batch it is computed in, nor on the kernels
 *       that run beside it on other streams (bit-identical to a serial
 *       re-score in the pipelined bench, tests/test_gpu_determinism.py;
 *       round 4's four-step fast kernel missed this in ~2 % of launches,
 *       DESIGN.md §8b). */
#define CE_GPU_FBANK_EXACT 0
#define CE_GPU_FBANK_FAST 1
int ce_gpu_ctx_set_fbank(ce_gpu_ctx *ctx, int mode);

/* Kernel timing for roofline reporting: while enabled, every launch of the
 * given kernel class is bracketed by a pair of HIP events on the context's
 * stream.  ce_gpu_ctx_profile_read synchronizes, returns the summed event
 * durations (ms) and launch count of the class since it was enabled, and
 * resets them.  Classes: 0 = TDNN GEMM, A operand in 16-byte vectors
 * (layers whose input width is a multiple of 32); 1 = TDNN GEMM, gathered A
 * (first layer); 2 = fbank; 3 = CMVN; 4 = log-softmax/prior finalize. */
#define CE_GPU_PROF_GEMM 0
#define CE_GPU_PROF_GEMM_GATHER 1
#define CE_GPU_PROF_FBANK 2
#define CE_GPU_PROF_CMVN 3
#define CE_GPU_PROF_FINALIZE 4
#define CE_GPU_PROF_QUANT 5 /* int8 path: per-layer min/max + quantize passes */
#define CE_GPU_PROF_CLASSES 6
int ce_gpu_ctx_profile(ce_gpu_ctx *ctx, int enable);
/* Restrict the timing to the classes whose bit (1 << class) is set in
 * `mask` (default: all).  Back-to-back GEMM launches of one call share their
 * boundary events, so timing only CE_GPU_PROF_GEMM costs one event record
 * per GEMM launch. */
int ce_gpu_ctx_profile_classes(ce_gpu_ctx *ctx, unsigned mask);
int ce_gpu_ctx_profile_read(ce_gpu_ctx *ctx, int kernel_class, double *total_ms, int64_t *launches);

/* Per-launch intervals for kernels that overlap across streams: record a
 * device-wide time origin on `stream` (before the launches of interest), then
 * read each launch's [start, end] in ms after it.  Consumes the records like
 * profile_read; fails with CE_GPU_EINVAL (and the needed *count) if capacity
 * is too small. */
int ce_gpu_profile_anchor(int device, void *stream);
int ce_gpu_ctx_profile_intervals(ce_gpu_ctx *ctx, int kernel_class, double *h_start_ms, double *h_end_ms,
                                 int capacity, int *count);

/* Window marker for an external kernel trace (rocprofv3 --kernel-trace):
 * launches one empty kernel, catears::trace_mark_kernel, of `tag` (1..64)
 * workgroups on `stream`.  bench.py marks the start (tag 1) and end (tag 2)
 * of its timed steps, and tools/trace_summary.py --window summarises only
 * the launches between the two.  Measurement plumbing; no reference
 * counterpart. */
int ce_gpu_trace_mark(int device, void *stream, int tag);

/* -------------------------------------------------------------- model --- */

/* AcousticModel::Read (src/am.cc:26-64): reads the key=value config (keys
 * nnet, prior, left_context, right_context, chunk_size, num_pdfs, tid2pdf;
 * relative paths resolved against the config's directory,
 * src/configuration.cc:52-66), the NN02 nnet (src/nnet.cc:221-293), the VEC0
 * prior (then log, src/am.cc:41-44) and the tid2pdf map; uploads weights.
 * Fails with CE_GPU_ENOTSUP for a topology whose whole-utterance result
 * would differ from the reference's chunked one. */
int ce_gpu_model_load_config(ce_gpu_ctx *ctx, const char *config_path, ce_gpu_model **out);

/* The same from explicit files; left/right context as AcousticModel reads
 * them from its config (src/am.cc:48-50). */
int ce_gpu_model_load(ce_gpu_ctx *ctx, const char *nnet_path, const char *prior_path,
                      int left_context, int right_context, ce_gpu_model **out);

/* Shape of a loaded model.  Any output pointer may be NULL. */
int ce_gpu_model_info(const ce_gpu_model *m, int *left_context, int *right_context,
                      int *input_dim, int *num_pdfs, int *num_linear, int64_t *num_params);

/* Switch a loaded model to the int8 path (BASELINE config C5): every
 * LinearLayer becomes Quantize + MatMat_U8U8F32 + bias (src/matrix.cc:329-420
 * -- the pieces the reference ships but never wires into Nnet,
 * src/nnet.cc:29).  Weights are quantized once here, per tensor; activations
 * per layer and per chunk of packed rows (the layer input block, before the
 * splice -- the same parameters as quantizing the spliced block); the int32
 * accumulation is exact (gemmlowp's ring), bias / ReLU / BatchNorm /
 * LogSoftmax stay fp32.  Irreversible for this model handle.
 * Batch dependence: like the reference's per-call Quantize, an activation
 * tensor's (scale, zero point) come from the whole block being scored, so in
 * ce_gpu_am_forward / ce_gpu_score an utterance's int8 log-likelihoods depend
 * on which utterances share its packed chunk.  ce_gpu_nnet_propagate_blocks
 * quantizes every block on its own instead, so there each block gets exactly
 * the rows it gets alone (the AcousticModel batcher's contract). */
int ce_gpu_model_quantize(ce_gpu_ctx *ctx, ce_gpu_model *m);

/* Matrix-core form of the fp32 Linear layers (LinearLayer::Propagate ->
 * MatMat -> cblas_sgemm, src/nnet.cc:22-36, src/matrix.cc:300-323):
 *   CE_GPU_GEMM_FP32   v_mfma_f32_32x32x2_f32 (exact fp32 products)
 *   CE_GPU_GEMM_BF16X6 every fp32 operand split exactly into three bf16
 *                      planes, six bf16 MFMA products per pair accumulated in
 *                      fp32; the dropped cross terms are < 2^-25 |w x|, below
 *                      one fp32 rounding, so the result is an fp32 GEMM
 *                      (differently ordered sum), on the 16x faster bf16
 *                      matrix cores.  Operands stay fp32 in HBM and are
 *                      split on their way into LDS.
 *   CE_GPU_GEMM_F16X3  every operand, scaled by a power of two, as two fp16
 *                      planes (22-23 significant bits), three fp16 MFMA
 *                      products in two fp32 accumulators; dropped term
 *                      < 2^-22 |w x|.  Log-likelihood error measured equal to
 *                      the FP32 path's.  Hidden activations must stay below
 *                      1.6e7 in magnitude (and finite): otherwise the
 *                      context's overflow word is set (ce_gpu_ctx_overflow)
 *                      and those results must be recomputed in another mode.
 * Models load in CE_GPU_GEMM_BF16X6 when their program allows it (every
 * Linear's input width after the first a multiple of 32, output widths
 * multiples of 4, every ReLU/BatchNorm fused into a Linear), else FP32.
 * F16X3 (22-23 significant bits per operand, not a full fp32 significand)
 * is opt-in.  Environment CATEARS_NNET_GEMM=fp32|bf16x6|bf16x6p|f16x3 overrides the
 * default.  Setting a mode the model does not allow returns CE_GPU_ENOTSUP. */
#define CE_GPU_GEMM_FP32 0
#define CE_GPU_GEMM_BF16X6 1
#define CE_GPU_GEMM_F16X3 2
/* BF16X6 with the operands kept as bf16 planes in HBM (each layer's
 * epilogue writes its output split; 6 B per element instead of 4).  The same
 * products in the same order as BF16X6: bit-identical results. */
#define CE_GPU_GEMM_BF16X6_PLANES 3
int ce_gpu_model_set_gemm(ce_gpu_model *m, int mode);
int ce_gpu_model_get_gemm(const ce_gpu_model *m, int *mode);

/* tid2pdf map (AcousticModel::TransitionPdfIdMap, src/am.h:38-40).  Copies
 * min(capacity, size) ints to h_out and returns the size via *size. */
int ce_gpu_model_tid2pdf(const ce_gpu_model *m, int32_t *h_out, int capacity, int *size);
int ce_gpu_model_destroy(ce_gpu_model *m);

/* Nnet::Read (src/nnet.cc:273-293) from an in-memory NN02 image (the bytes
 * Nnet::Read consumes).  h_prior (prior_dim probabilities, log taken as in
 * src/am.cc:40-44) may be NULL for a bare Nnet.  left/right_context < 0 take
 * the context from the network's Narrow layers; otherwise they must agree. */
int ce_gpu_model_load_mem(ce_gpu_ctx *ctx, const void *nnet, int64_t nbytes, const float *h_prior,
                          int prior_dim, int left_context, int right_context, ce_gpu_model **out);

/* Nnet::Read (src/nnet.cc:221-293) without a device: parses an NN02 image
 * exactly as ce_gpu_model_load_mem does -- CE_GPU_EIO "IOError: failed to
 * read: ..." for a truncated image (also for a section whose declared length
 * runs past the end, where the reference would first try to allocate it),
 * CE_GPU_ECORRUPT with the reference's messages for a wrong tag, a VEC0
 * section size, a MAT0 row width or an unknown layer type -- and reports the
 * layer count and the header's left / right context (any pointer may be
 * NULL).  Needs no GPU and touches none. */
int ce_gpu_nnet_check_mem(const void *nnet, int64_t nbytes, int *num_layers, int *left, int *right);

/* --------------------------------------------------------------- plan --- */

/* Frames of one utterance of n samples: 0 if n < 400 else 1 + (n - 400) / 160
 * (src/fbank.cc:35-42, snip-edges). */
int64_t ce_gpu_fbank_num_frames(int64_t num_samples);

/* Describe a batch of n_utt utterances laid out back to back in one PCM
 * buffer (utterance u starts at sample sum_{v<u} h_num_samples[v]).  Frames
 * and log-likelihood rows are laid out the same way (utterance u's rows start
 * at sum_{v<u} T_v).  If `model` is non-NULL the plan also packs the
 * utterances into nnet chunks of at most `max_rows` rows each (T_u + L + R
 * rows per utterance; longer utterances are split into segments that overlap
 * by L + R input rows, which the reference shows gives identical rows,
 * src/am.cc:73-80).  max_rows <= 0 selects 4096. */
int ce_gpu_plan_create(ce_gpu_ctx *ctx, const ce_gpu_model *model, const int64_t *h_num_samples,
                       int n_utt, int max_rows, ce_gpu_plan **out);
/* Totals of a plan; any output may be NULL. */
int ce_gpu_plan_info(const ce_gpu_plan *p, int *n_utt, int64_t *total_samples,
                     int64_t *total_frames, int *n_chunks, int *max_chunk_rows);
/* Per-utterance frame (= log-likelihood row) offsets, n_utt + 1 entries. */
int ce_gpu_plan_frame_offsets(const ce_gpu_plan *p, int64_t *h_out);
int ce_gpu_plan_destroy(ce_gpu_plan *p);

/* ------------------------------------------------------------ compute --- */

/* Fbank::Process over every utterance of the plan (one-shot, equivalent to
 * streaming, src/fbank.cc:265-314): d_pcm holds total_samples floats at raw
 * int16 scale (src/pcm_reader.cc:174); d_feats receives total_frames x 40
 * log-mel energies.  If d_mel is non-NULL the pre-log mel energies (same
 * shape) are written too (debug / parity). */
int ce_gpu_fbank(ce_gpu_ctx *ctx, const ce_gpu_plan *p, const float *d_pcm, float *d_feats,
                 float *d_mel);

/* The same from 16-bit PCM as it sits in a WAV payload (little-endian int16,
 * utterances back to back at the plan's sample offsets): the int16 -> float
 * conversion WaveReader::Process does on the host (src/pcm_reader.cc:148-190,
 * :174) happens in the kernel's loads, exactly, so the features are
 * bit-identical to ce_gpu_fbank on the converted floats -- at 2 B per sample
 * of HBM (and PCIe) traffic instead of 4. */
int ce_gpu_fbank_s16(ce_gpu_ctx *ctx, const ce_gpu_plan *p, const int16_t *d_pcm, float *d_feats,
                     float *d_mel);

/* Online CMVN (src/cmvn.cc:35-110) over every utterance: d_global_stats is
 * the 41-float VEC0 payload (40 sums + count); frames are processed in order
 * per utterance exactly like GetFrame(0), GetFrame(1), ...  d_out must not
 * overlap d_feats (the window subtracts frames read 600 steps earlier). */
int ce_gpu_cmvn(ce_gpu_ctx *ctx, const ce_gpu_plan *p, const float *d_global_stats,
                const float *d_feats, float *d_out);

/* AcousticModel::Process* + EndOfStream for every utterance of the plan:
 * d_feats is total_frames x input_dim; d_loglik receives total_frames x
 * num_pdfs rows of nnet output minus log prior (src/am.cc:104-112). */
int ce_gpu_am_forward(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p,
                      const float *d_feats, float *d_loglik);

/* Nnet::Propagate (src/nnet.cc:295-307) on one block of rows already padded
 * by the caller, optionally followed by AcousticModel::ComputeBatch's prior
 * subtraction (src/am.cc:104-112): d_in is rows x input_dim (row stride ld_in
 * floats), d_out receives (rows - L - R) x num_pdfs where L, R are the rows the
 * network's Narrow layers drop.  rows must exceed L + R (the reference's
 * Narrow passes shorter blocks through unchanged, src/nnet.cc:186-189; that
 * degenerate case is CE_GPU_EINVAL here). */
int ce_gpu_nnet_propagate(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *d_in, int rows, int ld_in,
                          int subtract_prior, float *d_out);

/* The same over n_blocks independent padded blocks laid back to back in d_in
 * (block b has h_rows[b] > L + R rows); d_out receives every block's
 * rows - L - R output rows back to back.  One launch sequence for all blocks:
 * the call a serving loop makes to score the ready chunks of many streams
 * at once (catears_amd/host AcousticModel batching).  Host-synchronous with
 * respect to the previous call on this context.  Every block's output equals
 * what ce_gpu_nnet_propagate gives for it alone (bit-exact; an int8 model
 * runs the blocks one by one so its quantization parameters stay per block). */
int ce_gpu_nnet_propagate_blocks(ce_gpu_ctx *ctx, const ce_gpu_model *m, const float *d_in, int ld_in,
                                 const int32_t *h_rows, int n_blocks, int subtract_prior, float *d_out);

/* The whole path: fbank -> (CMVN if d_global_stats != NULL) -> nnet -> - log
 * prior.  d_feats_ws must hold 2 x total_frames x 40 floats (features and
 * normalised features). */
int ce_gpu_score(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p,
                 const float *d_pcm, const float *d_global_stats, float *d_feats_ws,
                 float *d_loglik);

/* ce_gpu_score from 16-bit PCM (ce_gpu_fbank_s16 as its first stage). */
int ce_gpu_score_s16(ce_gpu_ctx *ctx, const ce_gpu_model *m, const ce_gpu_plan *p, const int16_t *d_pcm,
                     const float *d_global_stats, float *d_feats_ws, float *d_loglik);

/* ------------------------------------------------------- linear algebra --- */

/* MatMat (src/matrix.cc:300-323): C[m x n] = A[m x k] * B[k x n], all
 * row-major with leading dimensions lda/ldb/ldc (in floats), fp32 in, fp32
 * MFMA accumulate. */
int ce_gpu_sgemm(ce_gpu_ctx *ctx, int m, int n, int k, const float *d_a, int lda,
                 const float *d_b, int ldb, float *d_c, int ldc);

/* Quantize (src/matrix.cc:329-387): per-tensor asymmetric uint8 with the
 * reference's min/max (max initialised to FLT_MIN), scale = (max-min)/255
 * (double, stored float), zero point = round(-min/scale) unclamped.  d_q
 * receives count bytes; the parameters are written to d_params as
 * {float scale, int32 zero_point} (device, 8 bytes) so the call stays
 * asynchronous. */
int ce_gpu_quantize(ce_gpu_ctx *ctx, const float *d_x, int64_t count, uint8_t *d_q,
                    void *d_params);

/* MatMat_U8U8F32 (src/matrix.cc:389-420 -> gemmlowp EightBitIntGemm):
 * C[m x n] = float(int32 sum_k (A-zpA)(B-zpB)) * (sA*sB), A m x k and B k x n
 * row-major uint8, parameters read from the device records written by
 * ce_gpu_quantize.  The int32 accumulator is bit-exact. */
int ce_gpu_gemm_u8u8f32(ce_gpu_ctx *ctx, int m, int n, int k, const uint8_t *d_a,
                        const void *d_params_a, const uint8_t *d_b, const void *d_params_b,
                        float *d_c);

/* The same, int32 accumulators out (no scaling): the quantity gemmlowp's
 * GemmWithOutputPipeline produces before the float stage. */
int ce_gpu_gemm_u8u8i32(ce_gpu_ctx *ctx, int m, int n, int k, const uint8_t *d_a,
                        const void *d_params_a, const uint8_t *d_b, const void *d_params_b,
                        int32_t *d_c);

/* ------------------------------------------------------ layer primitives --- */
/* Single layers for Layer::Propagate (src/nnet.h:34-42) outside a fused
 * program.  All enqueue on the context's stream. */

/* LinearLayer::Propagate (src/nnet.cc:22-43): out = in * W + b, W in_dim x
 * out_dim row-major (MAT0 layout) with row stride ld_w; d_b may be NULL. */
int ce_gpu_linear(ce_gpu_ctx *ctx, int rows, int in_dim, int out_dim, const float *d_in, int ld_in,
                  const float *d_w, int ld_w, const float *d_b, float *d_out, int ld_out);

/* SpliceLayer::Propagate (src/nnet.cc:50-95): out (rows x dim*n_idx, dense)
 * row t = concat_s in[clamp(t + h_idx[s], 0, rows - 1)].  h_idx is host
 * memory, 1 <= n_idx <= CE_GPU_MAX_SPLICE. */
#define CE_GPU_MAX_SPLICE 32
int ce_gpu_splice(ce_gpu_ctx *ctx, int rows, int dim, const float *d_in, int ld_in, const int32_t *h_idx,
                  int n_idx, float *d_out);

/* In-place per-row layers: ReLU (src/nnet.cc:149-160), BatchNorm (x*scale
 * then +offset, :106-123), LogSoftmax (:137-146), Softmax, Normalize
 * (:163-178).  d_scale/d_offset only for BatchNorm. */
#define CE_GPU_ROW_RELU 0
#define CE_GPU_ROW_BATCHNORM 1
#define CE_GPU_ROW_LOGSOFTMAX 2
#define CE_GPU_ROW_SOFTMAX 3
#define CE_GPU_ROW_NORMALIZE 4
int ce_gpu_rowwise(ce_gpu_ctx *ctx, int op, int rows, int dim, float *d_x, int ld, const float *d_scale,
                   const float *d_offset);

/* Decoder::LogLikelihood (src/decoder.cc:97-102) in bulk, on the device:
 *   d_out[i] = am_scale * d_loglik[d_row[i] * ld + d_tid2pdf[d_trans[i]]]
 * for n (frame, transition-id) pairs -- the acoustic costs of a frame's
 * active arcs (ProcessEmitting, src/decoder.cc:327,350 negate them), so a
 * decoder reads n floats instead of whole 3456-wide rows.  `dim` is the row
 * width (num_pdfs, <= ld).  A pair whose frame is outside [0, rows), whose
 * transition id is outside [0, n_tid) or whose pdf (d_tid2pdf entry, e.g.
 * from a corrupt model file) is outside [0, dim) yields NaN (the reference
 * indexes out of bounds there). */
int ce_gpu_loglik_gather(ce_gpu_ctx *ctx, const float *d_loglik, int rows, int ld, int dim,
                         const int32_t *d_tid2pdf,
                         int n_tid, const int32_t *d_row, const int32_t *d_trans, int n, float am_scale,
                         float *d_out);

/* Column subset of a log-likelihood block: d_out[r * n_cols + j] =
 * d_loglik[r * ld + d_cols[j]] (NaN for a column outside [0, dim)) -- the
 * pdfs a decoding graph can reach, compacted before the D2H copy. */
int ce_gpu_loglik_columns(ce_gpu_ctx *ctx, const float *d_loglik, int rows, int ld, int dim,
                          const int32_t *d_cols, int n_cols, float *d_out);

/* *d_acc += the float64 sum of the n floats at d_x, on `stream` (a
 * hipStream_t; NULL = the null stream) of the current device; d_part is
 * device scratch for CE_GPU_SUM_PARTS doubles.  Each element is widened to
 * double before it is added.  Deterministic, not order-free: the summation
 * order depends on n, on whether d_x is 16-byte aligned (float4 or scalar
 * loads) and, in the _many form, on the whole list of buffers (the grid is
 * sized by the largest one and the buffers share per-thread accumulators) --
 * the same buffers at the same alignments give the same bits, the same rows
 * at another offset or folded with other buffers may differ in the last
 * places.  No reference counterpart: the consumer of the
 * log-likelihood rows gathered to rank 0 -- bench.py and
 * catears_amd/shard.py RowGather fold every row into this checksum, at HBM
 * speed where torch's float64 reduction runs at about a third of it. */
#define CE_GPU_SUM_PARTS 1024
int ce_gpu_sum_f64(void *stream, const float *d_x, int64_t n, double *d_part, double *d_acc);
/* The same over up to CE_GPU_SUM_MAX_BUFS buffers in one launch pair (host
 * arrays of device pointers and lengths): rank 0 folds every peer's rows of a
 * step at once, without a launch per peer. */
#define CE_GPU_SUM_MAX_BUFS 16
int ce_gpu_sum_f64_many(void *stream, int count, const float *const *d_x, const int64_t *n, double *d_part,
                        double *d_acc);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* CATEARS_GPU_H_ */
