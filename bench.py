#!/usr/bin/env python3
"""Benchmark of the MI355X acoustic-scoring path (BASELINE.json configs[2]/[3]).

Workload (config C3 of SURVEY.md 8): the full am.cc pipeline -- fbank ->
online CMVN -> TDNN-S nnet (Splice/Linear/ReLU/BatchNorm x6, Linear 1024->3456,
LogSoftmax) -> minus log prior -- in fp32, one step = one packed frame batch of
at most 4096 rows = four 10 s synthetic 16 kHz utterances (4 x 998 = 3992
output frames, 4 x 1018 = 4072 packed rows).  PCM for a pool of utterances is
resident in HBM before timing; weights are random-init TDNN-S in the
reference's NN02 format (no model ships with the reference).

One process per GPU (torchrun); each rank scores its own utterances (weak
scaling); for N > 1 every rank's log-likelihood batch is gathered to rank 0
with RCCL over xGMI (torch.distributed "nccl"), overlapped with the next step.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for every field.
"""
import argparse
import json
import re
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)



def default_back_streams(workload):
    """nnet streams per process when --back-streams is not given: 8 for C3
    and C4, whose default GEMM (512 x 128 tiles, 64 blocks per hidden layer)
    needs more batches in flight to fill the chip (profiles/r06h_group_abc.txt:
    C3 with 8 streams + the last batch on wide tiles +2.3 % at the driver's
    flags over the 256 x 128 kernel on 3; profiles/r06i_streams.txt: C4
    6.65 M against 6.20 M on 3); 3 for C5, whose int8 GEMM runs 256 blocks
    per layer (4-8 streams: 17-19 M against 23 M)."""
    return 8 if workload in ("c3", "c4") else 3


def _early_arg(argv, name, default):
    """The value of `--name X` / `--name=X` in argv, before argparse runs (the
    hardware queue count must be set before torch initialises HIP)."""
    for i, a in enumerate(argv):
        if a == name and i + 1 < len(argv):
            return argv[i + 1]
        if a.startswith(name + "="):
            return a.split("=", 1)[1]
    return default


# Hardware queues per process (HIP default 4): one per stream of the
# pipeline -- the front stream, the nnet streams and the gather's
# communication stream -- so no two streams share a queue.  Set before torch
# initialises HIP.  (Measured, round 4: 8 queues with two front streams cost
# 5-6 % against 4 with one; CATEARS_HW_QUEUES overrides.)
_NB_EARLY = int(_early_arg(sys.argv, "--back-streams", default_back_streams(_early_arg(sys.argv, "--workload", "c3"))))
HW_QUEUES = int(os.environ.get("CATEARS_HW_QUEUES", str(max(4, _NB_EARLY + 2))))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(HW_QUEUES, 32))

FLOPS_PER_FRAME = 2 * (200 * 1024 + 4 * 3072 * 1024 + 1024 * 1024 + 1024 * 3456)  # 34,750,464
# FLOPs per output frame of the GEMMs timed as CE_GPU_PROF_GEMM (all but layer 1)
FLOPS_PER_FRAME_FAST = FLOPS_PER_FRAME - 2 * 200 * 1024
MFMA_F32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: dense fp32 MFMA (= vector) peak
MFMA_I8_PEAK_TOPS = 5000.0       # MI355X_MICROARCH.md: int8 MFMA = 2x the ~2.5 PF dense bf16 rate
MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense bf16 / fp16 (no sparsity)
# measured: v_mfma_f32_16x16x32_bf16 sustained on the whole chip with changing operands, at the
# socket power cap (profiles/r05z10_mfma_power.txt, tools/probes/mfma_power_probe.hip)
MFMA_BF16_SUSTAINED_TFLOPS = 1966.0
# Split-plane GEMMs (ce_gpu_model_set_gemm): bf16x6 issues six bf16 MFMA
# products per fp32 multiply-add, f16x3 three fp16 ones, so the kernel's
# ceiling in fp32 (algorithmic) FLOP/s is the 16-bit dense peak / products.
SPLIT_PRODUCTS = {"bf16x6": 6, "bf16x6p": 6, "f16x3": 3}
HBM_PEAK_GBS = 8000.0
METRIC = "acoustic frames/sec (fbank->nnet posteriors), 16kHz, 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)  # 0.15 s of GPU time at C3: steady state
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prewarm-ms", type=float, default=150.0,
                    help="C3/C5: before the W warm-up steps, untimed steps until this much wall time has passed "
                         "(the chip's clocks reach their loaded steady state in tens of ms; 0 = none)")
    ap.add_argument("--utts-per-step", type=int, default=None, help="default 4 (c3), 8 (c5)")
    ap.add_argument("--pool", type=int, default=32, help="distinct utterances resident per rank")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--model", default="tdnn-s")
    ap.add_argument("--no-cmvn", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--cpu-utts", type=int, default=32, help="distinct utterances in the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="minimum wall time of the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip the HIP-event kernel timing")
    ap.add_argument("--step-times", action="store_true",
                    help="C3: print each timed step's completion time (ms after the window opens) to stderr")
    ap.add_argument("--stage-profile", action="store_true",
                    help="time every kernel class (fbank, CMVN, splice, finalize) besides the GEMM; by default "
                         "only the GEMM launches carry events (one per launch), which the roofline needs")
    ap.add_argument("--serial", action="store_true", help="one stream: no front/back stage overlap")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL) for real runs; gloo only to rehearse N ranks on one GPU "
                         "together with CATEARS_BENCH_DEVICE")
    ap.add_argument("--workload", choices=["c3", "c2", "c4", "c5"], default="c3",
                    help="c3: full pipeline fp32 (the headline metric); c2: batched fbank only, "
                         "1000 x 10 s utterances per step; c4: the 100 h length-mixed corpus sharded over "
                         "the ranks, one pass (steps = each rank's batches), ragged batches gathered to "
                         "rank 0; c5: full pipeline with the int8 nnet path, frame batch 8192")
    ap.add_argument("--c4-utts", type=int, default=36000,
                    help="c4 corpus size in utterances (36000 = 100 h; smaller for tests)")
    ap.add_argument("--c4-dump", default=None,
                    help="c4, tests only: rank 0 writes every gathered row (and its own) per utterance "
                         "to this .npz (small corpora)")
    ap.add_argument("--c4-dump-every", type=int, default=1,
                    help="c4 with --c4-dump on one process: keep only utterances u with u %% K == 0 (the full "
                         "corpus, sampled)")
    ap.add_argument("--host-io", action="store_true",
                    help="c3: the PCIe-inclusive rate of a host-side caller -- every step's PCM is copied from "
                         "pinned host memory and its log-likelihoods back to pinned host memory, on copy streams "
                         "overlapped with the compute (DESIGN.md §6; never the headline value)")
    ap.add_argument("--fold-all", action="store_true",
                    help="c3, tests only: fold every row of every step (warm-up included) into the checksum "
                         "on the stream that scored it -- what rank 0's gather folds at N > 1")
    ap.add_argument("--c3-dump", default=None,
                    help="c3, tests only: write every step's log-likelihood rows (every rank its own, as "
                         "sent; rank 0 also every peer's, as received) to this .npz (.rankR.npz at N > 1)")
    ap.add_argument("--verify-serial", action="store_true",
                    help="c3, tests only: keep every batch's fbank / CMVN output and per-row log-likelihood sums as "
                         "the pipelined streams produced them, then re-score every batch serially on one stream "
                         "in the same process and report each difference (the line gains a 'verify' object)")
    ap.add_argument("--as-rank", type=int, default=None,
                    help="c3, tests only: use this rank's PCM pool (one process reproducing one rank)")
    ap.add_argument("--fbank", choices=["exact", "fast"], default="exact",
                    help="fbank kernel (ce_gpu_ctx_set_fbank): exact = the reference's operation order "
                         "(bit-exact pre-log mel), fast = the same lane program with FMA contraction (not bit-exact; as close to the exact result as the reference)")
    ap.add_argument("--pcm", choices=["f32", "s16"], default="f32",
                    help="resident PCM format: f32 (raw int16 scale floats, WaveReader's output) or s16 "
                         "(the WAV payload; ce_gpu_fbank_s16 converts exactly in the kernel)")
    ap.add_argument("--gemm", choices=["fp32", "bf16x6", "bf16x6p", "f16x3"], default=None,
                    help="matrix-core form of the fp32 Linear layers (ce_gpu_model_set_gemm); default: "
                         "the library's (bf16x6: three exact bf16 planes, six products, fp32 GEMM)")
    ap.add_argument("--front-streams", type=int, default=1,
                    help="fbank + CMVN streams; consecutive batches alternate between them")
    ap.add_argument("--wide-tiles", choices=["none", "last", "ends", "last2", "last4", "ends2"], default=None,
                    help="c3: score the last (or the first and the last, the last 2 / 4, the first 2 and last 2) batch(es) of each run "
                         "of steps on 128 x 128 bf16x6 tiles (ce_gpu_ctx_set_wide_tiles: all CUs per launch while "
                         "the pipeline drains); same bits.  Default: last for c3, none otherwise")
    ap.add_argument("--sink-share", type=float, default=None,
                    help="c3 / c4, N > 1: the fraction of steps (c4: of the corpus share) rank 0 scores a batch "
                         "of its own (it also receives and folds every peer's rows).  Default on RCCL: "
                         "min(1, 1.066 - 0.055 (N - 1)), at least 0.5 (rank 0's receive + fold load and a sender's "
                         "send read, measured by --rehearse-peers / --rehearse-send, DESIGN.md §7); 1 on gloo")
    ap.add_argument("--rehearse-peers", type=int, default=0,
                    help="c3, one process, measurement only: after each batch, copy it into K receive buffers "
                         "and fold all K+1 (ce_gpu_sum_f64) on a stream of its own -- rank 0's per-step receive "
                         "and fold load at N = K+1 ranks, on one GPU (the copies read and write locally, more "
                         "than the peers' remote writes cost rank 0)")
    ap.add_argument("--rehearse-send", action="store_true",
                    help="c3, one process, measurement only: read every batch once more after it is scored "
                         "(float64 fold on a stream of its own) -- a sender's local cost of handing its rows "
                         "to RCCL at N > 1")
    ap.add_argument("--launch-check", action="store_true",
                    help="tests only: start and check the N ranks (self-launch, world size, gloo process group) "
                         "and print a line with n_gpus and the ranks seen, without touching a GPU")
    ap.add_argument("--back-streams", type=int, default=None,
                    help="nnet streams; consecutive batches alternate between them so one batch's "
                         "wave-quantisation tail overlaps the next batch's layers (default: 8 for c3, 3 otherwise)")
    args = ap.parse_args(argv)
    if args.back_streams is None:
        args.back_streams = default_back_streams(args.workload)
    if args.wide_tiles is None:
        args.wide_tiles = "last" if args.workload == "c3" else "none"
    return args


def usable_cores():
    """Host cores this process may run on: the CPU affinity set, capped by
    the cgroup CPU quota (a GPU box's share of a larger machine: nproc and
    os.cpu_count() report the whole machine there).  Returns (cores, how)."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None and math.ceil(quota) < aff:
        return max(1, int(math.floor(quota))), f"cgroup CPU quota {quota:g} of {aff} CPUs in the affinity set"
    return aff, f"CPU affinity set ({aff} CPUs, no smaller cgroup quota)"


def cpu_baseline(conf, n_utts, seconds, threads, min_wall):
    """Oracle restatement ('port') of fbank -> CMVN -> nnet -> -log prior on the
    host cores: one utterance per worker thread, single-threaded OpenBLAS sgemm
    (numpy) inside each worker, like the reference's cblas_sgemm path.  Passes
    over the n_utts distinct utterances repeat until min_wall seconds of CPU
    work have run (a bounded sample of the same workload)."""
    from concurrent.futures import ThreadPoolExecutor

    from catears_amd import formats, synth
    from oracle import pyoracle
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:  # pragma: no cover
        threadpool_limits = None
    am = formats.read_am(conf)
    gstats = synth.cmvn_stats_synthetic()
    n = int(16000 * seconds)
    waves = [synth.pcm(900000 + i, n) for i in range(n_utts)]

    def one(w):
        fb = pyoracle.Fbank()
        f = pyoracle.cmvn(gstats, fb.compute(w))
        return pyoracle.am_whole(am, f, gemm=lambda a, b: a @ b).shape[0]

    ctxm = threadpool_limits(limits=1) if threadpool_limits else None
    try:
        one(waves[0][:16000])  # warm up
        frames, passes = 0, 0
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            while True:
                frames += sum(ex.map(one, waves))
                passes += 1
                if time.perf_counter() - t0 >= min_wall or passes >= 200:
                    break
        dt = time.perf_counter() - t0
    finally:
        if ctxm is not None:
            ctxm.__exit__(None, None, None)
    return frames / dt, frames, dt, passes


ROOFLINE_KERNEL = "gemm_f32_glds_kernel<catears::Cfg<128, 64, 32, 2, 2>, 2, false>"
# split-plane hidden layers (split output), the default variants
SPLIT_ROOFLINE_KERNEL = {
    # the default: the first layer gathered in the loader on 128 x 128 tiles
    # (gemm_bf16x6d_kernel), layers 2-7 on 512 x 128 (gemm_bf16x6w_kernel);
    # every launch of both templates
    "bf16x6": "gemm_bf16x6*",
    "bf16x6_160": "gemm_bf16x6f_kernel<catears::X6Cfg<128, 256, 2, 4, 2>, 8, 0, false>",
    "bf16x6p": "gemm_bf16x6q_kernel<catears::X6Cfg<128, 128, 4, 2, 3>, true, 0>",
    "f16x3": "gemm_f16x3_kernel<catears::X3Cfg<128, 128, 2, 4, 2, 64>, true>",
}
SPLIT_DTYPE = {
    "bf16x6": "fp32 (bf16x6 GEMM: fp32 operands split exactly into 3 bf16 planes, 6 MFMA products, fp32 "
              "accumulate; every operand bit kept, dropped cross terms < 2^-25 |w x|; error vs oracle at the "
              "fp32-MFMA path's level, tests/test_gpu_parity.py)",
    "bf16x6p": "fp32 (bf16x6 GEMM with the planes stored in HBM: same products and order as bf16x6, "
               "bit-identical results)",
    "f16x3": "fp32 (f16x3 GEMM: fp32 operands scaled by powers of two and split into 2 fp16 planes, 22-23 "
             "significant bits, 3 MFMA products in 2 fp32 accumulators; error vs oracle at the fp32-MFMA "
             "path's level, tests/test_gpu_parity.py)",
}
I8_ROOFLINE_KERNEL = "gemm_i8_pipe_kernel<256, 128, 3, 4, 2*"  # CATEARS_I8_GEMM default 16 (nnet_i8.hip), any STAG


def gemm_algorithmic_bytes(rows, layers=((3072, 1024),) * 4 + ((1024, 1024), (1024, 3456))):
    """fp32 A (rows x K) + W (K x N) + C (rows x N) bytes of TDNN-S layers 2-7,
    per launch on average (one launch per layer)."""
    return sum(4 * (rows * k + k * n + rows * n) for k, n in layers) / len(layers)


def split_algorithmic_bytes(rows, eb, layers=((256, 1024),) + ((3072, 1024),) * 4 + ((1024, 1024), (1024, 3456)),
                            hidden_only=False):
    """Split-plane GEMM operands per launch on average over TDNN-S layers
    1-7 (or the six hidden layers 1-6, whose launches are the split-output
    instantiation the PMC traffic is quoted for): A and W at eb bytes per
    element (6: three bf16 planes, 4: two fp16 planes or fp32 operands; A
    counted once per row and segment), hidden outputs written at eb bytes, the
    last as fp32."""
    if hidden_only:
        layers = layers[:-1]
    tot = 0
    for i, (k, n) in enumerate(layers):
        out = 4 if i == 6 else eb
        tot += eb * rows * k + eb * k * n + out * rows * n
    return tot / len(layers)


def kernel_match(name, kernel):
    """A profiled kernel name is `kernel`, or, for a `kernel` ending in '*',
    any instantiation that begins with it (e.g. every value of a trailing
    template argument)."""
    name = name.replace("catears::", "")
    kernel = kernel.replace("catears::", "")
    if kernel.endswith("*"):
        return kernel[:-1] in name
    return name.endswith(kernel)


def pmc_traffic(kernel, workload="c3"):
    """Per-launch HBM bytes of `kernel` from the newest committed PMC summary
    (tools/pmc_traffic.py over rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
    of this same bench and workload); None if there is none."""
    import glob
    pattern = "r*_pmc_traffic.json" if workload == "c3" else f"r*_{workload}_pmc_traffic.json"
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", pattern))
                   if workload != "c3" or not re.search(r"_c\d_pmc_traffic\.json$", f))
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    # every instantiation of the kernel (the default GEMM's first-layer form
    # is its own), weighted by dispatches: bytes per launch over all layers
    hits = [v for name, v in data.get("kernels", {}).items() if kernel_match(name, kernel)]
    if not hits:
        return None, None
    n = sum(v["dispatches"] for v in hits)
    return round(sum(v["hbm_bytes_per_launch"] * v["dispatches"] for v in hits) / n), os.path.relpath(files[-1], ROOT)


TDNN_S_GEMMS = ((200, 1024),) + ((3072, 1024),) * 4 + ((1024, 1024), (1024, 3456))  # (K, N) of layers 1-7


def pmc_traffic_layers(rows):
    """Per-layer PMC bytes of the C3 GEMM launches (tools/pmc_traffic.py
    --layers 7 over the serial PMC passes of this bench) beside each layer's
    algorithmic bytes: fp32 activations once per row and segment (4 rows K),
    the weights at 4 B (the fp32 matrix) and at 6 B (the bf16x6 fragment
    image the kernel reads), fp32 outputs (4 rows N).  None without the file."""
    import glob
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json"))
                   if not re.search(r"_c\d_pmc_traffic\.json$", f))
    for f in reversed(files):
        data = json.load(open(f))
        if "gemm_layers" not in data:
            continue
        out = []
        for L, (k, n) in zip(data["gemm_layers"], TDNN_S_GEMMS):
            alg = 4 * rows * k + 4 * k * n + 4 * rows * n
            alg6 = alg + 2 * k * n
            out.append({"layer": L["layer"], "k": k, "n": n, "pmc_bytes": L["hbm_bytes_per_launch"],
                        "algorithmic_bytes": alg, "algorithmic_bytes_fragment_image": alg6,
                        "pmc_over_algorithmic": round(L["hbm_bytes_per_launch"] / alg, 3),
                        "pmc_over_fragment_image": round(L["hbm_bytes_per_launch"] / alg6, 3)})
        return {"source": os.path.relpath(f, ROOT), "rows": rows, "layers": out}
    return None


def sink_share_default(world):
    """Rank 0's share of the scoring at `world` ranks on RCCL:
    from the one-GPU rehearsals, rank 0's step grows about 0.034 ms per peer
    whose rows it receives and folds (--rehearse-peers), a sender's about
    0.04 ms for handing its batch over (--rehearse-send), on a 0.61 ms step;
    equal step times give 1 + (0.04 - 0.034 (N - 1)) / 0.61."""
    return max(0.5, min(1.0, 1.066 - 0.055 * (world - 1)))


def pmc_valu(kernel):
    """Measured VALU occupancy of `kernel` in the C2 launch from the newest
    committed counter summary (tools/pmc_valu.py over one rocprofv3 --pmc
    pass of `bench.py --workload c2`, tools/round_gpu.sh); None if there is
    none or the kernel is not in it."""
    import glob
    base = kernel.split("<")[0]
    tmpl = kernel.split("<")[1].rstrip("*") if "<" in kernel else ""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_c2_pmc_valu.json")), reverse=True):
        data = json.load(open(f))
        for name, v in data.get("kernels", {}).items():
            if kernel_match(name, base + "*") and tmpl.split("*")[0] in name:
                return dict(v, source=os.path.relpath(f, ROOT),
                            definition="tools/pmc_valu.py: valu_active_per_simd = SQ_ACTIVE_INST_VALU / "
                                       "SQ_BUSY_CU_CYCLES; valu_busy_amd = AMD's VALUBusy; valu_issue_2cyc = "
                                       "SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x cycles); wave_* = fractions "
                                       "of SQ_WAVE_CYCLES")
    return None


def pmc_mfma(kernel, workload="c3"):
    """Matrix-pipe utilisation of `kernel` from the newest committed
    rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE summary
    (tools/pmc_mfma.py over a serial run of this bench and workload): the
    rocprof MFMA-utilisation figure the north star asks for, beside the
    event-timed roofline fraction.  None if there is none."""
    import glob
    pattern = "r*_pmc_mfma.json" if workload == "c3" else f"r*_{workload}_pmc_mfma.json"
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", pattern))
                   if workload != "c3" or not re.search(r"_c\d_pmc_mfma\.json$", f))
    if not files:
        return None
    data = json.load(open(files[-1]))
    hits = [v for name, v in data.get("kernels", {}).items() if kernel_match(name, kernel)]
    if hits:
        n = sum(v["dispatches"] for v in hits)
        avg = lambda key: round(sum(v[key] * v["dispatches"] for v in hits) / n, 4)
        out = {"chip": avg("mfma_util_chip"), "active_cus": avg("mfma_util_active_cus"),
               "source": os.path.relpath(files[-1], ROOT),
               "definition": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x SIMDs), serial run: chip = "
                             "1024 SIMDs, active_cus = 4 x the CUs the grid occupies; dispatch-weighted over "
                             "the instantiations in `per_instantiation`"}
        if len(hits) > 1:
            out["per_instantiation"] = {
                name.replace("catears::", ""): {"dispatches": v["dispatches"], "active_cus": v["mfma_util_active_cus"]}
                for name, v in data["kernels"].items() if kernel_match(name, kernel)}
        return out
    return None


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) with no launcher around this process: start the N
    ranks as ONE child process, `python -m torch.distributed.run
    --nproc-per-node N bench.py <same arguments>` on 127.0.0.1, echo its
    output and exit with its return code.  This process has not touched the
    GPU (no HIP call before here; the children initialise their own devices)
    and never replaces itself (no exec).  Returns rank 0's JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=ROOT)
    line = None
    for ln in p.stdout:
        sys.stdout.write(ln)
        sys.stdout.flush()
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                pass
    rc = p.wait()
    if rc != 0:
        raise SystemExit(rc)
    if line is None:
        raise SystemExit("bench.py: the ranks printed no JSON line")
    return line


def world_of(args):
    """(rank, world) from the launcher's environment.  The line's n_gpus is
    the world size, so a run whose world differs from --gpus fails here
    instead of reporting a mislabelled line."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world} (launch N ranks with "
                         f"torch.distributed.run --nproc-per-node N, or run --gpus N without a launcher)")
    return rank, world


def launch_check(args):
    """--launch-check: the ranks join a gloo process group and rank 0 prints
    the world it sees.  No GPU call (the CPU test of the N-rank launch)."""
    import torch
    import torch.distributed as dist
    rank, world = world_of(args)
    if world > 1:
        dist.init_process_group("gloo")
        ranks = [None] * world
        dist.all_gather_object(ranks, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", 0)),
                                       "pid": os.getpid()})
    else:
        ranks = [{"rank": 0, "local_rank": 0, "pid": os.getpid()}]
    line = {"metric": METRIC, "n_gpus": world, "launch_check": True, "ranks": ranks,
            "torch": torch.__version__}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return line


def device_for_rank():
    """LOCAL_RANK's GPU; CATEARS_BENCH_DEVICE pins every rank to one device
    (rehearsing N ranks on a one-GPU box with --dist-backend gloo)."""
    pinned = os.environ.get("CATEARS_BENCH_DEVICE")
    return int(pinned) if pinned is not None else int(os.environ.get("LOCAL_RANK", 0))


def init_dist(args, local):
    import torch
    import torch.distributed as dist
    if args.dist_backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(args.dist_backend)


def cpu_calibration():
    """The port against the reference, one core each, in the build container
    (tools/cpu_calibrate.py -> profiles/cpu_calibration.json): the port's
    FFT time over the reference's own srfft.cc compiled there, and the port's
    fbank / nnet rates beside the reference's (BASELINE.md:35-37)."""
    path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if not os.path.exists(path):
        return None
    c = json.load(open(path))
    return {"fft_port_over_reference_time": c["fft_port_over_reference_time"],
            "port_fbank_frames_per_s_one_core": c["port_fbank_frames_per_s_one_core"],
            "reference_fbank_frames_per_s_one_core": "190-200 k",
            "port_nnet_frames_per_s_one_core": c["port_nnet_frames_per_s_one_core"],
            "reference_nnet_frames_per_s_one_core": "2.5 k",
            # the nnet is ~99 % of the port's CPU time, so the whole-path
            # baseline is about this much below what the reference would give
            "port_over_reference_rate": round(c["port_nnet_frames_per_s_one_core"] / 2500.0, 2),
            "note": "the port's nnet runs ~16 % below the reference's per-core rate, so cpu_baseline.value "
                    "understates the reference's CPU throughput by about that much",
            "source": "profiles/cpu_calibration.json (tools/cpu_calibrate.py, build container, one core)"}


def cpu_fbank_baseline(n_utts, seconds, threads, min_wall):
    """Oracle fbank ('port') on the host cores, one utterance per worker."""
    from concurrent.futures import ThreadPoolExecutor

    from catears_amd import synth
    from oracle import pyoracle
    n = int(16000 * seconds)
    waves = [synth.pcm(700000 + i, n) for i in range(n_utts)]

    def one(w):
        return pyoracle.Fbank().compute(w).shape[0]

    one(waves[0][:16000])
    frames, passes = 0, 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while True:
            frames += sum(ex.map(one, waves))
            passes += 1
            if time.perf_counter() - t0 >= min_wall or passes >= 500:
                break
    dt = time.perf_counter() - t0
    return frames / dt, frames, dt, passes


def main_c2(args):
    """BASELINE.json config C2: batched fbank (window + SRFFT + mel + log)
    over 1000 x 10 s synthetic utterances resident in HBM, one launch per
    step.  Roofline: HBM, algorithmic bytes = 4 B x samples (PCM read once)
    + 160 B x frames (features written)."""
    import torch
    import torch.distributed as dist

    from catears_amd import gpu, synth
    rank, world = world_of(args)
    local = device_for_rank()
    torch.cuda.set_device(local)
    if world > 1:
        init_dist(args, local)
    n_utt, n_samp = 1000, int(16000 * args.seconds)
    stream = torch.cuda.current_stream()
    ctx = gpu.Context(local, stream)
    ctx.set_fbank(args.fbank)
    plan = gpu.Plan(ctx, [n_samp] * n_utt)
    s16 = args.pcm == "s16"
    pcm = torch.empty((n_utt, n_samp), dtype=torch.int16 if s16 else torch.float32, device="cuda")
    for u in range(n_utt):
        w = synth.pcm(rank * 100003 + u, n_samp)
        pcm[u].copy_(torch.from_numpy(w.astype(np.int16) if s16 else w))
    pcm = pcm.reshape(-1)
    feats = torch.empty((plan.total_frames, 40), dtype=torch.float32, device="cuda")
    prewarm_steps = 0
    torch.cuda.synchronize()
    tw = time.perf_counter()
    while (time.perf_counter() - tw) * 1e3 < args.prewarm_ms:  # as main(): the chip settled under load
        for _ in range(10):
            gpu.fbank(ctx, plan, pcm, feats)
        prewarm_steps += 10
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        gpu.fbank(ctx, plan, pcm, feats)
    torch.cuda.synchronize()
    if not args.no_profile:
        gpu.profile_anchor(local, stream)
        ctx.profile(True)
    if world > 1:
        dist.barrier()
    gpu.trace_mark(local, stream, 1)  # the timed window, for tools/trace_summary.py --window
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gpu.fbank(ctx, plan, pcm, feats)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gpu.trace_mark(local, stream, 2)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    checksum = float(feats.double().sum().item())
    iv = []
    if not args.no_profile:
        iv = ctx.profile_intervals(ctx.PROF_FBANK)
        ctx.profile(False)
    value = plan.total_frames * args.steps * world / elapsed
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    roofline = None
    bytes_per_launch = (2 if s16 else 4) * n_utt * n_samp + 4 * 40 * plan.total_frames
    if iv:
        avg_ms = sum(b - a for a, b in iv) / len(iv)
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
        kname = ("fbank_fma_kernel" if args.fbank == "fast" else "fbank_kernel") + ("<short*" if s16 else "<float*")
        traffic, src = pmc_traffic(kname, "c2")
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
                    "kernel": kname, "launches": len(iv), "avg_launch_ms": round(avg_ms, 4),
                    "algorithmic_bytes_per_launch": bytes_per_launch,
                    "valu_flops_per_frame": 14000}
        # what the kernel's SIMDs did, from the committed PMC pass of this
        # workload (the HBM figure above is the contract's named bound)
        valu = pmc_valu(kname)
        if valu is not None:
            roofline["valu_counters"] = valu
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        threads, how = usable_cores()
        v, fr, dt, passes = cpu_fbank_baseline(max(64, 2 * threads), args.seconds, threads, args.cpu_seconds)
        cpu = {"value": round(v, 1), "unit": "frames/s", "cores": threads, "kind": "port",
               "per_core": round(v / threads, 1), "cores_basis": how, "calibration": cpu_calibration(),
               "sample": f"{passes} passes over {max(64, 2 * threads)} x {args.seconds:g} s utterances ({fr} frames, "
                         f"{dt:.1f} s wall, {threads} worker threads): oracle fbank (C restatement of src/fbank.cc "
                         "+ srfft.cc)"}
    line = {
        "metric": "fbank frames/sec (window+SRFFT+mel+log, 25ms/10ms, 40 bins), 16kHz",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "prewarm": {"ms": args.prewarm_ms, "steps": prewarm_steps},
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (seeded 16 kHz PCM at raw int16 scale)",
        "config": {"workload": f"C2 batched fbank only, {n_utt} x {args.seconds:g} s utterances per step per GPU",
                   "pcm": "int16 (WAV payload)" if s16 else "float32 at raw int16 scale",
                   "fbank": args.fbank,
                   "frames_per_step_per_gpu": plan.total_frames, "parallelism": f"utterance shard x{world}"},
        "roofline": roofline, "cpu_baseline": cpu, "checksum": checksum,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main_c4(args):
    """BASELINE.json config C4: the 100 h corpus (36 000 seeded 2-18 s
    utterances, exactly 100 h of 16 kHz audio, catears_amd.shard.c4_corpus)
    sharded over the ranks by shard_utterances (longest-first greedy by
    frames), each rank packing its utterances into <= 4096-row batches and
    scoring them through fbank -> CMVN -> TDNN-S -> -log prior with the C3
    pipeline (one front and `back_streams` nnet streams).  Every rank's
    log-likelihood batches -- ragged: their row counts are exchanged once at
    setup -- stream to rank 0 over RCCL point-to-point (RowGather), where
    every row is folded into a checksum.  The timed region is one pass over
    the whole corpus (steps = the largest rank's batch count); PCM for every
    utterance is resident in HBM before it starts.  value = all ranks' frames
    / the slowest rank's time.  --c4-dump (tests) makes rank 0 keep every
    row it consumed, per utterance."""
    import torch
    import torch.distributed as dist

    from catears_amd import gpu, synth
    from catears_amd.shard import RowGather, c4_corpus, exchange_counts, num_frames, pack_batches, shard_utterances

    rank, world = world_of(args)
    local = device_for_rank()
    torch.cuda.set_device(local)
    if world > 1:
        init_dist(args, local)
    mdir = os.path.join(tempfile.gettempdir(), f"catears_bench_{os.getuid()}")
    if int(os.environ.get("LOCAL_RANK", 0)) == 0:
        synth.write_model(mdir, args.model)
    if world > 1:
        dist.barrier()
    conf = synth.write_model(mdir, args.model)

    NB = 1 if args.serial else max(1, args.back_streams)
    backs = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(NB - 1)]
    front = backs[0] if args.serial else torch.cuda.Stream()
    ctxs = [gpu.Context(local, b) for b in backs]
    ctx_f = ctxs[0] if args.serial else gpu.Context(local, front)
    ctx_f.set_fbank(args.fbank)
    model = gpu.Model(ctxs[0], conf)
    if args.gemm:
        model.set_gemm(args.gemm)
    L, R, pdfs = model.left, model.right, model.num_pdfs

    # corpus, shard, batches (all deterministic; the row counts are exchanged)
    samples = c4_corpus(args.c4_utts)
    frames = [num_frames(int(n)) for n in samples]
    # rank 0 receives and folds every peer's rows: on RCCL it takes a smaller
    # share of the corpus (the same rule as C3's --sink-share)
    share = 1.0
    if world > 1 and not args.no_gather:
        share = args.sink_share if args.sink_share is not None else (
            sink_share_default(world) if args.dist_backend == "nccl" else 1.0)
    mine = shard_utterances(frames, world, rank, weights=[share] + [1.0] * (world - 1))
    batches = [[mine[i] for i in b] for b in pack_batches([frames[u] for u in mine], L, R, 4096)]
    my_rows = [sum(frames[u] for u in b) for b in batches]
    if world > 1:
        everyone = exchange_counts([(b, r) for b, r in zip(batches, my_rows)])
    else:
        everyone = [list(zip(batches, my_rows))]
    counts = [[r for _, r in e] for e in everyone]
    steps = max(len(c) for c in counts)
    frames_all = sum(sum(c) for c in counts)

    # resident PCM: utterance u = the first n_u samples of pool signal u % P
    # (content depends on the utterance only, not on the rank or batching)
    P, plen = 48, int(samples.max())
    pool_np = np.stack([synth.pcm(600000 + i, plen) for i in range(P)])
    s16 = args.pcm == "s16"
    pool = torch.from_numpy(pool_np.astype(np.int16) if s16 else pool_np).cuda()
    tot = int(sum(int(samples[u]) for u in mine))
    pcm = torch.empty(max(tot, 1), dtype=pool.dtype, device="cuda")
    bstart, at = [], 0
    for b in batches:
        bstart.append(at)
        for u in b:
            n = int(samples[u])
            pcm[at:at + n].copy_(pool[u % P, :n])
            at += n
    plans = [gpu.Plan(ctxs[0], [int(samples[u]) for u in b], model, max_rows=4096) for b in batches]
    for pl, rows in zip(plans, my_rows):
        assert pl.total_frames == rows
    gstats = None if args.no_cmvn else torch.from_numpy(synth.cmvn_stats_synthetic()).cuda()
    maxf = max(my_rows) if my_rows else 1
    F = 2 * NB + 2 if not args.serial else 2
    raw = [torch.empty((maxf, 40), dtype=torch.float32, device="cuda") for _ in range(F)]
    norm = [torch.empty_like(raw[0]) for _ in range(F)] if gstats is not None else raw
    ready = [torch.cuda.Event() for _ in range(F)]
    free = [torch.cuda.Event() for _ in range(F)]
    nbuf = max(3, NB + 1)
    outs = [torch.empty((maxf, pdfs), dtype=torch.float32, device="cuda") for _ in range(nbuf)]
    done = [None] * nbuf
    gather = world > 1 and not args.no_gather
    dump = {} if (args.c4_dump and rank == 0) else None
    assert args.c4_dump_every == 1 or world == 1, "--c4-dump-every samples one process's own batches only"
    gat = RowGather(counts, pdfs, torch.float32, "cuda", depth=nbuf, keep=dump is not None) if gather else None
    comm = torch.cuda.Stream() if gather else None
    checksum = torch.zeros((), dtype=torch.float64, device="cuda")
    # one process: each nnet stream folds its own batches into its own
    # accumulator (ce_gpu_sum_f64; no two streams touch one)
    sums = [torch.zeros((), dtype=torch.float64, device="cuda") for _ in range(NB)]
    parts = [torch.empty(gpu.SUM_PARTS, dtype=torch.float64, device="cuda") for _ in range(NB)]

    def front_stage(i):
        slot = i % F
        front.wait_event(free[slot])
        pl = plans[i]
        src = pcm[bstart[i]:bstart[i] + pl.total_samples]
        gpu.fbank(ctx_f, pl, src, raw[slot][:pl.total_frames])
        if gstats is not None:
            gpu.cmvn(ctx_f, pl, gstats, raw[slot][:pl.total_frames], norm[slot][:pl.total_frames])
        ready[slot].record(front)

    def back_stage(i, s, timed):
        # i: this rank's batch, s: the gather step
        slot, o, b = i % F, i % nbuf, i % NB
        stream = backs[b]
        if gat is not None and timed:
            with torch.cuda.stream(stream):
                gat.wait_slot(s % nbuf)
        if done[o] is not None:
            stream.wait_event(done[o])
        stream.wait_event(ready[slot])
        n = plans[i].total_frames
        gpu.am_forward(ctxs[b], model, plans[i], norm[slot][:n], outs[o][:n])
        free[slot].record(stream)
        ev = torch.cuda.Event()
        ev.record(stream)
        done[o] = ev
        if not timed:
            return
        if gat is not None:
            with torch.cuda.stream(comm):
                comm.wait_event(ev)
                gat.submit(s, outs[o], own=outs[o][:n] if rank == 0 else None)
        else:
            # one process: consume every row the same way rank 0 does
            with torch.cuda.stream(stream):
                gpu.sum_f64(outs[o][:n], sums[b], parts[b])
        if dump is not None and (rank == 0) and any(int(u) % args.c4_dump_every == 0 for u in batches[i]):
            stream.synchronize()
            _c4_keep(dump, batches[i], frames, outs[o][:n].cpu().numpy(), args.c4_dump_every)

    def idle_step(s):
        # this rank has no batch at step s but peers may (rank 0 receives)
        if gat is not None:
            with torch.cuda.stream(comm):
                gat.submit(s, None)

    # warm-up: the first W batches, scored untimed and not gathered
    W = min(args.warmup, len(batches))
    if W:
        front_stage(0)
        for i in range(W):
            if i + 1 < W:
                front_stage(i + 1)
            back_stage(i, i, False)
    torch.cuda.synchronize()
    done = [None] * nbuf
    if not args.no_profile:
        gpu.profile_anchor(local, backs[0])
        for c in set(ctxs + [ctx_f]):
            c.profile(True, classes=None if args.stage_profile else [ctxs[0].PROF_GEMM])
    if world > 1:
        dist.barrier()
    gpu.trace_mark(local, backs[0], 1)  # the timed window, for tools/trace_summary.py --window
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if batches:
        front_stage(0)
    for s in range(steps):
        if s < len(batches):
            if s + 1 < len(batches):
                front_stage(s + 1)
            back_stage(s, s, True)
        else:
            idle_step(s)
    if gat is not None:
        with torch.cuda.stream(comm):
            gat.drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gpu.trace_mark(local, backs[0], 2)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if gat is not None:
        checksum += gat.checksum
    for v in sums:
        checksum += v
    rows_in = gat.rows_in if gat is not None else 0
    busy = None
    n_gemm = 0
    stages = None
    if not args.no_profile:
        iv = []
        for c in ctxs:
            iv += c.profile_intervals(c.PROF_GEMM)
        if args.stage_profile:
            # the front stream's share: fbank and CMVN run there, beside the
            # nnet streams' GEMMs; a stage only holds the pipeline back when
            # the front stream is busy most of the wall time
            stages = {}
            front = []
            for name, cs, cls in (("fbank", [ctx_f], ctx_f.PROF_FBANK), ("cmvn", [ctx_f], ctx_f.PROF_CMVN),
                                  ("finalize", ctxs, ctx_f.PROF_FINALIZE)):
                civ = [x for c in cs for x in c.profile_intervals(cls)]
                if cs == [ctx_f]:
                    front += civ
                if civ:
                    u = gpu.union_ms(civ)
                    stages[name] = {"launches": len(civ), "avg_ms": round(sum(b - a for a, b in civ) / len(civ), 4),
                                    "busy_ms": round(u, 3), "share_of_wall": round(u / (elapsed * 1e3), 4)}
            fu = gpu.union_ms(front) if front else 0.0
            stages["front_stream"] = {"busy_ms": round(fu, 3), "share_of_wall": round(fu / (elapsed * 1e3), 4)}
            if "cmvn" in stages and fu > 0:
                stages["cmvn"]["share_of_front_busy"] = round(stages["cmvn"]["busy_ms"] / fu, 4)
        for c in ctxs:
            c.profile(False)
        ctx_f.profile(False)
        n_gemm = len(iv)
        busy = gpu.union_ms(iv)
    if dump is not None and gat is not None:
        for p, st, rows in gat.keep:
            _c4_keep(dump, everyone[p][st][0], frames, rows)
    value = frames_all / elapsed
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if dump is not None:
        np.savez(args.c4_dump, **{f"u{u}": a for u, a in dump.items()})
    roofline = None
    if busy:
        peak = MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS.get(model.gemm, 1) if model.gemm != "fp32" else MFMA_F32_PEAK_TFLOPS
        achieved = sum(counts[0]) * FLOPS_PER_FRAME / (busy * 1e-3) / 1e12  # rank 0's frames, rank 0's GEMMs
        roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4), "traffic": None,
                    "kernel": "rank 0's nnet GEMM launches (every TDNN-S Linear), union of their intervals",
                    "launches": n_gemm, "busy_ms": round(busy, 3)}
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
        "steps": steps, "warmup": W, "ms_per_step": round(elapsed * 1e3 / max(steps, 1), 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": SPLIT_DTYPE.get(model.gemm, "fp32"),
        "data": "synthetic (seeded 16 kHz PCM, random-init TDNN-S in NN02 format)",
        "config": {"workload": f"C4 {args.c4_utts} x 2-18 s utterances ({int(samples.sum()) / 16000 / 3600:.3g} h), "
                               f"utterance shard x{world}, <= 4096-row batches, fbank->CMVN->{args.model}->loglik, "
                               + ("ragged log-likelihood batches gathered to rank 0 (RCCL p2p)" if gather else
                                  "no gather"),
                   "utterances": int(args.c4_utts), "frames_total": int(frames_all),
                   "frames_per_rank": [int(sum(c)) for c in counts], "batches_per_rank": [len(c) for c in counts],
                   "rows_gathered_to_rank0": int(rows_in), "pcm": args.pcm, "cmvn": not args.no_cmvn,
                   "parallelism": f"utterance shard x{world}", "streams": 1 if args.serial else 1 + NB,
                   "gather": gather, "sink_share": share if gather else None},
        "roofline": roofline, "cpu_baseline": None,
        "checksum": float(checksum.item()),
    }
    if stages is not None:
        line["stages"] = stages
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _c4_keep(dump, utts, frames, rows, every=1):
    """Split a batch's rows (utterances back to back) per utterance; keep
    utterances u with u % every == 0."""
    at = 0
    for u in utts:
        if int(u) % every == 0:
            dump[int(u)] = rows[at:at + frames[u]].copy()
        at += frames[u]
    assert at == rows.shape[0]


def verify_serial(args, kept, ctx, model, plan, pcm, gstats, U, pool):
    """Re-score every batch the pipelined run scored, one at a time on one
    stream, and compare bit for bit with what the pipeline produced: the
    fbank output, the CMVN output and each log-likelihood row's float64 sum.
    The reference is a deterministic CPU path (per-utterance state only,
    src/ce_stt.cc:53-60), so scheduling may not change a bit."""
    import torch

    from catears_amd import gpu
    torch.cuda.synchronize()
    ctx.set_fbank(args.fbank)  # the front contexts' fbank mode (the re-score runs on one context)
    if not kept:
        return {"batches": 0, "differing": 0, "detail": []}
    raw = torch.empty_like(kept[min(kept)][0])  # step 0 is not kept where rank 0 scores part of the steps
    norm = torch.empty_like(raw) if gstats is not None else raw
    out = torch.empty((plan.total_frames, model.num_pdfs), dtype=torch.float32, device="cuda")
    bad = []
    for i in sorted(kept):
        first = (i * U) % (pool - U + 1)
        gpu.fbank(ctx, plan, pcm[first:first + U].reshape(-1), raw)
        if gstats is not None:
            gpu.cmvn(ctx, plan, gstats, raw, norm)
        gpu.am_forward(ctx, model, plan, norm, out)
        sums = out.sum(1, dtype=torch.float64)
        praw, pnorm, psums = kept[i]
        d_raw = (praw.view(torch.int32) != raw.view(torch.int32))
        d_norm = (pnorm.view(torch.int32) != norm.view(torch.int32))
        d_sum = psums.view(torch.int64) != sums.view(torch.int64)
        if bool(d_raw.any()) or bool(d_norm.any()) or bool(d_sum.any()):
            rows = torch.nonzero(d_raw.any(1)).flatten().tolist()
            # where each differing frame ran: both modes build fbank.hip's
            # lane program -- 8 lanes per frame, 8 frames per wave, 8 waves
            # per block (one grid pass at C3)
            lanes, fpw, wpb = 8, 8, 8
            where = []
            for r in rows[:4]:
                bands = torch.nonzero(d_raw[r]).flatten().tolist()
                g = r % fpw
                where.append({"row": r, "block": r // (fpw * wpb), "wave": (r // fpw) % wpb, "group": g,
                              "lanes": [g * lanes, g * lanes + lanes - 1], "bands": bands,
                              "pipelined": [float(praw[r, b]) for b in bands[:3]],
                              "serial": [float(raw[r, b]) for b in bands[:3]]})
            bad.append({"step": i, "fbank_rows": rows[:8], "fbank_rows_n": len(rows), "fbank_where": where,
                        "fbank_bands": [torch.nonzero(d_raw[r]).flatten().tolist() for r in rows[:4]],
                        "cmvn_rows_n": int(d_norm.any(1).sum()), "loglik_rows_n": int(d_sum.sum()),
                        "loglik_first_row": int(torch.nonzero(d_sum).flatten()[0]) if bool(d_sum.any()) else None})
    return {"batches": len(kept), "differing": len(bad), "detail": bad[:16]}


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, sys.argv[1:] if argv is None else argv)
    world_of(args)
    if args.launch_check:
        return launch_check(args)
    if args.workload == "c2":
        return main_c2(args)
    if args.workload == "c4":
        return main_c4(args)
    import torch
    import torch.distributed as dist

    from catears_amd import gpu, synth
    from catears_amd.shard import RowGather, exchange_counts

    rank, world = world_of(args)
    local = device_for_rank()
    torch.cuda.set_device(local)
    if world > 1:
        init_dist(args, local)

    # synthetic TDNN-S model, written once per node
    mdir = os.path.join(tempfile.gettempdir(), f"catears_bench_{os.getuid()}")
    if int(os.environ.get("LOCAL_RANK", 0)) == 0:
        synth.write_model(mdir, args.model)
    if world > 1:
        dist.barrier()
    conf = synth.write_model(mdir, args.model)  # no-op once written

    # Software pipeline: a front stream runs fbank + CMVN of batch i+1 (a
    # handful of waves) beside the nnet GEMMs of batch i, and the nnet work of
    # consecutive batches alternates between `back_streams` streams so the
    # partial last wave of one batch's layers overlaps the next batch's.
    # Every batch is still scored end to end inside the timed region.
    NB = 1 if args.serial else max(1, args.back_streams)
    backs = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(NB - 1)]
    # --front-streams 2 alternates batches between two front streams (batch
    # 1's fbank + CMVN beside batch 0's); measured slower than one (6 %: the
    # second front stream's fbank blocks displace GEMM blocks from CUs)
    NF = 1 if args.serial else max(1, args.front_streams)
    fronts = [torch.cuda.Stream() for _ in range(NF)] if not args.serial else [backs[0]]
    ctxs = [gpu.Context(local, b) for b in backs]
    ctx = ctxs[0]
    ctx_fs = [gpu.Context(local, f) for f in fronts] if not args.serial else [ctx]
    for c in ctx_fs:
        c.set_fbank(args.fbank)
    int8 = args.workload == "c5"
    model = gpu.Model(ctx, conf)
    if args.gemm:
        model.set_gemm(args.gemm)
    split = None if int8 or model.gemm == "fp32" else model.gemm
    if int8:
        model.quantize(ctx)
    n_samp = int(16000 * args.seconds)
    U = args.utts_per_step or (8 if int8 else 4)
    max_rows = 8192 if int8 else 4096
    plan = gpu.Plan(ctx, [n_samp] * U, model, max_rows=max_rows)
    frames_per_step = plan.total_frames
    assert plan.n_chunks == 1, "a step must be one frame batch"

    # resident PCM pool (distinct utterances per rank)
    pool = max(args.pool, U)
    seed_rank = rank if args.as_rank is None else args.as_rank
    pcm_np = np.stack([synth.pcm(seed_rank * 100003 + i, n_samp) for i in range(pool)])
    pcm = torch.from_numpy(pcm_np.astype(np.int16) if args.pcm == "s16" else pcm_np).cuda()
    gstats = None if args.no_cmvn else torch.from_numpy(synth.cmvn_stats_synthetic()).cuda()
    # feature slots: NB being scored plus NB + 2 already featurised, so the
    # front stream runs a whole round of batches ahead and a stream that
    # finishes a batch finds the next one's features ready (with NB + 1 slots
    # the front waited for each batch's completion: a ~0.3 ms bubble per
    # round of NB batches, tools/timeline.py)
    F = 2 * NB + 2 if not args.serial else 2
    raw = [torch.empty((frames_per_step, 40), dtype=torch.float32, device="cuda") for _ in range(F)]
    norm = [torch.empty_like(raw[0]) for _ in range(F)] if gstats is not None else raw
    ready = [torch.cuda.Event() for _ in range(F)]
    free = [torch.cuda.Event() for _ in range(F)]
    nbuf = max(3, NB + 1)
    outs = [torch.empty((frames_per_step, model.num_pdfs), dtype=torch.float32, device="cuda")
            for _ in range(nbuf)]
    done = [None] * nbuf  # event: the batch that last wrote outs[o] has finished
    step_ev = None  # --step-times: the timed steps' completion events
    gather = world > 1 and not args.no_gather
    # every rank sends each of its batches (all rows) to rank 0, which folds
    # every received row into a checksum; the per-step row counts are
    # exchanged once here (equal at C3; C4's are ragged, main_c4)
    gat = None
    if gather:
        counts = exchange_counts([frames_per_step] * (args.warmup + args.steps))
        gat = RowGather(counts, model.num_pdfs, torch.float32, "cuda", depth=nbuf,
                        keep=bool(args.c3_dump) and rank == 0)
    comm = torch.cuda.Stream() if gather else None
    checksum = torch.zeros((), dtype=torch.float64, device="cuda")
    reh = None
    if args.rehearse_send and not args.rehearse_peers:
        assert world == 1 and not gather, "--rehearse-send rehearses a sender in one process"
        reh = {"stream": torch.cuda.Stream(), "done": [None] * nbuf, "recv": [],
               "src": None, "acc": torch.zeros((), dtype=torch.float64, device="cuda"),
               "part": torch.empty(gpu.SUM_PARTS, dtype=torch.float64, device="cuda")}
    if args.rehearse_peers:
        assert world == 1 and not gather, "--rehearse-peers rehearses rank 0 in one process"
        reh = {"stream": torch.cuda.Stream(), "done": [None] * nbuf,
               "recv": [torch.empty_like(outs[0]) for _ in range(args.rehearse_peers)],
               "src": torch.zeros_like(outs[0]),
               "acc": torch.zeros((), dtype=torch.float64, device="cuda"),
               "part": torch.empty(gpu.SUM_PARTS, dtype=torch.float64, device="cuda")}
    fold = [torch.zeros((), dtype=torch.float64, device="cuda") for _ in backs] if args.fold_all else None
    fold_parts = [torch.empty(gpu.SUM_PARTS, dtype=torch.float64, device="cuda") for _ in backs] if args.fold_all else None
    dump = {} if args.c3_dump else None  # step -> device copy of this rank's rows
    kept = {} if args.verify_serial else None  # step -> (fbank out, CMVN out, per-row sums) as pipelined
    # --host-io: a host caller's buffers.  PCM slots on the device are
    # refilled from pinned host memory on an upload stream; each batch's
    # log-likelihoods go back to a pinned host ring on a download stream,
    # and a batch may overwrite outs[o] only once its download has finished.
    hio = None
    if args.host_io:
        host_pcm = pcm.cpu().pin_memory()
        dev_pcm = [torch.empty((U,) + tuple(pcm.shape[1:]), dtype=pcm.dtype, device="cuda") for _ in range(F)]
        host_out = [torch.empty(tuple(outs[0].shape), dtype=torch.float32).pin_memory() for _ in range(nbuf)]
        hio = {"up": torch.cuda.Stream(), "down": torch.cuda.Stream(),
               "down_done": [None] * nbuf}

    # front slots (raw / norm / PCM buffers) go by the scored ordinal, not the
    # step: with a sink share below 1 the scored steps are not consecutive,
    # and front_stage(todo[k + 1]) runs before back_stage(todo[k]), so two
    # scored steps must never share a slot
    slot_of, n_scored = {}, [0]

    def front_stage(i):
        slot = slot_of[i]
        front, ctx_f = fronts[i % NF], ctx_fs[i % NF]
        front.wait_event(free[slot])  # the batch F steps ago has finished reading this slot
        first = (i * U) % (pool - U + 1)
        if hio is not None:
            up = hio["up"]
            up.wait_event(free[slot])  # the fbank F steps ago has read dev_pcm[slot]
            with torch.cuda.stream(up):
                dev_pcm[slot].copy_(host_pcm[first:first + U], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(up)
            front.wait_event(ev)
            src = dev_pcm[slot].reshape(-1)
        else:
            src = pcm[first:first + U].reshape(-1)
        gpu.fbank(ctx_f, plan, src, raw[slot])
        if gstats is not None:
            gpu.cmvn(ctx_f, plan, gstats, raw[slot], norm[slot])
        ready[slot].record(front)

    def back_stage(i):
        slot, o, b = slot_of[i], i % nbuf, i % NB
        stream = backs[b]
        if gat is not None:
            # the gather from nbuf steps ago has read outs[o]: only this
            # stream waits for it (work.wait() orders the current stream)
            with torch.cuda.stream(stream):
                gat.wait_slot(o)
        if done[o] is not None:
            stream.wait_event(done[o])  # the batch nbuf steps ago (maybe another stream) wrote outs[o]
        if reh is not None and reh["done"][o] is not None:
            stream.wait_event(reh["done"][o])  # the rehearsed receives have read outs[o]
        if hio is not None and hio["down_done"][o] is not None:
            stream.wait_event(hio["down_done"][o])  # ... and its log-likelihoods are on the host
        stream.wait_event(ready[slot])
        gpu.am_forward(ctxs[b], model, plan, norm[slot], outs[o])
        if fold is not None or kept is not None:
            # (before free[slot] is recorded: the front stream may refill
            # this slot as soon as it is)
            with torch.cuda.stream(stream):
                if fold is not None:
                    gpu.sum_f64(outs[o], fold[b], fold_parts[b])
                if dump is not None:
                    dump[i] = outs[o].clone()
                    if os.environ.get("CATEARS_DUMP_FEATS"):
                        dump[f"raw{i}"] = raw[slot].clone()
                        dump[f"norm{i}"] = norm[slot].clone()
                if kept is not None:
                    kept[i] = (raw[slot].clone(), norm[slot].clone(), outs[o].sum(1, dtype=torch.float64))
        free[slot].record(stream)
        ev = torch.cuda.Event(enable_timing=args.step_times)
        ev.record(stream)
        done[o] = ev
        if step_ev is not None and i >= args.warmup:
            step_ev.append(ev)
        if hio is not None:
            down = hio["down"]
            down.wait_event(ev)
            with torch.cuda.stream(down):
                host_out[o].copy_(outs[o], non_blocking=True)
            dv = torch.cuda.Event()
            dv.record(down)
            hio["down_done"][o] = dv
        if reh is not None:
            rs = reh["stream"]
            rs.wait_event(ev)
            with torch.cuda.stream(rs):
                if not os.environ.get("CATEARS_REHEARSE_NOCOPY"):
                    for r in reh["recv"]:
                        r.copy_(outs[o])
                # the step's rows as RowGather folds them: own + every peer's, one launch pair
                gpu.sum_f64_many([outs[o]] + reh["recv"], reh["acc"], reh["part"])
                rev = torch.cuda.Event()
                rev.record(rs)
                reh["done"][o] = rev
        if gat is not None:
            # the transfer is enqueued from a stream of its own that waits
            # for this batch only, so the nnet streams never wait on each
            # other through it
            with torch.cuda.stream(comm):
                comm.wait_event(ev)
                if dump is not None:
                    dump[i] = outs[o].clone()
                assert gat.submit(i, outs[o], own=outs[o] if rank == 0 else None) == o

    # rank 0 hosts the gather sink: at N > 1 it scores a batch on a share of
    # the steps only (evenly spread) and on the others just receives and
    # folds its peers' rows
    share = 1.0
    if gather and rank == 0:
        share = args.sink_share if args.sink_share is not None else (
            sink_share_default(world) if args.dist_backend == "nccl" else 1.0)
        assert 0.0 < share <= 1.0, "--sink-share must be in (0, 1]"
    elif reh is not None and args.sink_share is not None:
        share = args.sink_share  # the rehearsal of rank 0 at that share
        assert 0.0 < share <= 1.0, "--sink-share must be in (0, 1]"

    def rehearse_receive():
        # --rehearse-peers, a step that scores no batch of its own: the peers'
        # receives and their fold only (from a buffer the pipeline never writes)
        rs = reh["stream"]
        with torch.cuda.stream(rs):
            if not os.environ.get("CATEARS_REHEARSE_NOCOPY"):
                for r in reh["recv"]:
                    r.copy_(reh["src"])
            gpu.sum_f64_many(reh["recv"], reh["acc"], reh["part"])

    def scores(i):
        return share >= 1.0 or int((i + 1) * share) > int(i * share)

    def run(first, count):
        todo = [i for i in range(first, first + count) if scores(i)]
        for i in todo:
            slot_of[i] = n_scored[0] % F
            n_scored[0] += 1
        wide = set()
        if todo and args.wide_tiles != "none":
            tail = {"last2": 2, "last4": 4, "ends2": 2}.get(args.wide_tiles, 1)
            head = {"ends": 1, "ends2": 2}.get(args.wide_tiles, 0)
            wide = set(todo[-tail:]) | set(todo[:head])
        if todo:
            front_stage(todo[0])
        k = 0
        for i in range(first, first + count):
            if not scores(i):
                if gat is not None:  # rank 0: this step's receives only
                    with torch.cuda.stream(comm):
                        gat.submit(i, None)
                if reh is not None:
                    rehearse_receive()
                continue
            if k + 1 < len(todo):
                front_stage(todo[k + 1])
            if i in wide:
                ctxs[i % NB].set_wide_tiles(True)
            back_stage(i)
            if i in wide:
                ctxs[i % NB].set_wide_tiles(False)
            k += 1

    # pre-warm: the same steps, nothing gathered, dumped or folded, until the
    # chip has run the loaded pipeline for --prewarm-ms (profiles/r04h_step_times*:
    # after 5 warm-up steps the step cadence is still 5-10 % slower than after
    # 50); then the W warm-up steps proper
    prewarm_steps = 0
    if args.prewarm_ms > 0 and dump is None and kept is None and fold is None:
        gat_, gat = gat, None
        torch.cuda.synchronize()
        tw = time.perf_counter()
        while (time.perf_counter() - tw) * 1e3 < args.prewarm_ms:
            run(prewarm_steps, 10)
            prewarm_steps += 10
            torch.cuda.synchronize()
        gat = gat_
    run(0, args.warmup)
    if gat is not None:
        gat.drain()
    torch.cuda.synchronize()
    if not args.no_profile:
        gpu.profile_anchor(local, backs[0])
        for c in set(ctxs + ctx_fs):
            c.profile(True, classes=None if args.stage_profile or int8 else [ctx.PROF_GEMM])
    if world > 1:
        dist.barrier()
    gpu.trace_mark(local, backs[0], 1)  # the timed window, for tools/trace_summary.py --window
    torch.cuda.synchronize()
    step_ev = [] if args.step_times else None
    if step_ev is not None:
        win = torch.cuda.Event(enable_timing=True)
        win.record(fronts[0])
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    if gat is not None:
        gat.drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gpu.trace_mark(local, backs[0], 2)
    if step_ev is not None:
        print(json.dumps({"rank": rank, "wall_ms": round(elapsed * 1e3, 4),
                          "step_done_ms": [round(win.elapsed_time(e), 4) for e in step_ev]}), file=sys.stderr)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # the outputs are consumed (checksum) so no work can be elided
    if gat is not None:
        checksum += gat.checksum
    elif fold is not None:
        checksum += sum(fold)
    else:
        checksum += outs[(args.warmup + args.steps - 1) % nbuf].double().sum()
    finite = bool(torch.isfinite(outs[0]).all().item())
    if dump is not None:
        arrs = {(f"r{seed_rank}s{k}" if isinstance(k, int) else f"r{seed_rank}{k}"): v.cpu().numpy()
                for k, v in dump.items()}
        for p, st, a in (gat.keep or []) if gat is not None else []:
            arrs[f"r{p}s{st}"] = a
        np.savez(args.c3_dump if world == 1 else args.c3_dump.replace(".npz", f".rank{rank}.npz"), **arrs)
    verify = verify_serial(args, kept, ctx, model, plan, pcm, gstats, U, pool) if kept is not None else None
    verify_ranks = None
    if verify is not None and world > 1:
        verify_ranks = [None] * world
        dist.all_gather_object(verify_ranks, verify)
    # f16x3: no activation left the two-plane range in any batch
    overflow = any(c.overflow() for c in set(ctxs + ctx_fs))

    prof = {}
    if not args.no_profile:
        for c in set(ctxs + ctx_fs):
            c.profile(False)
        for name, cs, cls in (("gemm", ctxs, ctx.PROF_GEMM), ("gemm_gather", ctxs, ctx.PROF_GEMM_GATHER),
                              ("fbank", ctx_fs, ctx.PROF_FBANK), ("cmvn", ctx_fs, ctx.PROF_CMVN),
                              ("finalize", ctxs, ctx.PROF_FINALIZE), ("quantize", ctxs, ctx.PROF_QUANT)):
            iv = []
            for c in cs:
                iv += c.profile_intervals(cls)
            # (sum of launch durations, launches, wall time the class was on the device)
            prof[name] = (sum(b - a for a, b in iv), len(iv), gpu.union_ms(iv))

    my_steps = sum(1 for i in range(args.warmup, args.warmup + args.steps) if scores(i))
    total_frames = frames_per_step * my_steps
    if world > 1:
        t = torch.tensor([total_frames], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        total_frames = int(t.item())
    value = total_frames / elapsed
    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    roofline = None
    stages = {}
    if prof:
        ms, n, busy = prof["gemm"]
        if n and int8:
            # every Linear layer is one int8 GEMM launch (class GEMM)
            ops_per_launch = frames_per_step * FLOPS_PER_FRAME / (n / args.steps)
            achieved = ops_per_launch * n / (busy * 1e-3) / 1e12
            traffic, src = pmc_traffic(I8_ROOFLINE_KERNEL, "c5")
            roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": MFMA_I8_PEAK_TOPS,
                        "unit": "TOP/s", "frac": round(achieved / MFMA_I8_PEAK_TOPS, 4),
                        "traffic": traffic, "traffic_source": src,
                        "kernel": I8_ROOFLINE_KERNEL + " (TDNN-S layers 1-7)",
                        "launches": n, "avg_launch_ms": round(ms / n, 4), "busy_ms": round(busy, 3),
                        "effective_ms_per_launch": round(busy / n, 4), "ops_per_launch": ops_per_launch,
                        "pmc_mfma_util": pmc_mfma(I8_ROOFLINE_KERNEL, "c5")}
        elif n and split:
            # split-plane GEMM: every Linear (layer 1 included) is one launch
            # of class GEMM.  `achieved` counts the algorithmic fp32 FLOPs
            # (2 K N per frame); the kernel's ceiling is the 16-bit dense peak
            # over the MFMA products each fp32 multiply-add costs; over the
            # union of the launches' intervals as below.
            prods = SPLIT_PRODUCTS[split]
            peak = MFMA_BF16_PEAK_TFLOPS / prods
            flops_per_launch = frames_per_step * FLOPS_PER_FRAME / (n / args.steps)
            achieved = flops_per_launch * n / (busy * 1e-3) / 1e12
            # bf16x6 default: fp32 operands split on the way into LDS, one
            # kernel instantiation for every layer (CATEARS_X6_F32IN=0: the
            # plane-operand kernels, hidden layers in their split-output form)
            f32in = split == "bf16x6" and os.environ.get("CATEARS_X6_F32IN", "1") != "0"
            variant = os.environ.get("CATEARS_X6_VARIANT", "0")
            kname = SPLIT_ROOFLINE_KERNEL[("bf16x6_160" if variant == "160" else "bf16x6") if f32in else
                                          split if split != "bf16x6" else "bf16x6p"]
            traffic, src = pmc_traffic(kname)
            eb = 4 if f32in else {"bf16x6": 6, "bf16x6p": 6, "f16x3": 4}[split]
            roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1),
                        "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                        "peak_basis": f"{'fp16' if split == 'f16x3' else 'bf16'} dense MFMA "
                                      f"{MFMA_BF16_PEAK_TFLOPS:g} TFLOP/s / {prods} MFMA products per fp32 "
                                      "multiply-add (achieved = fp32 algorithmic FLOPs)",
                        "mfma_16bit_tflops": round(achieved * prods, 1),
                        "vs_fp32_mfma_peak": round(achieved / MFMA_F32_PEAK_TFLOPS, 4),
                        # the same work against the bf16 rate the chip sustains at its power cap
                        "frac_of_sustained_mfma": round(achieved * prods / MFMA_BF16_SUSTAINED_TFLOPS, 4),
                        "traffic": traffic, "traffic_source": src,
                        "kernel": kname + (" (every TDNN-S Linear, layers 1-7; rocprof: tools/trace_summary.py)"
                                           if f32in else " + its fp32-output form (TDNN-S layers 1-7; rocprof: "
                                           "tools/trace_summary.py 'kernel template' union)"),
                        "launches": n, "avg_launch_ms": round(ms / n, 4), "busy_ms": round(busy, 3),
                        "effective_ms_per_launch": round(busy / n, 4),
                        "flops_per_launch": flops_per_launch,
                        "pmc_mfma_util": pmc_mfma(kname),
                        "algorithmic_bytes_per_launch": split_algorithmic_bytes(plan.max_chunk_rows, eb),
                        "traffic_per_layer": pmc_traffic_layers(plan.max_chunk_rows) if f32in else None,
                        "traffic_scope": ("PMC bytes per launch averaged over all 7 layers (fp32 operands)" if f32in else
                                          "PMC bytes per hidden-layer launch (split-output instantiation, layers "
                                          "1-6); algorithmic bytes of the same launches: "
                                          f"{split_algorithmic_bytes(plan.max_chunk_rows, eb, hidden_only=True):.4g}")}
        elif n:
            # With several nnet streams, launches of this kernel overlap each
            # other; a launch's own duration then includes time shared with
            # its neighbour.  `achieved` is therefore the algorithmic FLOPs of
            # all launches over the wall time during which at least one was
            # running (the union of their intervals) -- with one stream this
            # is exactly FLOPs per launch / average launch duration.
            flops_per_launch = frames_per_step * FLOPS_PER_FRAME_FAST / (n / args.steps)
            achieved = flops_per_launch * n / (busy * 1e-3) / 1e12
            traffic, src = pmc_traffic(ROOFLINE_KERNEL)
            roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": MFMA_F32_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(achieved / MFMA_F32_PEAK_TFLOPS, 4),
                        "traffic": traffic, "traffic_source": src,
                        "kernel": ROOFLINE_KERNEL + " (TDNN-S layers 2-7)",
                        "launches": n, "avg_launch_ms": round(ms / n, 4), "busy_ms": round(busy, 3),
                        "effective_ms_per_launch": round(busy / n, 4),
                        "flops_per_launch": flops_per_launch,
                        "pmc_mfma_util": pmc_mfma(ROOFLINE_KERNEL),
                        "algorithmic_bytes_per_launch": gemm_algorithmic_bytes(plan.max_chunk_rows)}
        for name, (ms, n, busy) in prof.items():
            if n:
                stages[name] = {"launches": n, "avg_ms": round(ms / n, 4), "busy_ms": round(busy, 3),
                                "share_of_step": round(busy / (elapsed * 1e3), 4)}
        if "fbank" in stages:
            fb_bytes = 4 * U * n_samp + 4 * 40 * frames_per_step  # PCM read once + features written
            stages["fbank"]["hbm_GBs"] = round(fb_bytes / (stages["fbank"]["avg_ms"] * 1e-3) / 1e9, 1)
            stages["fbank"]["hbm_frac"] = round(stages["fbank"]["hbm_GBs"] / HBM_PEAK_GBS, 4)

    accuracy = None
    if int8:
        # C5's question: how far do int8 posteriors move from fp32 (one batch)
        m32 = gpu.Model(ctx, conf)
        first = 0
        src = pcm[first:first + U].reshape(-1)
        a = gpu.score(ctx, m32, plan, src, gstats).double()
        b = gpu.score(ctx, model, plan, src, gstats).double()
        torch.cuda.synchronize()
        accuracy = {"frames": int(a.shape[0]), "max_abs_diff": float((a - b).abs().max().item()),
                    "mean_abs_diff": float((a - b).abs().mean().item()),
                    "argmax_agreement": float((a.argmax(1) == b.argmax(1)).double().mean().item())}

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        threads, how = usable_cores()
        n_cpu = max(args.cpu_utts, 2 * threads)
        v, fr, dt, passes = cpu_baseline(conf, n_cpu, args.seconds, threads, args.cpu_seconds)
        cpu = {"value": round(v, 1), "unit": "frames/s", "cores": threads, "kind": "port",
               "per_core": round(v / threads, 1), "cores_basis": how, "calibration": cpu_calibration(),
               "sample": f"{passes} passes over {n_cpu} x {args.seconds:g} s utterances ({fr} frames, "
                         f"{dt:.1f} s wall, {threads} worker threads): oracle fbank+CMVN (C) + TDNN-S with "
                         f"single-threaded OpenBLAS sgemm per worker"}

    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "prewarm": {"ms": args.prewarm_ms, "steps": prewarm_steps},
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": ("u8 x u8 -> int32 (fp32 features, epilogues, log-softmax)" if int8 else
                  SPLIT_DTYPE[split] if split else "fp32"),
        "data": "synthetic (seeded 16 kHz PCM, random-init TDNN-S in NN02 format)",
        "config": {"workload": ("C5 full pipeline with the int8 nnet path (Quantize + MatMat_U8U8F32 per "
                                f"Linear), frame batch <= {max_rows} rows " if int8 else
                                f"C3 full pipeline fbank->CMVN->TDNN-S->loglik, frame batch <= {max_rows} rows ") +
                               f"({U} x {args.seconds:g} s utterances/step/GPU)" +
                               ("" if not gather else "; C4 RCCL gather of log-likelihoods to rank 0"),
                   "frames_per_step_per_gpu": frames_per_step, "packed_rows": plan.max_chunk_rows,
                   "cmvn": not args.no_cmvn, "fbank": args.fbank, "pcm": args.pcm, "parallelism": f"utterance shard x{world}",
                   "streams": 1 if args.serial else 1 + NB,
                   "gather": gather, "host_io": bool(args.host_io),
                   "sink_share": share if gather else None, "rank0_scored_steps": my_steps if gather else None,
                   "frames_total": total_frames},
        "roofline": roofline, "cpu_baseline": cpu, "stages": stages,
        "end_to_end_mfma_frac": round(value / world * FLOPS_PER_FRAME / 1e12 /
                                      (MFMA_I8_PEAK_TOPS if int8 else
                                       MFMA_BF16_PEAK_TFLOPS / SPLIT_PRODUCTS[split] if split else
                                       MFMA_F32_PEAK_TFLOPS), 4),
        "gemm_mode": "int8" if int8 else model.gemm,
        "int8_vs_fp32": accuracy,
        "checksum": float(checksum.item()), "finite": finite, "split_overflow": overflow,
    }
    if verify is not None:
        line["verify"] = verify
        if verify_ranks is not None:
            line["verify_ranks"] = verify_ranks
    if args.wide_tiles != "none":
        line["config"]["wide_tiles"] = {"last": "the last batch of each run of steps",
                                        "ends": "the first and the last batch of each run of steps",
                                        "last2": "the last 2 batches of each run of steps",
                                        "last4": "the last 4 batches of each run of steps",
                                        "ends2": "the first 2 and the last 2 batches of each run of steps"}[
            args.wide_tiles] + " on 128 x 128 bf16x6 tiles (ce_gpu_ctx_set_wide_tiles, same bits)"
    if args.rehearse_send and not args.rehearse_peers:
        line["rehearse_send"] = "every batch read once more after it is scored (a sender's local cost); measurement only"
    if args.rehearse_peers:
        line["rehearse_peers"] = {"peers": args.rehearse_peers,
                                  "what": "rank 0's receive copies and float64 folds of N = peers + 1 ranks, "
                                          "on a stream of its own; measurement only"}
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return line


if __name__ == "__main__":
    main()
