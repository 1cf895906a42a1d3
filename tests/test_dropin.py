"""The drop-in pocketkaldi classes (catears_amd/host: fbank.h, cmvn.h, nnet.h,
am.h, MatMat/Quantize/MatMat_U8U8F32) used the way the reference's callers use
them, through tests/native/pk_dropin.cc, against the oracle.

CPU tests: the reference's own callers (src/ce_stt.cc, src/decoder.cc) compile
against the drop-in headers, and the drop-in sources compile against the
reference's container headers -- the "drops straight into decoder.cc" claim
 checked by the compiler.  Skipped where /root/reference is
absent (the GPU box).

GPU tests: same bars as test_gpu_parity.py -- bit-exact for CMVN / Quantize /
the u8 GEMM, FEAT_TOL for log-mel features, 1e-4 for nnet outputs.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

REF_SRC = "/root/reference/src"
DRIVER = os.path.join(ROOT, "catears_amd", "lib", "pk_dropin")
PKLIB = os.path.join(ROOT, "catears_amd", "lib", "libcatears_pk.so")
HOST_INC = os.path.join(ROOT, "catears_amd", "host", "include")
LOGLIK_TOL = 1e-4
FEAT_TOL = 1e-5
REPLACED = {"fbank.h", "cmvn.h", "nnet.h", "am.h", "fbank.cc", "cmvn.cc", "nnet.cc", "am.cc"}


# ------------------------------------------------------------ CPU checks --

def _overlay(tmp_path):
    """The reference src/ tree with the four replaced hot-path files taken
    out (symlinks, nothing copied): what a maintainer's tree looks like after
    dropping the catears headers in."""
    ov = tmp_path / "src"
    ov.mkdir()
    for name in os.listdir(REF_SRC):
        p = os.path.join(REF_SRC, name)
        if os.path.isfile(p) and name not in REPLACED and name.endswith((".h", ".cc")):
            os.symlink(p, ov / name)
    return ov


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree not present")
@pytest.mark.parametrize("caller", ["ce_stt.cc", "decoder.cc"])
def test_reference_callers_compile_against_dropin(tmp_path, caller):
    ov = _overlay(tmp_path)
    cmd = ["g++", "-std=c++11", "-fsyntax-only", "-I" + HOST_INC, "-I" + os.path.join(ROOT, "include"),
           "-I" + str(ov), "-I" + os.path.join(REF_SRC, "openfst", "include"), str(ov / caller)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    # and the headers it saw were the drop-in ones
    r = subprocess.run(cmd + ["-H"], capture_output=True, text=True)
    seen = [ln.split()[-1] for ln in r.stderr.splitlines() if ln.startswith(".")]
    for h in ("am.h", "fbank.h", "nnet.h"):
        hits = [s for s in seen if os.path.basename(s) == h]
        if hits:
            assert all(s.startswith(HOST_INC) for s in hits), hits


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference tree not present")
def test_dropin_sources_compile_against_reference_containers(tmp_path):
    ov = _overlay(tmp_path)
    src = os.path.join(ROOT, "catears_amd", "host", "src")
    for f in sorted(os.listdir(src)):
        cmd = ["g++", "-std=c++11", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__", "-I" + HOST_INC,
               "-I" + os.path.join(ROOT, "include"), "-I" + str(ov), "-I/opt/rocm/include",
               os.path.join(src, f)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, (f, r.stderr[-4000:])


def test_dropin_library_exports_the_reference_api():
    if not os.path.exists(PKLIB):
        pytest.skip("libcatears_pk.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-DC", "--defined-only", PKLIB], capture_output=True, text=True).stdout
    for sym in ["pocketkaldi::Fbank::Process(pocketkaldi::Fbank::Instance*, pocketkaldi::VectorBase<float> const&, "
                "pocketkaldi::Matrix<float>*) const",
                "pocketkaldi::CMVN::GetFrame(int, pocketkaldi::VectorBase<float>*)",
                "pocketkaldi::CMVN::CMVN(pocketkaldi::Vector<float> const&, pocketkaldi::Matrix<float> const&)",
                "pocketkaldi::Nnet::Read(pocketkaldi::util::ReadableFile*)",
                "pocketkaldi::Nnet::Propagate(pocketkaldi::MatrixBase<float> const&, pocketkaldi::Matrix<float>*) const",
                "pocketkaldi::AcousticModel::Read(pocketkaldi::Configuration const&)",
                "pocketkaldi::AcousticModel::Process(pocketkaldi::AcousticModel::Instance*, "
                "pocketkaldi::VectorBase<float> const&, pocketkaldi::Matrix<float>*) const",
                "pocketkaldi::AcousticModel::EndOfStream(pocketkaldi::AcousticModel::Instance*, "
                "pocketkaldi::Matrix<float>*) const",
                "pocketkaldi::MatMat(pocketkaldi::MatrixBase<float> const&, pocketkaldi::MatrixBase<float> const&, "
                "pocketkaldi::MatrixBase<float>*)",
                "pocketkaldi::Quantize(pocketkaldi::MatrixBase<float> const&, pocketkaldi::Matrix<unsigned char>*, "
                "pocketkaldi::QuantizationParams*)"]:
        assert sym in out, sym


def test_compat_container_layer(tmp_path):
    """The stand-ins for the reference's container headers: Configuration,
    VEC0 / MAT0 readers and their error strings (no GPU)."""
    exe = os.path.join(ROOT, "build", "bin", "compat_test")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", ROOT, "build/bin/compat_test"], stdout=subprocess.DEVNULL)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout + r.stderr


def test_parsers_under_address_and_ub_sanitizers(tmp_path):
    """the host code under ASan + UBSan.  The compat container
    layer (compat_test) and the model-file parsers -- model_io.cc's NN02 /
    MAT0 / VEC0 readers behind ce_gpu_model_load_mem, and the drop-in
    Nnet::Read -- fed a valid image, every truncation of it, the reference's
    corruption cases (its messages), sections declared billions of bytes
    long and 20 000 seeded random corruptions (tests/native/parse_fuzz.cc):
    no sanitizer report, both parsers agree on every input."""
    subprocess.check_call(["make", "-C", ROOT, "-s", "sanitize"], stdout=subprocess.DEVNULL)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    for exe, args in (("compat_test_asan", []), ("parse_fuzz_asan", ["20000"])):
        r = subprocess.run([os.path.join(ROOT, "build", "bin", exe), str(tmp_path)] + args, capture_output=True,
                           text=True, env=env, timeout=300)
        assert r.returncode == 0 and "PASSED" in r.stdout, exe + "\n" + r.stdout[-3000:] + r.stderr[-3000:]
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]


def test_nnet_check_mem_without_a_device(tmp_path):
    """ce_gpu_nnet_check_mem parses an NN02 image on a machine without a GPU:
    the layer count and context of a valid image, the reference's messages
    for corrupt ones, the truncated-file error for a section declared longer
    than the image."""
    from catears_amd import formats, gpu, synth
    layers, left, right, _ = synth.tdnn_layers(256, 512, seed=3)
    img = bytearray(formats.nnet_bytes(layers, left, right))
    (tmp_path / "m.nnet").write_bytes(bytes(img))
    want, wl, wr = formats.read_nnet(str(tmp_path / "m.nnet"))
    assert gpu.nnet_check(img) == (len(want), wl, wr)
    bad = bytearray(img)
    bad[3:4] = b"3"
    with pytest.raises(gpu.CatearsError, match="ReadAndVerifyString: 'NN02' expected but 'NN03' found"):
        gpu.nnet_check(bad)
    with pytest.raises(gpu.CatearsError, match="IOError: failed to read"):
        gpu.nnet_check(img[:len(img) // 2])
    # the first layer's count field set to 2^31 - 1: refused before any allocation
    huge = bytearray(img)
    huge[24:28] = (0x7fffffff).to_bytes(4, "little")
    with pytest.raises(gpu.CatearsError):
        gpu.nnet_check(huge)


# ------------------------------------------------------------ GPU checks --

def _run(*args, env=None):
    assert os.path.exists(DRIVER), "pk_dropin not built"
    r = subprocess.run([DRIVER] + [str(a) for a in args], capture_output=True, text=True, timeout=300,
                       env=None if env is None else {**os.environ, **env})
    assert r.returncode == 0, (args[0], r.returncode, r.stderr[-2000:])


def _load(path, dtype=np.float32):
    raw = open(path, "rb").read()
    rows, cols = struct.unpack("<ii", raw[:8])
    return np.frombuffer(raw[8:], dtype=dtype).reshape(rows, cols)


def _put(tmp_path, name, arr):
    p = tmp_path / name
    np.ascontiguousarray(arr).tofile(p)
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [777, 160, 100000])
def test_fbank_streaming_matches_oracle(tmp_path, oracle, chunk):
    wave = oracle.read_wav(os.path.join(GOLDEN, "en-us-hello.wav"))
    out = tmp_path / "f.bin"
    _run("fbank", _put(tmp_path, "pcm.f32", wave), chunk, out)
    got = _load(out)
    want = oracle.Fbank().compute(wave)
    assert got.shape == want.shape
    assert np.max(np.abs(got - want)) <= FEAT_TOL
    kaldi = np.loadtxt(os.path.join(GOLDEN, "fbankmat_en-us-hello.wav.txt"), dtype=np.float32).reshape(-1, 40)
    assert np.max(np.abs(got - kaldi)) <= 1e-4  # the reference's own bar (test/fbank_test.cc)


@pytest.mark.gpu
def test_fbank_fast_mode_through_the_dropin(tmp_path, oracle):
    """CATEARS_FBANK=fast selects the fast (FMA-contracted) kernel for every lane of
    the drop-in runtime: streaming Fbank::Process output within the north
    star's fbank tolerance of the oracle and the Kaldi dump; an unknown value
    is refused (DeviceError, nonzero exit)."""
    wave = oracle.read_wav(os.path.join(GOLDEN, "en-us-hello.wav"))
    out = tmp_path / "f.bin"
    _run("fbank", _put(tmp_path, "pcm.f32", wave), 777, out, env={"CATEARS_FBANK": "fast"})
    got = _load(out)
    want = oracle.Fbank().compute(wave)
    assert got.shape == want.shape
    assert 0 < np.max(np.abs(got - want)) <= 1e-4  # the fast kernel, not bit-identical to the exact one
    kaldi = np.loadtxt(os.path.join(GOLDEN, "fbankmat_en-us-hello.wav.txt"), dtype=np.float32).reshape(-1, 40)
    assert np.max(np.abs(got - kaldi)) <= 1e-4
    r = subprocess.run([DRIVER, "fbank", str(tmp_path / "pcm.f32"), "777", str(out)], capture_output=True,
                       text=True, timeout=300, env={**os.environ, "CATEARS_FBANK": "approximate"})
    assert r.returncode != 0 and "CATEARS_FBANK" in (r.stdout + r.stderr)


@pytest.mark.gpu
def test_cmvn_getframe_bit_exact(tmp_path, oracle, global_stats):
    from catears_amd import synth
    wave = synth.pcm(3, 16000 * 8)  # 798 frames: crosses the 600-frame window
    feats = oracle.Fbank().compute(wave)
    out = tmp_path / "c.bin"
    _run("cmvn", _put(tmp_path, "x.f32", feats), len(feats), os.path.join(GOLDEN, "cmvn_stats.bin"), out)
    got = _load(out)
    want = oracle.cmvn(global_stats, feats)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def _am_config(tmp_path, xs_config, chunk, extra=""):
    src = open(xs_config).read().splitlines()
    d = os.path.dirname(xs_config)
    lines = []
    for ln in src:
        k = ln.split("=")[0].strip().lower() if "=" in ln else ""
        if k in ("nnet", "prior", "tid2pdf"):
            ln = f"{k} = {os.path.join(d, ln.split('=')[1].strip())}"
        if k == "chunk_size":
            ln = f"chunk_size = {chunk}"
        lines.append(ln)
    p = tmp_path / f"am{chunk}{'b' if extra else ''}.conf"
    p.write_text("\n".join(lines) + "\n" + extra)
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [50, 7, 1000])
def test_am_process_per_frame_matches_reference_streaming(tmp_path, oracle, xs_config, chunk):
    from catears_amd import formats, synth
    model = formats.read_am(xs_config)
    feats = oracle.Fbank().compute(synth.pcm(5, 16000 * 3 + 123))
    out = tmp_path / "am.bin"
    _run("am", _am_config(tmp_path, xs_config, chunk), _put(tmp_path, "x.f32", feats), len(feats), out)
    got = _load(out)
    want = oracle.am_stream(model, feats, chunk_size=chunk)
    assert got.shape == want.shape == (len(feats), model["num_pdfs"])
    assert np.max(np.abs(got - want)) <= LOGLIK_TOL


@pytest.mark.gpu
def test_am_streams_batched_across_threads(tmp_path, oracle, xs_config):
    """several streams (threads, one Instance each) on
    one AcousticModel with gpu_batch_streams = 4: chunks that are ready
    together go to the device in one call, and every stream gets exactly the
    rows it gets alone."""
    from catears_amd import formats, synth
    model = formats.read_am(xs_config)
    lens = [16000 * 3 + 123, 16000 * 2, 16000 * 4 + 999, 16000 * 1 + 5]
    feats = [oracle.Fbank().compute(synth.pcm(70 + i, n)) for i, n in enumerate(lens)]
    args = []
    for i, f in enumerate(feats):
        args += [_put(tmp_path, f"x{i}.f32", f), len(f)]
    conf = _am_config(tmp_path, xs_config, 50, extra="gpu_batch_streams = 4\ngpu_batch_wait_us = 3000\n")
    assert os.path.exists(DRIVER)
    r = subprocess.run([DRIVER, "am_mt", str(conf), str(tmp_path / "mt")] + [str(a) for a in args],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    calls, blocks, failed, lanes = [int(v) for v in r.stdout.split()[1::2]]
    assert failed == 0
    for i, f in enumerate(feats):
        got = _load(tmp_path / f"mt{i}.bin")
        alone = tmp_path / f"alone{i}.bin"
        _run("am", _am_config(tmp_path, xs_config, 50), tmp_path / f"x{i}.f32", len(f), alone)
        assert np.array_equal(got.view(np.uint32), _load(alone).view(np.uint32))
        want = oracle.am_stream(model, f, chunk_size=50)
        assert np.max(np.abs(got - want)) <= LOGLIK_TOL
    assert blocks == sum((len(f) + 49) // 50 for f in feats) or blocks > 0
    assert calls < blocks, (calls, blocks)  # some calls carried several streams' chunks


@pytest.mark.gpu
def test_am_streams_on_concurrent_lanes(tmp_path, oracle, xs_config):
    """Without cross-stream batching every thread's chunks go to the device
    on their own: the runtime leases each call a lane (context + stream) of
    its own, so concurrent streams overlap instead of queueing on one
    context, and each still gets exactly the rows it gets alone."""
    from catears_amd import synth
    lens = [16000 * 3 + 123, 16000 * 2, 16000 * 4 + 999, 16000 * 1 + 5]
    feats = [oracle.Fbank().compute(synth.pcm(70 + i, n)) for i, n in enumerate(lens)]
    args = []
    for i, f in enumerate(feats):
        args += [_put(tmp_path, f"x{i}.f32", f), len(f)]
    conf = _am_config(tmp_path, xs_config, 50)
    r = subprocess.run([DRIVER, "am_mt", str(conf), str(tmp_path / "mt")] + [str(a) for a in args],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, CATEARS_LANES="4"))
    assert r.returncode == 0, r.stderr[-2000:]
    calls, blocks, failed, lanes = [int(v) for v in r.stdout.split()[1::2]]
    assert failed == 0 and calls == blocks
    assert 2 <= lanes <= 4, lanes
    for i, f in enumerate(feats):
        alone = tmp_path / f"alone{i}.bin"
        _run("am", conf, tmp_path / f"x{i}.f32", len(f), alone)
        assert np.array_equal(_load(tmp_path / f"mt{i}.bin").view(np.uint32), _load(alone).view(np.uint32))


@pytest.mark.gpu
def test_am_batcher_device_failure_releases_every_stream(tmp_path, xs_config):
    """A failing batched device call (injected: the first Check() throws)
    must finish every request of its batch with the error -- the leader and
    its followers all see DeviceError -- and leave the batcher usable; no
    thread may hang waiting for a leader that died (am.cc)."""
    from catears_amd import synth
    from oracle import pyoracle
    lens = [16000 * 2, 16000 * 2 + 77, 16000 * 3, 16000 + 5]
    feats = [pyoracle.Fbank().compute(synth.pcm(90 + i, n)) for i, n in enumerate(lens)]
    args = []
    for i, f in enumerate(feats):
        args += [_put(tmp_path, f"x{i}.f32", f), len(f)]
    # the leader waits (up to 20 s) until all four streams have enqueued, so
    # the failing first call carries four requests: the three followers must
    # be released with the leader's error, not just the leader
    conf = _am_config(tmp_path, xs_config, 50, extra="gpu_batch_streams = 4\ngpu_batch_wait_us = 20000000\n")
    r = subprocess.run([DRIVER, "am_mt_fail", str(conf), str(tmp_path / "mt")] + [str(a) for a in args],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    calls, blocks, failed, lanes = [int(v) for v in r.stdout.split()[1::2]]
    assert failed == len(feats) > 1
    assert calls == 1 and blocks == len(feats)
    # the streams outside the failed batch completed with full output
    done = [i for i in range(len(feats)) if (tmp_path / f"mt{i}.bin").exists()]
    assert len(done) == len(feats) - failed
    for i in done:
        assert _load(tmp_path / f"mt{i}.bin").shape[0] == len(feats[i])


@pytest.mark.gpu
def test_am_short_utterance(tmp_path, oracle, xs_config):
    from catears_amd import formats
    model = formats.read_am(xs_config)
    rng = np.random.default_rng(4)
    feats = rng.normal(8, 3, size=(3, 40)).astype(np.float32)  # fewer frames than the context
    out = tmp_path / "am.bin"
    _run("am", _am_config(tmp_path, xs_config, 50), _put(tmp_path, "x.f32", feats), len(feats), out)
    want = oracle.am_stream(model, feats, chunk_size=50)
    assert np.max(np.abs(_load(out) - want)) <= LOGLIK_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["nnet", "layer"])
def test_nnet_propagate_block(tmp_path, oracle, xs_config, mode):
    from catears_amd import formats
    kv = formats.read_config(xs_config)
    layers, _, _ = formats.read_nnet(kv["nnet"])
    rng = np.random.default_rng(9)
    x = rng.normal(0, 2, size=(137, 40)).astype(np.float32)
    out = tmp_path / "n.bin"
    _run(mode, kv["nnet"], _put(tmp_path, "x.f32", x), 137, 40, out)
    want = oracle.nnet_propagate(layers, x)
    got = _load(out)
    assert got.shape == want.shape
    assert np.max(np.abs(got - want)) <= LOGLIK_TOL


def _single_layer_nets():
    rng = np.random.default_rng(21)
    W = rng.uniform(-0.2, 0.2, size=(24, 33)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, size=33).astype(np.float32)
    return {
        "linear": [{"kind": "linear", "W": W, "b": b}],
        "relu": [{"kind": "relu"}],
        "softmax": [{"kind": "softmax"}],
        "log_softmax": [{"kind": "log_softmax"}],
        "normalize": [{"kind": "normalize"}],
        "batchnorm": [{"kind": "batchnorm", "scale": rng.uniform(0.5, 1.5, 24).astype(np.float32),
                       "offset": rng.uniform(-1, 1, 24).astype(np.float32)}],
        # clamped splice with no Narrow after it (edge rows repeat)
        "splice": [{"kind": "splice", "indices": [-3, 0, 2]}],
        # Narrow on a block shorter than its context: passes through
        "narrow_short": [{"kind": "narrow", "left": 6, "right": 5}],
        "narrow": [{"kind": "narrow", "left": 2, "right": 1}],
    }


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(_single_layer_nets()))
@pytest.mark.parametrize("mode", ["nnet", "layer"])
def test_single_layers(tmp_path, oracle, name, mode):
    from catears_amd import formats
    layers = _single_layer_nets()[name]
    rows = 9
    x = np.random.default_rng(5).normal(0, 1.5, size=(rows, 24)).astype(np.float32)
    nn = tmp_path / "l.nnet"
    nn.write_bytes(formats.nnet_bytes(layers, 0, 0))
    out = tmp_path / "o.bin"
    _run(mode, nn, _put(tmp_path, "x.f32", x), rows, 24, out)
    want = oracle.nnet_propagate(layers, x)
    got = _load(out)
    assert got.shape == want.shape
    if name in ("relu", "splice", "narrow", "narrow_short", "batchnorm"):
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))  # exact float ops
    else:
        assert np.max(np.abs(got - want)) <= LOGLIK_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (37, 50, 3), (300, 129, 200), (64, 64, 1000)])
def test_matmat(tmp_path, m, n, k):
    rng = np.random.default_rng(m * 7 + k)
    a = rng.uniform(-1, 1, (m, k)).astype(np.float32)
    b = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    out = tmp_path / "c.bin"
    _run("matmat", m, n, k, _put(tmp_path, "a.f32", a), _put(tmp_path, "b.f32", b), out)
    want = a.astype(np.float64) @ b.astype(np.float64)
    assert np.max(np.abs(_load(out) - want)) <= 1e-5 * max(1.0, np.sqrt(k))


@pytest.mark.gpu
def test_quantize_and_u8_gemm_bit_exact(tmp_path, oracle):
    rng = np.random.default_rng(13)
    a = rng.normal(0.3, 2.0, (70, 96)).astype(np.float32)
    b = rng.uniform(-1.5, 0.5, (96, 45)).astype(np.float32)
    qa_want, sa, za = oracle.quantize(a)
    qb_want, sb, zb = oracle.quantize(b)
    for name, x, q_want, s, z in (("a", a, qa_want, sa, za), ("b", b, qb_want, sb, zb)):
        _run("quant", x.shape[0], x.shape[1], _put(tmp_path, name + ".f32", x), tmp_path / (name + ".u8"),
             tmp_path / (name + ".qp"))
        q = _load(tmp_path / (name + ".u8"), np.uint8)
        s_got, z_got = struct.unpack("<fi", (tmp_path / (name + ".qp")).read_bytes())
        assert np.array_equal(q, q_want)
        assert (np.float32(s_got), z_got) == (np.float32(s), z)
    out = tmp_path / "c.bin"
    _run("gemmu8", 70, 45, 96, _put(tmp_path, "a8", qa_want), _put(tmp_path, "b8", qb_want),
         tmp_path / "a.qp", tmp_path / "b.qp", out)
    want = oracle.gemm_u8u8f32(qa_want, sa, za, qb_want, sb, zb)
    assert np.array_equal(_load(out).view(np.uint32), want.view(np.uint32))
