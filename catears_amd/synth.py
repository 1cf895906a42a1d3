"""Deterministic synthetic inputs for tests and the benchmark.

No acoustic model or audio corpus ships with the reference, so both are
generated from a portable splitmix64 stream (identical bits on every machine):
  * PCM: 3 sinusoids (f ~ U[100,4000) Hz, a ~ U[500,4000)) + N(0, 1000) noise,
    rounded and clipped to int16, stored as float at raw scale like
    src/pcm_reader.cc:174; seed 20250117 + utterance index.
  * TDNN in the reference's NN02 format: Splice -> Narrow -> Linear -> ReLU ->
    BatchNorm per hidden layer, then Linear -> LogSoftmax, exactly the layer
    pattern tool/convert_am.py:272-285 emits.  TDNN-S (hidden 1024, 3456 pdfs)
    is the benchmark model, TDNN-XS (256, 512) the fixture model.
"""
import os

import numpy as np

from . import formats

GOLDEN = 0x9E3779B97F4A7C15
SPLICES_S = [[-2, -1, 0, 1, 2], [-1, 0, 1], [-1, 0, 1], [-3, 0, 3], [-3, 0, 3], [0]]
MODELS = {"tdnn-s": dict(hidden=1024, pdfs=3456), "tdnn-xs": dict(hidden=256, pdfs=512)}


def splitmix64(seed, n):
    with np.errstate(over="ignore"):
        z = np.uint64(seed % (1 << 64)) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed, n, lo=0.0, hi=1.0):
    u = (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    return lo + (hi - lo) * u


def pcm(u, n_samples=160000, seed_base=20250117):
    s = seed_base + u
    m = (n_samples + 1) // 2
    r = uniform(s, 6 + 2 * m)
    f = 100.0 + 3900.0 * r[0:3]
    a = 500.0 + 3500.0 * r[3:6]
    u1, u2 = r[6::2][:m], r[7::2][:m]
    rad = np.sqrt(-2.0 * np.log1p(-u1))
    z = np.empty(2 * m)
    z[0::2] = rad * np.cos(2 * np.pi * u2)
    z[1::2] = rad * np.sin(2 * np.pi * u2)
    t = np.arange(n_samples) / 16000.0
    x = sum(a[i] * np.sin(2 * np.pi * f[i] * t) for i in range(3)) + 1000.0 * z[:n_samples]
    return np.clip(np.rint(x), -32768, 32767).astype(np.float32)


def tdnn_layers(hidden, pdfs, in_dim=40, splices=SPLICES_S, seed=7):
    layers = []
    width = in_dim
    tensor = [0]

    def draw(n, lo, hi):
        tensor[0] += 1
        return uniform(seed * 1000003 + tensor[0], n, lo, hi)

    def linear(k, n):
        W = (draw(k * n, -1.0, 1.0) * np.sqrt(3.0 / k)).astype(np.float32).reshape(k, n)
        b = (0.1 * draw(n, -1.0, 1.0)).astype(np.float32)
        return {"kind": "linear", "W": W, "b": b}

    for idx in splices:
        layers.append({"kind": "splice", "indices": list(idx)})
        layers.append({"kind": "narrow", "left": -min(min(idx), 0), "right": max(max(idx), 0)})
        layers.append(linear(width * len(idx), hidden))
        layers.append({"kind": "relu"})
        layers.append({"kind": "batchnorm",
                       "scale": (1.0 + 0.1 * draw(hidden, -1.0, 1.0)).astype(np.float32),
                       "offset": (0.1 * draw(hidden, -1.0, 1.0)).astype(np.float32)})
        width = hidden
    layers.append(linear(width, pdfs))
    layers.append({"kind": "log_softmax"})
    left = sum(-min(min(s), 0) for s in splices)
    right = sum(max(max(s), 0) for s in splices)
    prior = draw(pdfs, 0.5, 1.5)
    prior = (prior / prior.sum()).astype(np.float32)
    return layers, left, right, prior


def write_model(out_dir, name="tdnn-s", chunk_size=50, seed=7):
    """Writes <name>.nnet / .prior / .tid2pdf / .conf; returns the config path."""
    spec = MODELS[name]
    os.makedirs(out_dir, exist_ok=True)
    conf = os.path.join(out_dir, name + ".conf")
    if os.path.exists(conf):
        return conf
    layers, left, right, prior = tdnn_layers(spec["hidden"], spec["pdfs"], seed=seed)
    base = os.path.join(out_dir, name)
    with open(base + ".nnet", "wb") as f:
        f.write(formats.nnet_bytes(layers, left, right))
    with open(base + ".prior", "wb") as f:
        f.write(formats.vec_bytes(prior))
    tid2pdf = np.concatenate([[0], np.repeat(np.arange(spec["pdfs"], dtype=np.int32), 2)])
    with open(base + ".tid2pdf", "wb") as f:
        f.write(formats.vec_bytes(tid2pdf, np.int32))
    tmp = conf + ".tmp"
    with open(tmp, "w") as f:
        f.write(f"# synthetic {name} (catears_amd.synth)\n")
        f.write(f"nnet = {name}.nnet\nprior = {name}.prior\ntid2pdf = {name}.tid2pdf\n")
        f.write(f"left_context = {left}\nright_context = {right}\nchunk_size = {chunk_size}\n")
        f.write(f"num_pdfs = {spec['pdfs']}\n")
    os.replace(tmp, conf)
    return conf


def cmvn_stats_synthetic(seed=11):
    """A 41-float global-stats vector shaped like test/data/cmvn_stats.bin:
    40 sums with mean ~U(8,16) over N = 1e6 frames, then N."""
    n = 1.0e6
    mean = uniform(seed, 40, 8.0, 16.0)
    return np.concatenate([mean * n, [n]]).astype(np.float32)
