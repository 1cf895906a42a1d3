"""Readers/writers of the reference's binary model formats.

VEC0 / MAT0 (src/vector.cc:267-300, src/matrix.cc:159-191), NN02 nnet with LAY0
layers (src/nnet.cc:221-293; writer side tool/convert_am.py:26-168) and the
key = value AM config (src/configuration.cc:14-90, keys of src/am.cc:31-60).
Host-side plumbing shared by the synthetic-model generator, tests and bench;
the device loader of the product is the C++ one in csrc/capi.cc.
"""
import os
import struct

import numpy as np

LINEAR, RELU, NORMALIZE, SOFTMAX, SPLICE, BATCHNORM, LOG_SOFTMAX, NARROW = 0, 1, 2, 3, 6, 7, 8, 9
_KIND = {LINEAR: "linear", RELU: "relu", NORMALIZE: "normalize", SOFTMAX: "softmax",
         SPLICE: "splice", BATCHNORM: "batchnorm", LOG_SOFTMAX: "log_softmax", NARROW: "narrow"}


def vec_bytes(v, dtype=np.float32):
    v = np.ascontiguousarray(v, dtype=dtype)
    return b"VEC0" + struct.pack("<ii", v.size * 4 + 4, v.size) + v.tobytes()


def mat_bytes(m):
    m = np.ascontiguousarray(m, dtype=np.float32)
    out = [b"MAT0", struct.pack("<iii", 8, m.shape[0], m.shape[1])]
    out += [vec_bytes(row) for row in m]
    return b"".join(out)


def nnet_bytes(layers, left, right):
    """layers: list of dicts {kind, ...} in the reader's vocabulary."""
    out = [b"NN02", struct.pack("<iii", left, right, len(layers))]
    ids = {v: k for k, v in _KIND.items()}
    for L in layers:
        out.append(b"LAY0" + struct.pack("<i", ids[L["kind"]]))
        k = L["kind"]
        if k == "linear":
            out += [mat_bytes(L["W"]), vec_bytes(L["b"])]
        elif k == "splice":
            out.append(struct.pack("<i", len(L["indices"])))
            out += [struct.pack("<i", int(i)) for i in L["indices"]]
        elif k == "batchnorm":
            out += [vec_bytes(L["scale"]), vec_bytes(L["offset"])]
        elif k == "narrow":
            out.append(struct.pack("<ii", L["left"], L["right"]))
    return b"".join(out)


class _Buf:
    def __init__(self, data, name):
        self.d, self.p, self.name = data, 0, name

    def take(self, n):
        if self.p + n > len(self.d):
            raise IOError(f"failed to read: {self.name}")
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def tag(self, t):
        got = self.take(4)
        if got != t:
            raise ValueError(f"'{t.decode()}' expected but '{got!r}' found in {self.name}")

    def i32(self):
        return struct.unpack("<i", self.take(4))[0]

    def vec(self, dtype=np.float32):
        self.tag(b"VEC0")
        sec, dim = self.i32(), self.i32()
        if dim * 4 + 4 != sec:
            raise ValueError(f"section_size mismatch in {self.name}")
        return np.frombuffer(self.take(4 * dim), dtype=dtype).copy()

    def mat(self):
        self.tag(b"MAT0")
        self.i32()
        r, c = self.i32(), self.i32()
        m = np.zeros((r, c), np.float32)
        for i in range(r):
            row = self.vec()
            if row.size != c:
                raise ValueError(f"row size mismatch in {self.name}")
            m[i] = row
        return m


def read_vec(path, dtype=np.float32):
    return _Buf(open(path, "rb").read(), path).vec(dtype)


def read_nnet(path):
    """Returns (layers, left, right) with layers as dicts (kind + params)."""
    b = _Buf(open(path, "rb").read(), path)
    b.tag(b"NN02")
    left, right, n = b.i32(), b.i32(), b.i32()
    layers = []
    for _ in range(n):
        b.tag(b"LAY0")
        lid = b.i32()
        if lid not in _KIND:
            raise ValueError(f"unexpected layer type: {lid} ({path})")
        L = {"kind": _KIND[lid]}
        if lid == LINEAR:
            L["W"], L["b"] = b.mat(), b.vec()
        elif lid == SPLICE:
            L["indices"] = [b.i32() for _ in range(b.i32())]
        elif lid == BATCHNORM:
            L["scale"], L["offset"] = b.vec(), b.vec()
        elif lid == NARROW:
            L["left"], L["right"] = b.i32(), b.i32()
        layers.append(L)
    return layers, left, right


def read_config(path):
    kv = {}
    for line in open(path):
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        k, v = line.split("=")
        kv[k.strip().lower()] = v.strip()
    d = os.path.dirname(os.path.abspath(path))
    for key in ("nnet", "prior", "tid2pdf"):
        if key in kv and not kv[key].startswith("/"):
            kv[key] = os.path.join(d, kv[key])
    return kv


def read_am(config_path):
    """AcousticModel::Read (src/am.cc:26-64) on the host: layers, log prior
    (ApplyLog in float), contexts, chunk size, tid2pdf."""
    kv = read_config(config_path)
    layers, _, _ = read_nnet(kv["nnet"])
    prior = read_vec(kv["prior"])
    return {"layers": layers, "log_prior": np.log(prior).astype(np.float32),
            "left": int(kv["left_context"]), "right": int(kv["right_context"]),
            "chunk": int(kv["chunk_size"]), "num_pdfs": int(kv["num_pdfs"]),
            "tid2pdf": read_vec(kv["tid2pdf"], np.int32)}
