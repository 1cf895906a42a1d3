"""Extract the reference's golden vectors into small data fixtures.

Run in the build container (needs /root/reference, read-only).  It copies the
data files the reference's own tests hold (WAVs, Kaldi feature dumps, CMVN
global stats) and extracts the *numbers* of the known-answer tests embedded in
test/srfft_test.cc and test/nnet_test.cc into JSON.  No reference source text
is kept.  Output: tests/golden/ref/.
"""
import json
import os
import re
import shutil
import sys

REF = os.environ.get("CATEARS_REF", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref")

FLOAT = r"-?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?"


def floats_in(text):
    return [float(x) for x in re.findall(FLOAT + r"(?=f?\b)", text)]


def array_after(src, name):
    m = re.search(r"float\s+" + name + r"\[[^\]]*\]\s*=\s*\{(.*?)\};", src, re.S)
    return [float(x) for x in re.findall(FLOAT, m.group(1))]


def main():
    os.makedirs(OUT, exist_ok=True)
    data = os.path.join(REF, "test", "data")
    for f in ("en-us-hello.wav", "en-us-cat.wav", "fbankmat_en-us-hello.wav.txt",
              "fbankcmvnmat_en-us-hello.wav.txt", "cmvn_stats.bin", "kaldi_fbank.conf"):
        shutil.copyfile(os.path.join(data, f), os.path.join(OUT, f))

    # test/srfft_test.cc: 128-point real FFT, input data[] and expected fft_data[],
    # tolerance 1e-4 (srfft_test.cc:285); only the listed prefix is checked.
    src = open(os.path.join(REF, "test", "srfft_test.cc")).read()
    inp = array_after(src, "data")
    exp = array_after(src, "fft_data")
    json.dump({"n": 128, "input": inp, "expected_prefix": exp, "tol": 1e-4,
               "source": "test/srfft_test.cc:13,144,285"},
              open(os.path.join(OUT, "srfft128.json"), "w"), indent=0)

    # test/nnet_test.cc known answers (tolerance 1e-3, nnet_test.cc:23-25).
    src = open(os.path.join(REF, "test", "nnet_test.cc")).read()

    def fn(name):
        m = re.search(r"void " + name + r"\(\)\s*\{(.*?)\n\}", src, re.S)
        return m.group(1)

    def arr(body, name):
        m = re.search(r"float\s+" + name + r"\[\]\s*=\s*\{(.*?)\};", body, re.S)
        return [float(x) for x in re.findall(FLOAT, m.group(1))]

    def rows(body):
        return [[float(x) for x in re.findall(FLOAT, r)]
                for r in re.findall(r"CheckVector\(y\.Row\(\d+\),\s*\{(.*?)\}\)", body)]

    def eqs(body):
        return [float(v) for v in re.findall(r"CheckEq\(y\(0, \d\), (" + FLOAT + r")f?\)", body)]

    kat = {"tol": 1e-3, "source": "test/nnet_test.cc"}
    b = fn("TestLinearLayer")
    kat["linear"] = {"W_out_by_in": arr(b, "W_data"), "shape": [4, 3], "b": arr(b, "b_data"),
                     "x": arr(b, "x_data"), "y": eqs(b)}
    b = fn("TestSoftmaxLayer")
    kat["softmax"] = {"x": arr(b, "x_data"), "y": eqs(b)}
    b = fn("TestLogSoftmaxLayer")
    kat["log_softmax"] = {"x": arr(b, "x_data"), "shape": [4, 3], "y": rows(b)}
    b = fn("TestReLULayer")
    kat["relu"] = {"x": arr(b, "x_data"), "y": eqs(b)}
    b = fn("TestNormalizeLayer")
    kat["normalize"] = {"x": arr(b, "x_data"), "sum_sq": 4.0, "tol": 1e-4}
    b = fn("TestSpliceLayer")
    kat["splice"] = {"x": arr(b, "x_data"), "shape": [4, 2],
                     "indices": [int(v) for v in re.search(r"spliceLayer\(\{(.*?)\}\)", b).group(1).split(",")],
                     "y": rows(b)}
    b = fn("TestBatchNormLayer")
    kat["batchnorm"] = {"scale": arr(b, "scale_data"), "offset": arr(b, "offset_data"),
                        "x": arr(b, "x_data"), "shape": [2, 3], "y": rows(b)}
    b = fn("TestNarrowLayer")
    ys = rows(b)
    kat["narrow"] = {"x": arr(b, "W_data"), "shape": [5, 3], "left": 1, "right": 2,
                     "y_full": ys[:2], "y_small_rows": 3, "y_small": ys[2:]}
    json.dump(kat, open(os.path.join(OUT, "nnet_kat.json"), "w"), indent=1)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    sys.exit(main())
