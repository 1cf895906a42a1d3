import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden", "ref")
# the measurement build (make EXPERIMENTS=1): the same kernels plus the
# tuning switches the product library compiles out (CE_KNOB, internal.h)
EXP_LIB = os.path.join(ROOT, "catears_amd", "lib", "libcatears_hip_exp.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")


def _ensure_oracle():
    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")],
                              stdout=subprocess.DEVNULL)
    return lib


@pytest.fixture(scope="session")
def oracle():
    _ensure_oracle()
    from oracle import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def models_dir(tmp_path_factory):
    from catears_amd import synth
    d = str(tmp_path_factory.mktemp("models"))
    synth.write_model(d, "tdnn-xs")
    return d


@pytest.fixture(scope="session")
def xs_config(models_dir):
    return os.path.join(models_dir, "tdnn-xs.conf")


@pytest.fixture(scope="session")
def s_config(models_dir):
    from catears_amd import synth
    return synth.write_model(models_dir, "tdnn-s")


@pytest.fixture(scope="session")
def global_stats():
    """test/data/cmvn_stats.bin payload (41 floats)."""
    from catears_amd import formats
    return formats.read_vec(os.path.join(GOLDEN, "cmvn_stats.bin"))


@pytest.fixture(scope="session")
def exp_lib():
    """Path of the experiments library, for child processes that select an
    alternative schedule through its CATEARS_* switches."""
    if not os.path.exists(EXP_LIB):
        pytest.skip("libcatears_hip_exp.so not built (make EXPERIMENTS=1 lib)")
    return EXP_LIB
