import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "yuv-manipulations-2_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")


@pytest.fixture(scope="session")
def golden():
    import myyuv_file

    def load(name):
        return myyuv_file.YUVFile.load(os.path.join(GOLDEN, name))

    return load


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O

    O.lib()
    return O


def _codec_with(env):
    import myyuv_hip

    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        os.environ[k] = v
    try:
        return myyuv_hip.Codec(0)
    finally:
        for k in env:
            if old[k] is None:
                del os.environ[k]
            else:
                os.environ[k] = old[k]


# kernel arrangements (MYYUV_ENCODER / MYYUV_DECODER are read when a context
# is created): "default" is the product (K1 -> K2 through HBM, the fused
# decoder k_decode_idct), "split" K1 -> K2 and K5 -> K6 through HBM
ARRANGEMENTS = {"default": {"MYYUV_ENCODER": "split", "MYYUV_DECODER": "fused"},
                "split": {"MYYUV_ENCODER": "split", "MYYUV_DECODER": "split"}}


@pytest.fixture(scope="session", params=list(ARRANGEMENTS))
def codec(request):
    """A codec context per kernel arrangement (ARRANGEMENTS); every test
    taking `codec` runs on both."""
    c = _codec_with(ARRANGEMENTS[request.param])
    yield c
    c.close()


@pytest.fixture(scope="session")
def fused_encoder():
    """A context with the fused single-pass encoder k_encode_tile
    (MYYUV_ENCODER=fused).  It measured slower than K1 -> K2
    in every round, so it is not the product and not in the
    `codec` matrix; tests/test_gpu_fused_encoder.py keeps it bit-exact."""
    c = _codec_with({"MYYUV_ENCODER": "fused", "MYYUV_DECODER": "fused"})
    yield c
    c.close()


@pytest.fixture(scope="session")
def chef_big(golden, oracle):
    """The decode of chef-with-trumpet-big-DCT-50 (4032x3008): the stand-in for
    the missing raw 4K input (SURVEY.md §7 hard part 6)."""
    f = golden("chef-with-trumpet-big-DCT-50.myyuv")
    raw = oracle.decompress(f.data, f.width, f.height, tuple(f.params))
    return f, raw
