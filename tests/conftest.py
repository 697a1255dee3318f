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


@pytest.fixture(scope="session", params=["split", "fused"])
def codec(request):
    """A codec context per kernel arrangement: "split" (K1 -> K2 and K5 -> K6
    through HBM) and "fused" (the single-pass encoder k_encode_tile and the
    single-pass decoder k_decode_idct, the decoder's default; MYYUV_ENCODER /
    MYYUV_DECODER are read when the context is created).  Every test taking
    `codec` runs on both."""
    import myyuv_hip

    vals = {"MYYUV_ENCODER": request.param, "MYYUV_DECODER": request.param}
    old = {k: os.environ.get(k) for k in vals}
    for k, v in vals.items():
        os.environ[k] = v
    try:
        c = myyuv_hip.Codec(0)
    finally:
        for k in vals:
            if old[k] is None:
                del os.environ[k]
            else:
                os.environ[k] = old[k]
    yield c
    c.close()


@pytest.fixture(scope="session")
def chef_big(golden, oracle):
    """The decode of chef-with-trumpet-big-DCT-50 (4032x3008): the stand-in for
    the missing raw 4K input (SURVEY.md §7 hard part 6)."""
    f = golden("chef-with-trumpet-big-DCT-50.myyuv")
    raw = oracle.decompress(f.data, f.width, f.height, tuple(f.params))
    return f, raw
