"""Host checks of the division- and roundf-free arithmetic of K1/K6
(yuv-manipulations-2_amd/csrc/k_transform.hip): tools/check_numerics.c, built
with gcc -ffp-contract=off, runs the same IEEE binary32 operations the GPU
does.  roundf == truncf(x + copysignf(0.49999997f, x)) is checked on a
257-stride sample here (all 2^32 encodings with `check_numerics all`, ~20 s,
done when the rule was adopted); the K1 quantisation shortcut is checked for
every Q in 1..255 at and around every tie point (+/-256 ulps) and at random;
the K6 magic-add rounding around every half-integer in [-150, 150]."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tools", "check_numerics.c")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    exe = str(tmp_path_factory.mktemp("num") / "check_numerics")
    subprocess.run([cc, "-O2", "-ffp-contract=off", "-fno-fast-math", "-o", exe, SRC, "-lm"], check=True)
    return exe


def test_fast_paths_match_reference_arithmetic(checker):
    r = subprocess.run([checker], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
    assert int(r.stdout.split()[1]) > 80_000_000
