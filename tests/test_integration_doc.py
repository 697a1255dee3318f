"""INTEGRATION.md's plugin (option B) is the committed translation unit
integration/myyuv_hip_plugin.cpp, verbatim, and both integration units compile
against the reference's own headers and this repo's C ABI header (syntax and
types; tests/test_reference_binding.py links and runs them).  The compile
check needs /root/reference (this container)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

REF_LIB = "/root/reference/myyuv_lib"
UNITS = [os.path.join(ROOT, "integration", n) for n in ("myyuv_hip_plugin.cpp", "myyuv_dct_hip.cpp")]


def test_doc_shows_the_plugin_unit_verbatim():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```cpp\n(.*?)```", doc, re.S)
    assert open(UNITS[0]).read() in blocks


@pytest.mark.parametrize("unit", UNITS)
def test_integration_unit_compiles(unit):
    if not os.path.isdir(REF_LIB):
        pytest.skip("reference sources not present")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", REF_LIB, "-I", os.path.join(ROOT, "include"),
                        unit], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
