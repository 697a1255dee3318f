"""INTEGRATION.md's plugin (option B) is real code: its C++ blocks compile
against the reference's own headers and this repo's C ABI header (syntax and
types only, no link).  Needs /root/reference (this container)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

REF_LIB = "/root/reference/myyuv_lib"


def test_plugin_snippet_compiles(tmp_path):
    if not os.path.isdir(REF_LIB):
        pytest.skip("reference sources not present")
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```cpp\n(.*?)```", doc, re.S)
    assert len(blocks) >= 2
    # the BMP entry sits next to the first block's helpers (same anonymous namespace)
    first = blocks[0].rstrip()
    assert first.endswith("}  // namespace")
    src = first[: -len("}  // namespace")] + blocks[1] + "\n}  // namespace\n"
    f = tmp_path / "plugin.cpp"
    f.write_text(src)
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", REF_LIB, "-I", os.path.join(ROOT, "include"),
                        str(f)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
