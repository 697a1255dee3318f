"""The reference-side bindings of INTEGRATION.md, executed: the reference's own
CLI and library (its sources untouched, built by oracle/Makefile `hipref`)
with the MI355X codec bound in
  * Seam 1 — integration/myyuv_hip_plugin.cpp re-registers
    YUV::compress_map / decompress_map [DCT][IYUV] and bmp_to_yuv_map[IYUV]
    (myyuv_yuv.hpp:106-116) at static init: myyuv_cli_hipplugin and
    libmyyuv_ref_hipplugin.so (YUV::compress / decompress in-process);
  * Seam 2 — integration/myyuv_dct_hip.cpp defines myyuvDCT::compress_DCT_planar
    / decompress_DCT_planar (DCT.hpp:16,25) on the C ABI, linked under the
    reference's myyuv_yuv.cpp without myyuv_DCT/: myyuv_cli_hipdct.
The GPU tests check the files these produce against the reference's golden
images and the reference CLI's own output, and that the dispatch reached the
HIP codec (MYYUV_HIP_PLUGIN_TRACE)."""
import gzip
import hashlib
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

REF = os.path.join(ROOT, "oracle", "_ref")
PLUGIN_CLI = os.path.join(REF, "myyuv_cli_hipplugin")
DCT_CLI = os.path.join(REF, "myyuv_cli_hipdct")
REF_CLI = os.path.join(REF, "myyuv_cli_ref")
SMALL = os.path.join(GOLDEN, "chef-with-trumpet.myyuv")
C50 = os.path.join(GOLDEN, "chef-with-trumpet-DCT-50.myyuv")
C90 = os.path.join(GOLDEN, "chef-with-trumpet-DCT-90.myyuv")
BIG50 = os.path.join(GOLDEN, "chef-with-trumpet-big-DCT-50.myyuv")


def need(*paths):
    for p in paths:
        if not os.path.exists(p):
            pytest.skip(f"{os.path.basename(p)} not built (make -C oracle ref hipref)")


def run(exe, *args, trace=False):
    env = dict(os.environ)
    if trace:
        env["MYYUV_HIP_PLUGIN_TRACE"] = "1"
    return subprocess.run([exe, *args], capture_output=True, text=True, env=env)


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


@pytest.mark.parametrize("exe", [PLUGIN_CLI, DCT_CLI])
def test_bound_cli_info_matches_reference(exe):
    """No codec work: the bound CLIs start (the plugin's static registration
    runs) and print what the reference CLI prints."""
    need(exe, REF_CLI)
    for path in (SMALL, C50):
        a, b = run(exe, path, "-info"), run(REF_CLI, path, "-info")
        assert a.returncode == b.returncode == 0, a.stderr
        assert a.stdout == b.stdout


def test_plugin_is_linked_to_the_hip_codec():
    need(PLUGIN_CLI, DCT_CLI)
    for exe in (PLUGIN_CLI, DCT_CLI):
        out = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
        assert "libmyyuv_hip.so" in out, out


@pytest.mark.gpu
@pytest.mark.parametrize("exe,tag", [(PLUGIN_CLI, "myyuv_hip plugin: compress"),
                                     (DCT_CLI, "myyuv_dct_hip: compress_DCT_planar")])
@pytest.mark.parametrize("q,gold", [(["50"], C50), (["90", "90", "90"], C90)])
def test_bound_cli_compress_is_golden(tmp_path, exe, tag, q, gold):
    """The reference's CLI (main.cpp:151-185 -> YUV::compress) through the HIP
    codec writes the reference's golden files byte for byte."""
    need(exe)
    out = tmp_path / "o.myyuv"
    r = run(exe, SMALL, "-compress", "DCT", *q, "-o", str(out), trace=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert tag in r.stderr
    assert out.read_bytes() == open(gold, "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("exe,tag", [(PLUGIN_CLI, "myyuv_hip plugin: decompress"),
                                     (DCT_CLI, "myyuv_dct_hip: decompress_DCT_planar")])
@pytest.mark.parametrize("src", [C50, C90, BIG50])
def test_bound_cli_decompress_matches_reference_cli(tmp_path, exe, tag, src):
    """-decompress through the HIP codec equals the reference CLI's own output
    file (CPU path, same run)."""
    need(exe, REF_CLI)
    a, b = tmp_path / "hip.myyuv", tmp_path / "ref.myyuv"
    r = run(exe, src, "-decompress", "-o", str(a), trace=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert tag in r.stderr
    r = run(REF_CLI, src, "-decompress", "-o", str(b))
    assert r.returncode == 0, r.stdout + r.stderr
    assert sha(a) == sha(b)
    if src == BIG50:  # the decoded big frame
        assert sha(a) == "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"


@pytest.mark.gpu
def test_plugin_cli_bmp_to_yuv_is_golden(tmp_path):
    """-to_yuv IYUV through the re-registered bmp_to_yuv_map[IYUV] writes the
    reference's chef-with-trumpet.myyuv."""
    need(PLUGIN_CLI)
    bmp = tmp_path / "chef.bmp"
    bmp.write_bytes(gzip.open(os.path.join(GOLDEN, "chef-with-trumpet.bmp.gz")).read())
    out = tmp_path / "o.myyuv"
    r = run(PLUGIN_CLI, str(bmp), "-to_yuv", "IYUV", "-o", str(out), trace=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "myyuv_hip plugin: bmp_to_iyuv" in r.stderr
    assert out.read_bytes() == open(SMALL, "rb").read()


@pytest.mark.gpu
def test_plugin_library_in_process(codec, golden, oracle, chef_big):
    """The reference library with the plugin linked in, called in-process
    through its public YUV::compress / YUV::decompress (oracle/ref_harness.cpp):
    golden bytes and the oracle's decode, on the small and the big frame."""
    need(os.path.join(REF, "libmyyuv_ref_hipplugin.so"))
    from oracle import ref as R
    raw = golden("chef-with-trumpet.myyuv")
    for q, gname in (((50, 50, 50), "chef-with-trumpet-DCT-50.myyuv"), ((90, 90, 90), "chef-with-trumpet-DCT-90.myyuv")):
        pay = R.compress(raw.data, raw.width, raw.height, q, variant="hipplugin")
        assert pay == golden(gname).data
        assert R.decompress(pay, raw.width, raw.height, q, variant="hipplugin") == \
            oracle.decompress(pay, raw.width, raw.height, q)
    f, big = chef_big
    pay = R.compress(big, f.width, f.height, (50, 50, 50), variant="hipplugin")
    assert hashlib.sha256(pay).hexdigest() == hashlib.sha256(oracle.compress(big, f.width, f.height, (50, 50, 50))).hexdigest()
    # the plugin's errors are the reference's messages
    with pytest.raises(R.RefError, match="Level of quality must be between 1 and 100"):
        R.compress(raw.data, raw.width, raw.height, (0, 50, 50), variant="hipplugin")
