"""myyuv_cli drop-in: same command line and output files as the reference CLI
(myyuv_cli/main.cpp).  CPU tests cover the paths with no codec work (-info,
argument errors) against the reference CLI built in oracle/_ref; GPU tests run
compress / decompress and compare the files byte for byte."""
import os
import subprocess

import pytest

from conftest import GOLDEN, PKG, ROOT

CLI = os.path.join(PKG, "myyuv_cli")
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "myyuv_cli_ref")
SMALL = os.path.join(GOLDEN, "chef-with-trumpet.myyuv")
C50 = os.path.join(GOLDEN, "chef-with-trumpet-DCT-50.myyuv")


def run(exe, *args):
    return subprocess.run([exe, *args], capture_output=True, text=True)


def need_ref():
    if not os.path.exists(REF_CLI):
        pytest.skip("reference CLI not built (make -C oracle ref)")


@pytest.mark.parametrize("path", [SMALL, C50])
def test_info_matches_reference(path):
    need_ref()
    a, b = run(CLI, path, "-info"), run(REF_CLI, path, "-info")
    assert a.returncode == b.returncode == 0
    assert a.stdout == b.stdout


def test_argument_errors_match_reference(tmp_path):
    need_ref()
    for args in ([SMALL, "-bogus"], [SMALL, "-compress"], [SMALL, "-compress", "DCT", "50"],
                 [SMALL, "-decompress", "-o", str(tmp_path / "x")], [C50, "-decompress", "x"]):
        a, b = run(CLI, *args), run(REF_CLI, *args)
        assert a.returncode == b.returncode, args
        assert a.stdout.splitlines()[0] == b.stdout.splitlines()[0], args


def test_no_args_prints_usage():
    r = run(CLI, SMALL)
    assert r.returncode == 0 and "Usage" in r.stdout


def test_unknown_magic_fails(tmp_path):
    p = tmp_path / "junk.bin"
    p.write_bytes(b"XXjunk")
    r = run(CLI, str(p), "-info")
    assert r.returncode != 0
    assert "Unknown image format (magic)" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("q,gold", [(["50"], "chef-with-trumpet-DCT-50.myyuv"),
                                    (["90", "90", "90"], "chef-with-trumpet-DCT-90.myyuv")])
def test_cli_compress_matches_golden(tmp_path, q, gold):
    out = tmp_path / "out.myyuv"
    r = run(CLI, SMALL, "-compress", "DCT", *q, "-o", str(out))
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("YUV DCT compression (") and r.stdout.rstrip().endswith("Success!")
    assert out.read_bytes() == open(os.path.join(GOLDEN, gold), "rb").read()


@pytest.mark.gpu
def test_cli_decompress_matches_reference(tmp_path, oracle, golden):
    out = tmp_path / "dec.myyuv"
    r = run(CLI, C50, "-decompress", "-o", str(out))
    assert r.returncode == 0, r.stderr
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    exp = g.decompressed(oracle.decompress(g.data, g.width, g.height, tuple(g.params))).dumps()
    assert out.read_bytes() == exp
    if os.path.exists(REF_CLI):
        ref_out = tmp_path / "ref.myyuv"
        assert run(REF_CLI, C50, "-decompress", "-o", str(ref_out)).returncode == 0
        assert out.read_bytes() == ref_out.read_bytes()


@pytest.mark.gpu
def test_cli_roundtrip_big(tmp_path):
    big = os.path.join(GOLDEN, "chef-with-trumpet-big-DCT-50.myyuv")
    dec, rec = tmp_path / "dec.myyuv", tmp_path / "rec.myyuv"
    assert run(CLI, big, "-decompress", "-o", str(dec)).returncode == 0
    assert run(CLI, str(dec), "-compress", "DCT", "50", "-o", str(rec)).returncode == 0
    import hashlib
    assert hashlib.sha256(dec.read_bytes()).hexdigest() == \
        "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"
    assert hashlib.sha256(rec.read_bytes()).hexdigest() == \
        "18405d3e6f79a0054fbdb166ae76f58d8dbffc605263f4c3c0b65e51babefbf7"


@pytest.mark.gpu
def test_cli_bad_quality_fails_like_reference(tmp_path):
    r = run(CLI, SMALL, "-compress", "DCT", "0", "-o", str(tmp_path / "x"))
    assert r.returncode != 0
    assert "Compression parameters for DCT must range between [1..100]" in r.stderr


def _bmp_file(tmp_path):
    import gzip

    p = tmp_path / "chef.bmp"
    p.write_bytes(gzip.open(os.path.join(GOLDEN, "chef-with-trumpet.bmp.gz")).read())
    return str(p)


def test_bmp_info_matches_reference(tmp_path):
    need_ref()
    bmp = _bmp_file(tmp_path)
    a, b = run(CLI, bmp, "-info"), run(REF_CLI, bmp, "-info")
    assert a.returncode == b.returncode == 0
    assert a.stdout == b.stdout


def test_bmp_argument_errors_match_reference(tmp_path):
    need_ref()
    bmp = _bmp_file(tmp_path)
    for args in ([bmp, "-bogus"], [bmp, "-to_yuv", "IYUV"], [bmp, "-to_yuv", "IYUV", "-x", "o"]):
        a, b = run(CLI, *args), run(REF_CLI, *args)
        assert a.returncode == b.returncode, args
        assert a.stdout.splitlines()[0] == b.stdout.splitlines()[0], args


@pytest.mark.gpu
def test_cli_to_yuv_matches_golden(tmp_path):
    """myyuv_cli chef.bmp -to_yuv IYUV -o out: the reference's own
    chef-with-trumpet.myyuv, byte for byte (header included)."""
    out = tmp_path / "o.myyuv"
    r = run(CLI, _bmp_file(tmp_path), "-to_yuv", "IYUV", "-o", str(out))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "BMP to YUV (IYUV) : " in r.stdout and r.stdout.endswith("Success!\n")
    assert out.read_bytes() == open(SMALL, "rb").read()


@pytest.mark.gpu
def test_cli_batch_compress_matches_per_file(tmp_path, golden, oracle):
    """-batch-compress (many frames per invocation): two
    copies of the small golden frame and a frame of another geometry; every
    output equals the per-file result (the golden DCT-50 file for chef)."""
    import numpy as np
    import myyuv_file
    a = tmp_path / "a.myyuv"
    b = tmp_path / "b.myyuv"
    c = tmp_path / "c.myyuv"
    a.write_bytes(open(SMALL, "rb").read())
    b.write_bytes(open(SMALL, "rb").read())
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 256, 128 * 64 * 3 // 2).astype(np.uint8).tobytes()
    myyuv_file.YUVFile(width=128, height=64, data=raw).dump(str(c))
    out = tmp_path / "out"
    out.mkdir()
    r = run(CLI, "-batch-compress", "DCT", "50", "-o", str(out), str(a), str(b), str(c))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "(3 frames)" in r.stdout and r.stdout.endswith("Success!\n")
    gold = open(C50, "rb").read()
    assert (out / "a.myyuv").read_bytes() == gold
    assert (out / "b.myyuv").read_bytes() == gold
    one = tmp_path / "c1.myyuv"
    assert run(CLI, str(c), "-compress", "DCT", "50", "-o", str(one)).returncode == 0
    assert (out / "c.myyuv").read_bytes() == one.read_bytes()
    # and back: -batch-decompress equals -decompress per file
    dec = tmp_path / "dec"
    dec.mkdir()
    # (with an uncompressed frame, which -decompress copies, and another quality)
    q90 = tmp_path / "q90.myyuv"
    assert run(CLI, str(a), "-compress", "DCT", "90", "-o", str(q90)).returncode == 0
    ra = tmp_path / "raw_a.myyuv"
    ra.write_bytes(open(SMALL, "rb").read())
    r = run(CLI, "-batch-decompress", "-o", str(dec), str(out / "a.myyuv"), str(out / "c.myyuv"), str(ra),
            str(q90), str(out / "b.myyuv"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "(5 frames)" in r.stdout
    one_d = tmp_path / "c1d.myyuv"
    assert run(CLI, str(one), "-decompress", "-o", str(one_d)).returncode == 0
    assert (dec / "c.myyuv").read_bytes() == one_d.read_bytes()
    per_file = tmp_path / "d_q90.myyuv"
    assert run(CLI, str(q90), "-decompress", "-o", str(per_file)).returncode == 0
    assert (dec / "q90.myyuv").read_bytes() == per_file.read_bytes()
    # (-decompress refuses an uncompressed file; the batch copies it, as YUV::decompress does)
    # (its header as YUV::load normalises it: compression_params_pos = 64, myyuv_yuv.cpp:501)
    want_raw = bytearray(open(SMALL, "rb").read())
    want_raw[16:20] = (64).to_bytes(4, "little")
    assert (dec / "raw_a.myyuv").read_bytes() == bytes(want_raw)
    assert (dec / "b.myyuv").read_bytes() == (dec / "a.myyuv").read_bytes()
    want = myyuv_file.YUVFile.load(gold)
    assert myyuv_file.YUVFile.load(str(dec / "a.myyuv")).data == oracle.decompress(want.data, 992, 736, (50, 50, 50))


@pytest.mark.gpu
def test_python_compress_batch(codec, golden, chef_big):
    f, raw = chef_big
    small = golden("chef-with-trumpet.myyuv").data
    pays = codec.compress_batch([raw, raw], f.width, f.height, (50, 50, 50))
    one = codec.compress(raw, f.width, f.height, (50, 50, 50))
    assert pays == [one, one]
    assert codec.compress_batch([small], 992, 736, (50, 50, 50)) == [golden("chef-with-trumpet-DCT-50.myyuv").data]


def test_batch_rejects_duplicate_output_names(tmp_path):
    """Batch outputs are OUTDIR/<input file name>: two inputs with the same
    file name from different directories are refused before any work."""
    d1, d2, out = tmp_path / "a", tmp_path / "b", tmp_path / "out"
    for d in (d1, d2, out):
        d.mkdir()
    data = open(SMALL, "rb").read()
    (d1 / "f.myyuv").write_bytes(data)
    (d2 / "f.myyuv").write_bytes(data)
    r = run(CLI, "-batch-compress", "DCT", "50", "-o", str(out), str(d1 / "f.myyuv"), str(d2 / "f.myyuv"))
    assert r.returncode != 0
    assert "share the file name f.myyuv" in r.stderr
    assert not os.listdir(out)


@pytest.mark.gpu
def test_python_compress_batch_checks_frame_sizes(codec):
    raw = open(SMALL, "rb").read()[64:]
    with pytest.raises(ValueError, match="frame 1"):
        codec.compress_batch([raw, raw[:-1]], 992, 736, (50, 50, 50))


@pytest.mark.gpu
def test_cli_batch_compress_over_devices(tmp_path, oracle):
    """-batch-compress -devices 0,0,0: frames dealt round-robin over three
    host threads with a codec context each (the C++ side of the
    frame-per-GPU sharding; one physical GPU here, so the three
    entries name the same device); every output equals the per-file result."""
    import numpy as np
    import myyuv_file
    rng = np.random.default_rng(9)
    files = []
    for i in range(7):  # mixed geometries, uneven shares (3, 2, 2)
        w, h = (128, 64) if i % 2 else (256, 128)
        raw = rng.integers(0, 256, w * h * 3 // 2).astype(np.uint8).tobytes()
        p = tmp_path / f"f{i}.myyuv"
        myyuv_file.YUVFile(width=w, height=h, data=raw).dump(str(p))
        files.append(p)
    out = tmp_path / "out"
    out.mkdir()
    r = run(CLI, "-batch-compress", "DCT", "60", "-devices", "0,0,0", "-o", str(out), *map(str, files))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "(7 frames)" in r.stdout
    for p in files:
        f = myyuv_file.YUVFile.load(str(p))
        want = f.compressed(bytes([60] * 3), oracle.compress(f.data, f.width, f.height, (60, 60, 60))).dumps()
        assert (out / p.name).read_bytes() == want, p.name
