"""CPU restatement (oracle/) pinned against the reference's own fixtures and,
when oracle/_ref was built from the reference sources, against the reference
library itself.  No GPU needed."""
import hashlib
import os

import numpy as np
import pytest

import blockgen
import synth

ZZ = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
               41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15,
               23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_fixture_hashes(golden):
    """The committed fixtures are the reference's images."""
    import os
    from conftest import GOLDEN
    pins = {
        "chef-with-trumpet.myyuv": "28ebaf7a645baf6fe39fabb89ca7e8e934e260ad66230d023bc6ed46abc0d80e",
        "chef-with-trumpet-DCT-50.myyuv": "080260fe22a0cba6b81e34619480a211e7a452a8179cb95b15c4a5cd5a16c4e8",
        "chef-with-trumpet-DCT-90.myyuv": "bf3060f50306770ac3f8fb1632cd405036bef76529868f309a7ddc46d7c4e936",
        "chef-with-trumpet-big-DCT-50.myyuv": "c206e462e3af517680615f3b46750098652c165ebfb38ea1d5bcdf3919647e62",
    }
    for name, h in pins.items():
        with open(os.path.join(GOLDEN, name), "rb") as f:
            assert sha(f.read()) == h, name


@pytest.mark.parametrize("q,gold", [(50, "chef-with-trumpet-DCT-50.myyuv"),
                                    (90, "chef-with-trumpet-DCT-90.myyuv")])
def test_oracle_golden_compress(oracle, golden, q, gold):
    raw = golden("chef-with-trumpet.myyuv")
    g = golden(gold)
    assert oracle.compress(raw.data, raw.width, raw.height, (q, q, q)) == g.data


def test_oracle_golden_decompress(oracle, golden):
    g = golden("chef-with-trumpet-DCT-50.myyuv")
    out = oracle.decompress(g.data, g.width, g.height, tuple(g.params))
    assert sha(g.decompressed(out).dumps()) == \
        "a95127da471524c1f7860c47d9b11e2c835ffa220c6d7aadf71e0fb6e45a9306"


def test_oracle_big_pins(oracle, chef_big):
    f, raw = chef_big
    dec = f.decompressed(raw)
    assert sha(dec.dumps()) == "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"
    pay = oracle.compress(raw, f.width, f.height, (50, 50, 50))
    assert len(pay) == 3363749
    assert sha(dec.compressed(b"222", pay).dumps()) == \
        "18405d3e6f79a0054fbdb166ae76f58d8dbffc605263f4c3c0b65e51babefbf7"


def test_synthetic_generators(chef_big):
    import myyuv_file
    assert bytes(synth.splitmix64_bytes(8)) == bytes.fromhex("db1c182f1bf60cbb")
    f, raw = chef_big
    t = synth.tiled_frame(raw, f.width, f.height, 3840, 2160)
    img = myyuv_file.YUVFile(width=3840, height=2160, data=t.tobytes())
    assert sha(img.dumps()) == "d578631d41859dcd4b94de5784a9435a638c8127e478a062db47f13804455127"


def test_tiled_4k_known_answers(oracle, chef_big):
    """tiled 3840x2160 q50 payload size and file hash."""
    import myyuv_file
    f, raw = chef_big
    t = synth.tiled_frame(raw, f.width, f.height, 3840, 2160).tobytes()
    pay = oracle.compress(t, 3840, 2160, (50, 50, 50))
    assert len(pay) == 2155708
    img = myyuv_file.YUVFile(width=3840, height=2160, data=t)
    assert sha(img.compressed(b"222", pay).dumps()) == \
        "f7de6788c9c7574eeb145689a55936f2d5f9d9e4740e6d70198b9976298d5d31"


def test_block_roundtrip_edge_classes(oracle):
    """Every edge-class block encodes to a chunk that decodes back to itself."""
    for name, b in blockgen.edge_blocks():
        nat = np.zeros(64, np.int16)
        nat[ZZ] = b
        ch = oracle.huff_encode_block(nat)
        assert 7 <= len(ch) <= 155, name
        assert np.array_equal(oracle.huff_decode_block(ch), nat), name


def test_kat_fixture(oracle):
    """Committed per-block known answers (tests/golden/block_kats.npz, made
    by tests/golden/make_kats.py from the pinned oracle)."""
    import os
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "block_kats.npz"))
    coefs, sizes, chunks = d["coef_zz"], d["sizes"], d["chunks"]
    off = 0
    for i in range(len(coefs)):
        nat = np.zeros(64, np.int16)
        nat[ZZ] = coefs[i]
        ch = oracle.huff_encode_block(nat)
        assert ch == chunks[off:off + sizes[i]].tobytes(), i
        off += sizes[i]


def test_length8_table_decodes(oracle):
    """A chunk whose table has a length-8 group (legal in the format, never
    emitted by the encoder) decodes like the reference's bit-serial decoder:
    lengths 1..8 with one symbol each plus two of length 8."""
    # canonical codes: L1:0, L2:10, L3:110, ..., L7:1111110, L8: 11111110, 11111111
    syms = [5, -3, 7, 9, -11, 13, 2]
    l8 = [100, -100]
    table = bytearray()
    for L, s in enumerate(syms, start=1):
        table.append(((L - 1) << 5) | 0)
        u = s & 0x7FF
        table += bytes([u & 0xFF, u >> 8])
    table.append((7 << 5) | 1)
    packed = (l8[0] & 0x7FF) | ((l8[1] & 0x7FF) << 11)
    table += packed.to_bytes(3, "little")
    # message: 5, 100, -100, 13
    codes = ["0", "11111110", "11111111", "111110"]
    bits = "".join(codes)
    nb = len(bits)
    enc = bytearray((nb + 7) // 8)
    for t, c in enumerate(bits):
        if c == "1":
            enc[t >> 3] |= 1 << (t & 7)
    chunk = bytes([nb & 0xFF, nb >> 8, len(table)]) + bytes(table) + bytes(enc)
    out = oracle.huff_decode_block(chunk)
    exp = np.zeros(64, np.int16)
    exp[ZZ[:4]] = [5, 100, -100, 13]
    assert np.array_equal(out, exp)


@pytest.fixture(scope="module")
def ref():
    from oracle import ref as R
    if not R.available("omp") or not R.available("serial"):
        pytest.skip("oracle/_ref not built (needs /root/reference; `make -C oracle ref`)")
    return R


@pytest.mark.parametrize("q", [1, 5, 25, 50, 51, 75, 90, 99, 100])
def test_oracle_vs_reference_edge_frame(oracle, ref, q):
    w, h = 256, 128
    fr = blockgen.edge_frame(w, h).tobytes()
    a = oracle.compress(fr, w, h, (q, q, q))
    assert a == ref.compress(fr, w, h, (q, q, q), "serial")
    assert a == ref.compress(fr, w, h, (q, q, q), "omp")
    assert oracle.decompress(a, w, h, (q, q, q)) == ref.decompress(a, w, h, (q, q, q), "serial")


@pytest.mark.parametrize("q", [(50, 50, 50), (90, 90, 90), (100, 100, 100), (3, 60, 97)])
def test_oracle_vs_reference_noise(oracle, ref, q):
    w, h = 512, 256
    fr = synth.noise_frame(w, h).tobytes()
    a = oracle.compress(fr, w, h, q)
    assert a == ref.compress(fr, w, h, q)
    assert oracle.decompress(a, w, h, q) == ref.decompress(a, w, h, q)


def test_oracle_vs_reference_big(oracle, ref, chef_big):
    f, raw = chef_big
    for q in ((90, 90, 90), (20, 40, 60)):
        assert oracle.compress(raw, f.width, f.height, q) == ref.compress(raw, f.width, f.height, q)


MSGS = {2: "Level of quality must be between 1 and 100", 3: "Error. width % 8 must be 0",
        4: "Error. height % 8 must be 0", 6: "DCTYUV load bad size",
        7: "DCTYUVPlane load bad size", 8: "DCTYUVPlane load chunks_sizes_size bad size",
        9: "DCTYUVPlane load content_size bad size", 10: "Huffman bad code",
        11: "Huffman unknown symbol"}


def _oracle_code(fn):
    try:
        fn()
        return 0
    except RuntimeError as e:
        return e.args[0]


@pytest.mark.parametrize("gold", ["chef-with-trumpet-DCT-50.myyuv", "chef-with-trumpet-DCT-90.myyuv"])
def test_error_behaviour_vs_reference(oracle, ref, golden, gold):
    """Malformed streams with a defined reference outcome fail with the
    reference's exact message; bad arguments likewise."""
    import malformed
    g = golden(gold)
    w, h, q = g.width, g.height, tuple(g.params)
    for name, pay, kind in malformed.cases(g.data):
        if kind != "defined":
            continue
        code = _oracle_code(lambda: oracle.decompress(pay, w, h, q))
        assert code in MSGS, (name, code)
        with pytest.raises(ref.RefError) as e:
            ref.decompress(pay, w, h, q, "serial")
        assert str(e.value) == MSGS[code], name
    assert _oracle_code(lambda: oracle.decompress(g.data, w, h, (0, 50, 50))) == 2
    with pytest.raises(ref.RefError) as e:
        ref.decompress(g.data, w, h, (0, 50, 50))
    assert str(e.value) == MSGS[2]
    for (ww, hh, code) in ((72, 64, 3), (64, 72, 4), (40, 64, 3), (64, 40, 4)):
        assert _oracle_code(lambda: oracle.compress(bytes(ww * hh * 3 // 2), ww, hh, (50, 50, 50))) == code
        with pytest.raises(ref.RefError) as e2:
            ref.compress(bytes(ww * hh * 3 // 2), ww, hh, (50, 50, 50), "serial")
        assert str(e2.value) == MSGS[code]


def test_tiled_8192_q50_known_answer(oracle, chef_big):
    """tiled 8192x8192 input and q50 file hashes."""
    import myyuv_file
    f, raw = chef_big
    t = synth.tiled_frame(raw, f.width, f.height, 8192, 8192).tobytes()
    img = myyuv_file.YUVFile(width=8192, height=8192, data=t)
    assert sha(img.dumps()) == "02843f4286c9b8a8d15272c7900283de3a8241725f2a42f805aea41ec46f5813"
    pay = oracle.compress(t, 8192, 8192, (50, 50, 50))
    assert len(pay) == 18269428
    assert sha(img.compressed(b"222", pay).dumps()) == \
        "ef0d2416b76466116558ea341c732123cc72657fe9969d54813327a3c97c236d"


def test_noise_4k_known_answer(oracle):
    import myyuv_file
    n = synth.noise_frame(3840, 2160).tobytes()
    img = myyuv_file.YUVFile(width=3840, height=2160, data=n)
    assert sha(img.dumps()).startswith("9a69b129")
    pay = oracle.compress(n, 3840, 2160, (50, 50, 50))
    assert len(pay) == 9613725
    assert sha(img.compressed(b"222", pay).dumps()).startswith("88ba856a")


@pytest.mark.parametrize("f", [0, 1, 300, 511])
def test_batch4k_manifest(oracle, chef_big, f):
    """tests/golden/batch4k_512.json (BASELINE configs[3]/[4], made by
    tests/golden/make_batch4k.py): frame f's generated input, its q50 stream
    and its decode agree with the oracle here; frame 0 is SURVEY.md §8(d)'s
    pinned tiled 4K file (f7de6788...).  The torch generator the bench and
    the GPU test use equals the numpy one."""
    import hashlib
    import json
    import torch
    import myyuv_file
    import synth
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "batch4k_512.json")) as fh:
        man = json.load(fh)
    assert man["frames_total"] == len(man["frames"]) == 512 and man["quality"] == 50
    m = man["frames"][f]
    g, raw = chef_big
    ox, oy = synth.batch_origin(f, g.width, g.height)
    assert m["f"] == f and m["origin"] == [ox, oy]
    px = synth.tiled_frame(raw, g.width, g.height, 3840, 2160, ox, oy).tobytes()
    tpx = synth.tiled_frame_torch(torch.frombuffer(bytearray(raw), dtype=torch.uint8), g.width, g.height,
                                  3840, 2160, ox, oy)
    assert bytes(tpx.numpy()) == px
    sha = lambda b: hashlib.sha256(b).hexdigest()  # noqa: E731
    assert sha(px) == m["input_sha"]
    pay = oracle.compress(px, 3840, 2160, (50, 50, 50))
    assert len(pay) == m["payload_size"] and sha(pay) == m["payload_sha"]
    assert sha(oracle.decompress(pay, 3840, 2160, (50, 50, 50))) == m["decoded_sha"]
    if f == 0:
        img = myyuv_file.YUVFile(width=3840, height=2160, data=px)
        assert sha(img.compressed(b"222", pay).dumps()) == \
            "f7de6788c9c7574eeb145689a55936f2d5f9d9e4740e6d70198b9976298d5d31"
