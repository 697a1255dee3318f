"""Malformed DCTYUV streams for the error-behaviour tests.

`defined` cases have a well-defined reference outcome (a std::runtime_error
with a fixed message); `strict` cases are undefined in the reference (it
reads past a chunk or past content_size with asserts compiled out) and this
build rejects them with its own codes — compared GPU vs oracle only."""


def _chunk_size_table(payload):
    nblk = int.from_bytes(payload[12:16], "little")
    sizes = payload[20:20 + nblk]
    return nblk, sizes, 20 + nblk  # first chunk of plane 0 starts after the sizes


def _replace_chunk(payload, new_chunk_fn, min_size=12):
    """Replace the first plane-0 chunk of at least min_size bytes (same size,
    so every other offset is unchanged)."""
    p = bytearray(payload)
    nblk, sizes, c0 = _chunk_size_table(p)
    off = c0
    for k in range(nblk):
        if sizes[k] >= min_size:
            s = sizes[k]
            ch = new_chunk_fn(bytes(p[off:off + s]), s)
            assert len(ch) == s
            p[off:off + s] = ch
            return bytes(p)
        off += sizes[k]
    raise ValueError("no chunk large enough")


def _bits_run_out(chunk, s):
    # table: 0 -> "0" (length 1), 5 -> "10" (length 2); one stream bit "1":
    # the decoder needs a second bit that is not there -> "Huffman bad code"
    table = bytes([(0 << 5) | 0, 0, 0, (1 << 5) | 0, 5, 0])
    body = bytes([1, 0, len(table)]) + table + b"\x01"
    return body + bytes(s - len(body))


def _unknown_symbol(chunk, s):
    # table: one symbol (value 5) of length 2 -> code "00"; bits "11111111..."
    table = bytes([(1 << 5) | 0, 5, 0])
    nbits = 8 * (s - 3 - len(table))
    body = bytes([len(table)]) + table + b"\xff" * (s - 3 - len(table))
    return bytes([nbits & 0xFF, nbits >> 8]) + body


def _pack11(vals):
    acc = 0
    for i, v in enumerate(vals):
        acc |= (v & 0x7FF) << (11 * i)
    return acc.to_bytes((11 * len(vals) + 7) // 8, "little")


def _irregular_chunk(groups, seq, s):
    """A valid chunk whose table is not what the reference encoder writes.
    groups: [(length, [values...]), ...] in stream order (a length may recur:
    Huffman::fromDump appends); seq: values to emit.  Codes follow the
    decoder's rule: length-L codes start at first_L, in append order."""
    by_len = {}
    for L, vals in groups:
        by_len.setdefault(L, []).extend(vals)
    code_of, first = {}, 0
    for L in range(1, 9):
        for k, v in enumerate(by_len.get(L, [])):
            code_of.setdefault(v, (L, first + k))
        first = (first + len(by_len.get(L, []))) << 1
    table = b"".join(bytes([((L - 1) << 5) | (len(v) - 1)]) + _pack11(v) for L, v in groups)
    bits, nbits = 0, 0
    for v in seq:
        L, code = code_of[v]
        for b in range(L - 1, -1, -1):  # MSB-first into an LSB-first stream
            bits |= ((code >> b) & 1) << nbits
            nbits += 1
    body = bytes([nbits & 0xFF, nbits >> 8, len(table)]) + table + \
        bits.to_bytes((nbits + 7) // 8, "little")
    assert len(body) <= s, (len(body), s)
    return body + bytes(s - len(body))


def irregular_cases(payload):
    """(name, payload) of VALID streams with tables outside the encoder's
    form: lengths out of order and split across groups; more than 32 codes of
    one length (two groups).  The decode must match the oracle exactly."""
    g1 = [(3, [-7]), (1, [0]), (3, [1023]), (2, [-1024])]
    seq1 = [0, -7, 1023, 0, -1024, 0, 0, -7, -1024, 1023] * 3
    vals = list(range(-20, 21))  # 41 distinct
    g2 = [(2, [vals[0]]), (7, vals[1:33]), (7, vals[33:])]
    seq2 = vals[:64] + vals[:23]
    out = []
    for name, g, seq in (("split_out_of_order", g1, seq1), ("over_32_per_length", g2, seq2)):
        need = len(_irregular_chunk(g, seq, 4096).rstrip(b"\0")) + 1
        out.append((name, _replace_chunk(payload, lambda c, s, g=g, q=seq: _irregular_chunk(g, q, s),
                                         min_size=need)))
    return out


def cases(payload):
    """(name, payload, kind) with kind 'defined' or 'strict'."""
    data = bytearray(payload)
    out = [
        ("tiny", bytes(data[:8]), "defined"),
        ("truncated", bytes(data[:100]), "defined"),
        ("plane_size_zero", bytes(b"\0\0\0\0" + data[4:]), "defined"),
        ("bad_code", _replace_chunk(payload, _bits_run_out), "defined"),
        ("unknown_symbol", _replace_chunk(payload, _unknown_symbol), "defined"),
    ]
    nblk, sizes, c0 = _chunk_size_table(data)
    small = bytearray(data)
    small[16:20] = (1).to_bytes(4, "little")  # content_size 1: chunks run past it
    out.append(("content_too_small", bytes(small), "strict"))
    over = bytearray(data)
    c_first = c0
    over[c_first] = 0xFF  # nbits past the chunk end
    over[c_first + 1] = 0x01
    out.append(("nbits_past_chunk", bytes(over), "strict"))
    return out
