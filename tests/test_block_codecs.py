"""Structural-block decompression (forst_block_uncompress, block_codecs.cc),
what BlockFetcher does after the checksum check (table/block_fetcher.cc:
333-345 -> UncompressSerializedBlock, table/format.cc:637-700).

* zlib, pinned: every compressed index / index-partition block of the SST
  files the reference's own SstFileWriter wrote (tests/golden/sst/builder_*,
  format_version 0-6, i.e. compress_format_version 1 and 2) decodes to what
  Python's zlib makes of the raw deflate stream, and the decoded index blocks
  list the handles of the file's data blocks;
* LZ4 / ZSTD / BZip2 (the image has their runtime libraries, no reference
  build with them): blocks made with the same libraries' compressors in
  RocksDB's block format (util/compression.h: varint32 size in front for
  compress_format_version 2; LZ4's 8-byte legacy header for version 1)
  round-trip -- "parity unpinned" for these codecs;
* Snappy (ForSt's default, options/options.cc:123), decoded from the
  published block format: streams made by the real snappy library (pyarrow
  bundles it; Snappy_Compress calls the same snappy::RawCompress) decode to
  their input; hand-assembled streams cover every tag kind (literals with
  0-4 length bytes, copies with 1/2/4-byte offsets, overlapping copies); and
  every accept / reject verdict on hand-made and randomly mutated streams
  equals the real snappy::RawUncompress's (through pyarrow) -- parity with
  the reference's Snappy_Uncompress (util/compression.h:729-754) is
  therefore pinned to the library it calls, not to a reference build (the
  image has no libsnappy for one);
* corrupt / truncated streams and XPRESS give the reference's Status texts."""
import ctypes
import json
import os
import struct
import zlib

import numpy as np
import pytest

import sstwalk
from forst_amd._lib import lib

HERE = os.path.dirname(os.path.abspath(__file__))
BUILDER = json.load(open(os.path.join(HERE, "golden", "sst", "builder_manifest.json")))["files"]


def uncompress(ctype, fv, data, cap=1 << 22):
    out = np.zeros(cap, np.uint8)
    n = ctypes.c_uint64()
    err = ctypes.c_char_p()
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    rc = lib().forst_block_uncompress(ctype, fv, src.ctypes.data, len(data), out.ctypes.data,
                                      cap, ctypes.byref(n), ctypes.byref(err))
    return rc, out[:n.value].tobytes() if rc == 0 else (err.value or b"").decode()


def varint32(n):
    out = bytearray()
    while n >= 128:
        out.append((n & 127) | 128)
        n >>= 7
    out.append(n)
    return bytes(out)


def test_zlib_structural_blocks_of_reference_files():
    n = 0
    for e in BUILDER:
        f = open(os.path.join(HERE, "golden", "sst", e["file"]), "rb").read()
        fv = e["format_version"]
        for kind, off, size, t in e["blocks"]:
            if t != 2 or kind not in ("index", "index_partition", "data") or \
                    (kind == "data" and e["dict_bytes"]):  # (dictionary-compressed)
                continue
            rc, got = uncompress(2, fv, f[off:off + size])
            assert rc == 0, (e["file"], kind, got)
            assert got == sstwalk.contents(f, (off, size), fv)
            n += 1
    assert n > 100


def _lib(name):
    try:
        return ctypes.CDLL(name)
    except OSError:
        pytest.skip(f"{name} not on this machine")


def test_lz4_zstd_bzip2_round_trip():
    rng = np.random.default_rng(1)
    raw = (b"".join(rng.choice([b"state", b"flink", b"window", b"key00"], 3000))
           + rng.integers(0, 256, 999, np.uint8).tobytes())
    # LZ4 (4) and LZ4HC (5): LZ4_compress_default
    L = _lib("liblz4.so.1")
    L.LZ4_compressBound.restype = ctypes.c_int
    cap = L.LZ4_compressBound(len(raw))
    buf = ctypes.create_string_buffer(cap)
    k = L.LZ4_compress_default(raw, buf, len(raw), cap)
    body = buf.raw[:k]
    for t in (4, 5):
        assert uncompress(t, 5, varint32(len(raw)) + body) == (0, raw)
        assert uncompress(t, 1, struct.pack("<II", len(raw), 0) + body) == (0, raw)
    # ZSTD (7): a zstd frame
    Z = _lib("libzstd.so.1")
    Z.ZSTD_compressBound.restype = ctypes.c_size_t
    Z.ZSTD_compress.restype = ctypes.c_size_t
    cap = Z.ZSTD_compressBound(ctypes.c_size_t(len(raw)))
    buf = ctypes.create_string_buffer(cap)
    k = Z.ZSTD_compress(buf, ctypes.c_size_t(cap), raw, ctypes.c_size_t(len(raw)), 3)
    assert uncompress(7, 6, varint32(len(raw)) + buf.raw[:k]) == (0, raw)
    # BZip2 (3): BZ2_bzBuffToBuffCompress
    B = _lib("libbz2.so.1")
    cap = len(raw) * 2 + 600
    buf = ctypes.create_string_buffer(cap)
    dlen = ctypes.c_uint(cap)
    assert B.BZ2_bzBuffToBuffCompress(buf, ctypes.byref(dlen), raw, len(raw), 9, 0, 30) == 0
    body = buf.raw[:dlen.value]
    assert uncompress(3, 5, varint32(len(raw)) + body) == (0, raw)
    assert uncompress(3, 1, body) == (0, raw)


def test_zlib_format_versions_and_errors():
    raw = bytes(range(256)) * 40
    co = zlib.compressobj(6, zlib.DEFLATED, -14)
    body = co.compress(raw) + co.flush()
    assert uncompress(2, 2, varint32(len(raw)) + body) == (0, raw)
    assert uncompress(2, 1, body) == (0, raw)  # compress_format_version 1: no size
    # (raw deflate has no integrity check: a reserved block type is a sure error)
    rc, msg = uncompress(2, 5, varint32(len(raw)) + b"\x07\x00\x00\x00")
    assert rc != 0 and msg == "Corrupted compressed block contents: Zlib"
    rc, msg = uncompress(1, 5, b"\x06hello")
    assert msg == "Corrupted compressed block contents: Snappy"
    rc, msg = uncompress(6, 5, b"\x05hello")
    assert msg == "Unsupported compression method for this build: Xpress"
    assert uncompress(0, 5, b"plain") == (0, b"plain")


def test_bzip2_truncated_stream_is_corrupt_not_a_hang():
    """BZ2_bzDecompress returns BZ_OK, not an error, when its input runs out
    mid-stream; the decoder must report that as corruption (the reference's
    loop, compression.h:1072-1098, would grow its output forever)"""
    B = _lib("libbz2.so.1")
    raw = bytes(range(256)) * 64
    cap = len(raw) * 2 + 600
    buf = ctypes.create_string_buffer(cap)
    dlen = ctypes.c_uint(cap)
    assert B.BZ2_bzBuffToBuffCompress(buf, ctypes.byref(dlen), raw, len(raw), 9, 0, 30) == 0
    body = buf.raw[:dlen.value]
    for cut in (len(body) // 2, len(body) - 1, 10):
        rc, msg = uncompress(3, 5, varint32(len(raw)) + body[:cut])
        assert rc != 0 and msg == "Corrupted compressed block contents: BZip2", (cut, msg)
        rc, msg = uncompress(3, 1, body[:cut])
        assert rc != 0 and msg == "Corrupted compressed block contents: BZip2", (cut, msg)


def test_zlib_empty_block_decodes():
    """a v2 block whose stated size is 0 decodes to nothing (zlib must not be
    handed a null output pointer)"""
    co = zlib.compressobj(6, zlib.DEFLATED, -14)
    body = co.compress(b"") + co.flush()
    assert uncompress(2, 5, varint32(0) + body) == (0, b"")


# ---- Snappy ---------------------------------------------------------------
def _snappy():
    try:
        import pyarrow as pa
        if not pa.Codec.is_available("snappy"):
            raise ImportError
        return pa.Codec("snappy")
    except ImportError:
        pytest.skip("no snappy library (pyarrow) to pin against")


def _snappy_len(data):
    """the preamble varint as snappy parses it (<= 5 bytes, 32 bits), or None"""
    r = 0
    for i, b in enumerate(data[:5]):
        if i == 4 and b >= 16:
            return None
        r |= (b & 127) << (7 * i)
        if not b & 128:
            return r
    return None


def real_snappy(data):
    """snappy::RawUncompress's verdict: (0, bytes) or (nonzero, None)"""
    c = _snappy()
    n = _snappy_len(data)
    if n is None or n > 1 << 24:
        return 1, None
    try:
        return 0, c.decompress(data, decompressed_size=n, asbytes=True)[:n]
    except Exception:
        return 1, None


def ours(data, fv=5):
    rc, got = uncompress(1, fv, data, cap=1 << 24)
    if rc:
        assert got == "Corrupted compressed block contents: Snappy", got
        return 1, None
    return rc, got


def lit(b):
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    nb = (n.bit_length() + 7) // 8
    return bytes([(59 + nb) << 2]) + n.to_bytes(nb, "little") + b


def copy1(length, off):
    assert 4 <= length <= 11 and off < 2048
    return bytes([1 | ((length - 4) << 2) | ((off >> 8) << 5), off & 255])


def copy2(length, off):
    return bytes([2 | ((length - 1) << 2)]) + struct.pack("<H", off)


def copy4(length, off):
    return bytes([3 | ((length - 1) << 2)]) + struct.pack("<I", off)


def test_snappy_streams_from_the_real_library():
    c = _snappy()
    rng = np.random.default_rng(7)
    cases = [b"", b"x", b"ab" * 3, bytes(100000), b"a" * 70000,
             rng.integers(0, 256, 5000, np.uint8).tobytes(),
             b"".join(rng.choice([b"user0000", b"flink", b"state-", b"\x00\x01"], 20000)),
             bytes(range(256)) * 300 + rng.integers(0, 4, 70000, np.uint8).tobytes()]
    for raw in cases:
        body = c.compress(raw, asbytes=True)
        for fv in (1, 2, 5, 6):  # Snappy's framing is the same in both format versions
            assert ours(body, fv) == (0, raw), (len(raw), fv)


def test_snappy_every_tag_kind_hand_assembled():
    rng = np.random.default_rng(11)
    r = lambda n: rng.integers(0, 256, n, np.uint8).tobytes()  # noqa: E731
    good = []
    # literals: inline lengths 1..60, then 1/2/3/4 length bytes
    for n in (1, 2, 59, 60, 61, 256, 257, 65536, 65537, 1 << 16 | 5):
        b = r(n)
        good.append((varint32(n) + lit(b), b))
    b4 = r(300)  # a 4-byte length field holding a small length
    good.append((varint32(300) + bytes([63 << 2]) + (299).to_bytes(4, "little") + b4, b4))
    # copies: 1-byte offset (len 4..11, offsets up to 2047), 2- and 4-byte
    # offsets, overlapping (run-length) copies with offset 1 and 2
    base = r(3000)
    for name, tag, ln, off in (("c1", copy1, 4, 1), ("c1", copy1, 11, 2047), ("c1", copy1, 7, 300),
                               ("c2", copy2, 1, 1), ("c2", copy2, 64, 3000), ("c2", copy2, 64, 1),
                               ("c4", copy4, 64, 2999), ("c4", copy4, 33, 2), ("c4", copy4, 1, 3000)):
        out = bytearray(base)
        for _ in range(ln):
            out.append(out[-off])
        good.append((varint32(len(out)) + lit(base) + tag(ln, off), bytes(out)))
    # many elements chained
    out = bytearray(b"abc")
    s = lit(b"abc")
    for i in range(200):
        ln, off = 4 + i % 8, 1 + i % len(out) % 2000
        s += copy1(ln, off)
        for _ in range(ln):
            out.append(out[-off])
        s += lit(bytes([i]))
        out.append(i)
    good.append((varint32(len(out)) + s, bytes(out)))
    good.append((b"\x00", b""))  # empty
    for stream, want in good:
        assert real_snappy(stream) == (0, want)  # the streams are valid snappy
        assert ours(stream) == (0, want)


def test_snappy_bad_streams_rejected_like_the_real_library():
    bad = [
        b"",                                        # no preamble
        b"\x80",                                    # preamble cut
        b"\x80\x80\x80\x80\x80\x01",                # preamble longer than 5 bytes
        b"\xff\xff\xff\xff\x1f",                    # preamble > 32 bits
        b"\x05" + lit(b"abc"),                      # too short output
        b"\x02" + lit(b"abc"),                      # literal past the stated length
        b"\x03" + lit(b"abc") + b"\x00",            # trailing tag, literal cut
        b"\x05" + bytes([60 << 2]),                 # literal length byte missing
        b"\x05" + bytes([62 << 2, 4, 0]),           # 3-byte length cut
        b"\x05" + lit(b"a") + copy1(4, 0),          # offset 0
        b"\x05" + lit(b"a") + copy2(4, 2),          # offset past the output
        b"\x05" + lit(b"a") + copy4(4, 1 << 20),    # offset past the output (4-byte)
        b"\x05" + lit(b"a") + copy2(5, 1),          # copy past the stated length
        b"\x05" + lit(b"a") + bytes([1]),           # copy-1 cut
        b"\x05" + lit(b"a") + bytes([2, 1]),        # copy-2 cut
        b"\x05" + lit(b"a") + bytes([3, 1, 0, 0]),  # copy-4 cut
        b"\x04" + copy1(4, 1),                      # copy into empty output
        b"\x00\x00",                                # element after a complete empty stream
    ]
    for stream in bad:
        assert real_snappy(stream)[0] != 0, stream
        assert ours(stream)[0] != 0, stream


def test_snappy_mutated_streams_agree_with_the_real_library():
    """random single- and multi-byte mutations, truncations and extensions of
    real snappy streams: our verdict and output equal snappy::RawUncompress's
    on every one"""
    c = _snappy()
    rng = np.random.default_rng(2024)
    srcs = [b"".join(rng.choice([b"key", b"value", b"0123", b"zz"], 600)),
            bytes(range(200)) * 10, rng.integers(0, 3, 3000, np.uint8).tobytes()]
    n_ok = n_bad = 0
    for raw in srcs:
        body = bytearray(c.compress(raw, asbytes=True))
        for i in range(700):
            m = bytearray(body)
            k = i % 4
            if k == 0:
                m[int(rng.integers(0, len(m)))] ^= 1 << int(rng.integers(0, 8))
            elif k == 1:
                for _ in range(3):
                    m[int(rng.integers(0, len(m)))] = int(rng.integers(0, 256))
            elif k == 2:
                m = m[:int(rng.integers(0, len(m)))]
            else:
                m += rng.integers(0, 256, int(rng.integers(1, 6)), np.uint8).tobytes()
            want = real_snappy(bytes(m))
            assert ours(bytes(m)) == want, (i, bytes(m[:16]))
            n_ok += want[0] == 0
            n_bad += want[0] != 0
    assert n_ok > 50 and n_bad > 500
