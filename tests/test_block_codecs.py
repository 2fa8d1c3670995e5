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
* corrupt streams and Snappy / XPRESS give the reference's Status texts."""
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
    rc, msg = uncompress(1, 5, b"\x05hello")
    assert msg == "Unsupported compression method for this build: Snappy"
    rc, msg = uncompress(6, 5, b"\x05hello")
    assert msg == "Unsupported compression method for this build: Xpress"
    assert uncompress(0, 5, b"plain") == (0, b"plain")
