"""Corrupted-input corpus for the host parsers that read untrusted file bytes
(sst_host.cc, block_codecs.cc): every truncation of reference-written footers,
index partitions and properties blocks, block handles with oversized varint64s,
and compressed blocks whose size preamble lies.  Each call must return data or
a clean error -- never read out of bounds.  tools/asan_cpu.sh runs this file
(with test_sst.py, test_block_codecs.py, test_table_writer.py, the emulator
tests) against lib/libforst_checksum_asan.so under AddressSanitizer and
UndefinedBehaviorSanitizer; without the sanitizers it still checks the
verdicts.  References: table/format.cc:334-463 (Footer::DecodeFrom),
:69-78 (BlockHandle::DecodeFrom), :124-148 (IndexValue::DecodeFrom),
block_based_table_reader.cc:2457-2574, util/compression.h:729-754."""
import json
import os
import zlib

import numpy as np
import pytest

import sstwalk
from forst_amd import sst
from test_block_codecs import uncompress, varint32

HERE = os.path.dirname(os.path.abspath(__file__))
BUILDER = json.load(open(os.path.join(HERE, "golden", "sst", "builder_manifest.json")))["files"]


def _files():
    for f in BUILDER:
        yield f, open(os.path.join(HERE, "golden", "sst", f["file"]), "rb").read()


def test_every_footer_truncation():
    """the tail of every reference file cut to every length 0..file end: a
    decoded footer or SstCorruption"""
    seen_ok = 0
    for f, data in _files():
        for cut in list(range(0, 80)) + [len(data) - k for k in range(0, 64)]:
            tail = data[:cut] if cut <= len(data) else data
            try:
                sst.decode_footer(tail)
                seen_ok += 1
            except sst.ForstError:
                pass
    assert seen_ok > 0


def test_footer_bytes_overwritten():
    """every byte of every footer set to 0x00, 0x80 (a varint continuation that
    runs on) and 0xff, one at a time"""
    for f, data in _files():
        n = len(data)
        for k in range(1, 54):
            for v in (0x00, 0x80, 0xFF):
                b = bytearray(data)
                b[n - k] = v
                try:
                    sst.decode_footer(bytes(b))
                except sst.ForstError:
                    pass


def _index_blocks():
    for f, data in _files():
        blocks, foot = sstwalk.walk(data)
        for kind, o, n, t in blocks:
            if kind in ("index", "index_partition"):
                try:
                    blk = sstwalk.contents(data, (o, n), f["format_version"])
                except Exception:
                    continue
                yield f, blk


def test_index_partitions_truncated_at_every_byte():
    k = 0
    for f, blk in _index_blocks():
        delta = f["format_version"] >= 4
        first = f["index_type"] == 3
        for cut in range(0, len(blk) + 1, max(1, len(blk) // 97)):
            try:
                sst.index_handles(blk[:cut], delta, first)
            except sst.ForstError:
                pass
        k += 1
    assert k > 5


def test_block_handles_with_oversized_varints():
    """index entries whose BlockHandle varint64s run 10+ bytes (past 64 bits) or
    never end, and restart arrays pointing past the block"""
    def block(entries, restarts=None):
        body = b""
        offs = []
        for key, value in entries:
            offs.append(len(body))
            body += varint32(0) + varint32(len(key)) + varint32(len(value)) + key + value
        r = restarts if restarts is not None else offs
        return body + b"".join(x.to_bytes(4, "little") for x in r) + len(r).to_bytes(4, "little")

    cases = [
        block([(b"k1", b"\xff" * 10 + b"\x01" + b"\x05")]),    # offset varint > 64 bits
        block([(b"k1", b"\xff" * 20)]),                          # never terminates
        block([(b"k1", b"\x80\x80\x80\x80\x80\x80\x80\x80\x80\x01\x05")]),
        block([(b"k1", b"\x05")]),                               # size missing
        block([(b"k1", b"\x05\x06")], restarts=[10_000]),       # restart past the block
        block([(b"k1", b"\x05\x06")], restarts=[2**32 - 1]),
        b"\x00\x00\x00\x00",                                     # zero restarts, no entries
        b"\xff\xff\xff\x7f",                                     # restart count huge
    ]
    for blk in cases:
        for delta in (False, True):
            try:
                sst.index_handles(blk, delta, False)
            except sst.ForstError:
                pass


def test_properties_blocks_truncated_and_mutated():
    rng = np.random.default_rng(3)
    for f, data in _files():
        blocks, foot = sstwalk.walk(data)
        for kind, o, n, t in blocks:
            if kind != "properties":
                continue
            blk = sstwalk.contents(data, (o, n), f["format_version"])
            for cut in range(0, len(blk) + 1, max(1, len(blk) // 61)):
                try:
                    sst.properties(blk[:cut])
                except sst.ForstError:
                    pass
            for _ in range(40):
                b = bytearray(blk)
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
                try:
                    sst.properties(bytes(b))
                except sst.ForstError:
                    pass


def test_compressed_blocks_with_lying_size_preambles():
    """zlib (compress_format_version 2: varint32 decompressed size in front) and
    Snappy (its own varint32 length) whose stated size is too small, too big,
    enormous, or cut short.  zlib: the stated size only sizes the first output
    buffer, which grows as inflate needs (Zlib_Uncompress, util/compression.h:
    917-944), so the result is the true contents or an error; Snappy: its
    length is binding, so anything but the true length is an error."""
    raw = b"state value checkpoint " * 300
    z = zlib.compressobj(6, zlib.DEFLATED, -14)
    deflated = z.compress(raw) + z.flush()
    for stated in (0, 1, len(raw) - 1, len(raw), len(raw) + 1, 1 << 20, (1 << 32) - 1):
        blk = varint32(stated) + deflated
        rc, out = uncompress(2, 5, blk)
        if rc == 0:
            assert out == raw, stated
    for cut in range(0, 6):
        uncompress(2, 5, b"\xff\xff\xff\xff\x0f"[:cut])
    for stated in (0, 5, 300, (1 << 32) - 1):  # snappy: one 255-byte literal
        lit = bytes([60 << 2, 254]) + raw[:255]
        rc, out = uncompress(1, 5, varint32(stated) + lit)
        if rc == 0:
            assert len(out) == stated == 255
    # a caller's output buffer far smaller than the contents
    rc, out = uncompress(2, 5, varint32(len(raw)) + deflated, cap=64)
    assert rc != 0


@pytest.mark.parametrize("ctype", [1, 2, 4, 5, 7])
def test_random_bytes_as_compressed_blocks(ctype):
    """500 random byte strings per codec (Snappy, zlib, LZ4, ZSTD, BZip2
    where the runtime library exists): decoded or rejected, no crash.  (A
    random size preamble can state up to 4 GiB, which the codecs allocate
    and zero as the reference allocates it: some calls take 0.1 s.)"""
    rng = np.random.default_rng(ctype)
    for i in range(500):
        n = int(rng.integers(0, 300))
        b = rng.integers(0, 256, n, np.uint8).tobytes()
        if i % 3 == 0 and n:
            b = varint32(int(rng.integers(0, 5000))) + b
        uncompress(ctype, 2 + (i & 3), b, cap=1 << 16)
