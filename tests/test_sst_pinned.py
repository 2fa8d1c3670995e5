"""SST layout pinned to the reference's own writer code (a11 / f1 / f3).

tests/golden/sst/*.sst were written by tests/golden/gen_sst_golden.py with
every encoding done by the REFERENCE (BlockBuilder, BlockHandle / IndexValue
encoders, PropertyBlockBuilder, MetaIndexBuilder, FooterBuilder::Build,
ComputeBuiltinChecksumWithLastByte + ChecksumModifierForContext, compiled
from /root/reference); tests/golden/ref_footers.json holds FooterBuilder::Build
for format_version 0-6 x the 5 checksum types.  CPU: tests/sstgen.py's
restated encodings write those files byte for byte (so every SST the other
tests generate is pinned), the product's footer decoder reads every reference
footer, and forst_sst_footer_build writes the fv < 6 footers.  GPU: the
whole-file verify accepts every reference file and names the first corrupted
block exactly; the deferred-trailer writer rewrites every reference file byte
for byte from its blocks; fv6 footers (checksum on the GPU) equal the
reference's."""
import json
import os
import struct

import pytest

import sstgen

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "sst", "manifest.json")))["files"]
FOOTERS = json.load(open(os.path.join(GOLD, "ref_footers.json")))["footers"]


def ref_file(e):
    with open(os.path.join(GOLD, "sst", e["file"]), "rb") as fh:
        return fh.read()


def writer(e):
    return sstgen.SstWriter(fv=e["format_version"], ctype=e["checksum"],
                            index_type=e["index_type"], base_context=e["base_context_checksum"],
                            restart_interval=e["restart_interval"], seed=e["seed"])


@pytest.mark.parametrize("e", MANIFEST, ids=[e["file"] for e in MANIFEST])
def test_sstgen_writes_the_reference_bytes(e):
    w = writer(e)
    assert w.build(n_data=e["n_data"], external=e["external"]) == ref_file(e)
    assert [[k, o, n] for k, o, n in w.blocks] == e["blocks"]


def _valid_for_product(fr):
    """footers the reference accepts in a debug build (FooterBuilder::Build's
    asserts, table/format.cc:260-276): fv 0 only with kNoChecksum / kCRC32c,
    fv >= 6 only with a base context checksum"""
    fv, ct, bcc = fr["format_version"], fr["checksum"], fr["base_context_checksum"]
    if fv == 0:
        return ct in (0, 1)
    if fv >= 6:
        return bcc != 0
    return True


def test_pycodec_footers_equal_reference():
    codec = sstgen.PyCodec()
    n = 0
    for fr in FOOTERS:
        if not _valid_for_product(fr):
            continue
        got = codec.footer(fr["format_version"], fr["checksum"], fr["footer_offset"],
                           tuple(fr["metaindex"]), tuple(fr["index"]),
                           fr["base_context_checksum"])
        assert got.hex() == fr["hex"], fr
        n += 1
    assert n == 91


def test_footer_decode_reads_every_reference_footer():
    """Footer::DecodeFrom restated in the product (sst_host.cc) on the
    reference's bytes: version, checksum type, handles, base context"""
    from forst_amd import sst
    for fr in FOOTERS:
        if not _valid_for_product(fr):
            continue
        raw = bytes.fromhex(fr["hex"])
        fv = fr["format_version"]
        # the footer ends the file; the metaindex sits in front of it for fv6
        size = fr["footer_offset"] + len(raw)
        pad = bytes(max(0, 53 - len(raw)))
        f = _decode_tail(sst, pad + raw, size)
        assert f.format_version == fv
        assert f.checksum_type == (1 if fv == 0 else fr["checksum"])
        assert f.footer_offset == fr["footer_offset"]
        if fv < 6:
            assert (f.metaindex_offset, f.metaindex_size) == tuple(fr["metaindex"])
            assert (f.index_offset, f.index_size) == tuple(fr["index"])
        else:
            assert f.base_context_checksum == fr["base_context_checksum"]
            assert f.metaindex_size == fr["metaindex"][1]
            assert f.metaindex_offset == fr["footer_offset"] - 5 - fr["metaindex"][1]


def _decode_tail(sst, tail, file_size):
    import ctypes

    import numpy as np
    a = np.frombuffer(tail, np.uint8).copy()
    f = sst.Footer()
    from forst_amd._lib import lib
    rc = lib().forst_sst_footer_decode(a.ctypes.data, len(a), file_size, ctypes.byref(f))
    assert rc == 0, lib().forst_sst_last_error()
    return f


@pytest.mark.parametrize("fv", [0, 1, 2, 3, 4, 5])
def test_footer_build_equals_reference_without_gpu(fv):
    from forst_amd import table_writer as tw
    for fr in FOOTERS:
        if fr["format_version"] != fv or not _valid_for_product(fr):
            continue
        got = tw.footer_build(fv, fr["checksum"], fr["footer_offset"], 0,
                              tuple(fr["metaindex"]), tuple(fr["index"]))
        assert got.hex() == fr["hex"], fr


@pytest.mark.gpu
def test_footer_build_fv6_equals_reference():
    from forst_amd import table_writer as tw
    n = 0
    for fr in FOOTERS:
        if fr["format_version"] < 6 or not _valid_for_product(fr):
            continue
        got = tw.footer_build(6, fr["checksum"], fr["footer_offset"],
                              fr["base_context_checksum"], tuple(fr["metaindex"]),
                              tuple(fr["index"]))
        assert got.hex() == fr["hex"], fr
        n += 1
    assert n == 10


@pytest.mark.gpu
@pytest.mark.parametrize("e", MANIFEST, ids=[e["file"] for e in MANIFEST])
def test_verify_reference_file_and_a_corrupted_block(e):
    from forst_amd import sst
    f = ref_file(e)
    name = "/db/" + e["file"]
    r = sst.verify_file(f, file_name=name)
    assert r.status == 0, r.message
    data = [(o, n) for k, o, n in e["blocks"] if k == "data"]
    assert r.data_blocks == len(data)
    if e["checksum"] == 0:
        return  # kNoChecksum: nothing to mismatch
    o, n = data[len(data) // 2]
    b = bytearray(f)
    b[o + n // 2] ^= 0x04
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.status == 2
    # the reference's text (table/block_based/reader_common.cc:48-60)
    from oracle import oracle as O
    ct = e["checksum"]
    mod = O.checksum_modifier_for_context(e["base_context_checksum"], o)
    stored = (struct.unpack_from("<I", b, o + n + 1)[0] - mod) & 0xFFFFFFFF
    computed = O.compute_builtin_checksum(ct, bytes(b[o:o + n + 1]))
    if ct == 1:
        stored, computed = O.unmask(stored), O.unmask(computed)
    want = (f"Corruption: block checksum mismatch: stored{'(context removed)' if mod else ''} "
            f"= {stored}, computed = {computed}, type = {ct}  in {name} offset {o} size {n}")
    assert r.message.decode() == want


@pytest.mark.gpu
@pytest.mark.parametrize("window", [4096, 0])
@pytest.mark.parametrize("e", MANIFEST, ids=[e["file"] for e in MANIFEST])
def test_trailer_writer_rewrites_reference_file(e, window):
    """the deferred-trailer writer (table_writer.cc) fed the reference file's
    blocks in builder order reproduces it byte for byte: every trailer from
    the GPU batches, the footer from forst_sst_footer_build"""
    from forst_amd import table_writer as tw
    f = ref_file(e)
    fv = e["format_version"]
    ct = 1 if fv == 0 else e["checksum"]
    tr = tw.TrailerWriter(ct, e["base_context_checksum"], start_offset=0, window_bytes=window)
    hs = {}
    for kind, off, n in sorted(e["blocks"], key=lambda b: b[1]):
        assert tr.add(f[off:off + n], f[off + n], is_data_block=(kind == "data")) == (off, n)
        hs[kind] = (off, n)
    tr.footer(fv, hs["metaindex"], hs["index"])
    assert tr.close() == f


# ---- whole files from the reference's own SstFileWriter (round 3) ----------
BUILDER = json.load(open(os.path.join(GOLD, "sst", "builder_manifest.json")))["files"]


def test_builder_files_tile_and_match_their_manifest():
    """tests/sstwalk.py (the test-side reader used to place corruptions and
    feed the writer) lists exactly the blocks recorded when the reference
    wrote the file, and they tile the file up to the footer; the files hold
    compressed data AND index blocks, filter (full / partitioned), index
    partitions, range deletions and a compression dictionary"""
    import sstwalk
    kinds, types = set(), set()
    for e in BUILDER:
        f = ref_file(e)
        blocks, foot = sstwalk.walk(f)
        assert sstwalk.tiles(blocks, foot), e["file"]
        assert [list(b) for b in blocks] == e["blocks"], e["file"]
        kinds |= {b[0] for b in blocks}
        types |= {(b[0], b[3]) for b in blocks}
    assert {"data", "index", "index_partition", "filter", "filter_index", "filter_partition",
            "rangedel", "dict", "properties", "metaindex"} <= kinds
    assert ("index", 2) in types and ("index_partition", 2) in types and ("data", 2) in types


def _builder_status(r):
    return "OK" if r.status == 0 else r.message.decode()


@pytest.mark.gpu
@pytest.mark.parametrize("e", BUILDER, ids=[e["file"] for e in BUILDER])
def test_verify_builder_file_matches_reference_status(e):
    """forst_sst_verify_file on the reference-built file (zlib-compressed
    index / partitions decoded on the host, every checksum on the GPU): OK;
    and for every single-byte corruption the generator ran through the
    reference's SstFileReader::VerifyChecksum, the same Status text"""
    from forst_amd import sst
    f = ref_file(e)
    name = "/db/" + e["file"]
    r = sst.verify_file(f, file_name=name)
    assert r.status == 0, r.message
    assert r.data_blocks == sum(1 for b in e["blocks"] if b[0] == "data")
    for fl in e["flips"]:
        b = bytearray(f)
        b[fl["offset"]] ^= 0x20 if fl["kind"] != "footer" else 0x01
        got = _builder_status(sst.verify_file(bytes(b), file_name=name))
        want = fl["status"].replace("{file}", name)
        if e["checksum"] == 0 and fl["kind"] in ("index", "metaindex"):
            # kNoChecksum: a corrupted structural block is only found by
            # what its garbage decodes to (the reference's text then comes
            # from its prefetch-buffer read of a garbage handle); both report
            # a Corruption
            assert got.startswith("Corruption: ") and want.startswith("Corruption: "), (fl, got)
            continue
        assert got == want, (e["file"], fl["kind"], got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("e", BUILDER, ids=[e["file"] for e in BUILDER])
def test_trailer_writer_rewrites_builder_file(e):
    """GpuTrailerWriter fed the blocks the reference builder wrote (compressed
    contents with their compression type byte) reproduces the file byte for
    byte, footer included"""
    from forst_amd import table_writer as tw
    f = ref_file(e)
    fv = e["format_version"]
    ct = 1 if fv == 0 else e["checksum"]
    import sstwalk
    foot = sstwalk.footer(f)
    tr = tw.TrailerWriter(ct, foot["bcc"], start_offset=0, window_bytes=8192)
    for kind, off, n, t in e["blocks"]:
        assert tr.add(f[off:off + n], t, is_data_block=(kind == "data")) == (off, n)
    ix = foot["index"] or (0, 0)
    tr.footer(fv, foot["metaindex"], ix)
    assert tr.close() == f
