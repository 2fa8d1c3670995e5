"""Whole-SST-file checksum verification (§8f-1, BlockBasedTable::VerifyChecksum,
block_based_table_reader.cc:2457-2574).

CPU: host decoders (footer of every format version, index blocks with and
without value delta encoding / first keys, partitions, properties) against
the files tests/sstgen.py writes, and the reference's footer error texts.
GPU: forst_sst_verify_file over whole files -- every checksum on the device
-- returns OK with the right block counts, and for injected corruption the
reference's exact Status text of the first failing block.

The layout of the files tests/sstgen.py writes is pinned to the reference's
own writer code (tests/test_sst_pinned.py, tests/golden/sst); every block
checksum is pinned through the oracle."""
import struct

import numpy as np
import pytest

import sstgen
from forst_amd import sst
from oracle import oracle as O

CASES = [  # (fv, ctype, index_type, restart_interval)
    (0, 1, 0, 1), (1, 2, 0, 1), (2, 3, 0, 1), (3, 4, 1, 1), (4, 1, 0, 4), (5, 4, 3, 1),
    (5, 1, 2, 1), (5, 3, 3, 4), (6, 1, 0, 1), (6, 4, 2, 4), (6, 2, 3, 1), (6, 0, 0, 1),
]


def make(fv, ct, it, ri, seed=3, **kw):
    w = sstgen.SstWriter(fv=fv, ctype=ct, index_type=it, base_context=0x5EED1234 + seed,
                         restart_interval=ri, seed=seed)
    return w, w.build(**kw)


def blocks_of(w, kind):
    return [(o, n) for k, o, n in w.blocks if k == kind]


@pytest.mark.parametrize("fv,ct,it,ri", CASES)
def test_host_decoders(fv, ct, it, ri):
    w, f = make(fv, ct, it, ri)
    ft = sst.decode_footer(f)
    assert ft.format_version == fv
    assert ft.checksum_type == (1 if fv == 0 else ct)
    mi = blocks_of(w, "metaindex")[0]
    assert (ft.metaindex_offset, ft.metaindex_size) == mi
    ix = blocks_of(w, "index")[0]
    if fv < 6:
        assert (ft.index_offset, ft.index_size) == ix
        assert ft.base_context_checksum == 0
    else:
        assert ft.base_context_checksum == w.bcc
        assert ft.footer_offset == w.footer_offset
        assert ft.footer_checksum_modifier == O.checksum_modifier_for_context(w.bcc, w.footer_offset)
    pr = blocks_of(w, "properties")[0]
    p = sst.properties(f[pr[0]:pr[0] + pr[1]])
    assert p.index_type == it and p.num_data_blocks == 40
    assert p.index_value_is_delta_encoded == (1 if fv >= 4 else 0)
    offs, sizes = sst.index_handles(f[ix[0]:ix[0] + ix[1]], p.index_value_is_delta_encoded,
                                    it == 3)
    want = blocks_of(w, "partition" if it == 2 else "data")
    assert list(zip(offs.tolist(), sizes.tolist())) == want
    if it == 2:
        got = []
        for o, n in want:
            po, ps = sst.index_handles(f[o:o + n], p.index_value_is_delta_encoded, False)
            got += list(zip(po.tolist(), ps.tolist()))
        assert got == blocks_of(w, "data")


def test_footer_errors():
    w, f = make(6, 1, 0, 1)
    f = bytearray(f)
    with pytest.raises(sst.SstCorruption, match="too short"):
        sst.decode_footer(bytes(20))
    bad = bytearray(f)
    bad[-12:-8] = struct.pack("<I", 9)
    with pytest.raises(sst.SstCorruption, match="Corrupt or unsupported format_version: 9"):
        sst.decode_footer(bad)
    bad = bytearray(f)
    bad[-53] = 7
    with pytest.raises(sst.SstCorruption, match="Corrupt or unsupported checksum type: 7"):
        sst.decode_footer(bad)
    bad = bytearray(f)
    bad[-52] = 0x3f
    with pytest.raises(sst.SstCorruption, match="Bad extended magic number: 0x3F007A00"):
        sst.decode_footer(bad)
    bad = bytearray(f)
    bad[-44:-40] = bytes(4)
    with pytest.raises(sst.SstCorruption, match="Invalid base context checksum"):
        sst.decode_footer(bad)
    bad = bytearray(f)
    bad[-8:] = struct.pack("<Q", 0x8242229663BF9564)  # plain table: no block checksums
    with pytest.raises(Exception, match="not a block-based table"):
        sst.decode_footer(bad)


def test_index_block_errors():
    w, f = make(5, 1, 0, 1)
    ix = blocks_of(w, "index")[0]
    blk = bytearray(f[ix[0]:ix[0] + ix[1]])
    blk[-4:] = struct.pack("<I", 10**6)  # num_restarts past the block
    with pytest.raises(sst.SstCorruption):
        sst.index_handles(bytes(blk), True)


# ---------------------------------------------------------------- GPU ----

def _expected_mismatch(w, f, off, n, fname):
    """reader_common.cc:50-60 message for the block at off"""
    ct = w.ctype
    stored = struct.unpack("<I", f[off + n + 1:off + n + 5])[0]
    mod = O.checksum_modifier_for_context(w.bcc, off)
    stored = (stored - mod) & 0xFFFFFFFF
    computed = O.compute_builtin_checksum(ct, f[off:off + n + 1])
    if ct == 1:
        stored, computed = O.unmask(stored), O.unmask(computed)
    ctx = "(context removed)" if mod else ""
    return (f"Corruption: block checksum mismatch: stored{ctx} = {stored}, computed = "
            f"{computed}, type = {ct}  in {fname} offset {off} size {n}")


@pytest.mark.gpu
@pytest.mark.parametrize("fv,ct,it,ri", CASES)
def test_verify_file_ok(fv, ct, it, ri):
    w, f = make(fv, ct, it, ri)
    r = sst.verify_file(f, file_name="000042.sst")
    assert r.status == 0, r.message
    assert r.data_blocks == 40 and r.n_failed == 0
    assert r.format_version == fv and r.index_type == it
    n_meta = 1 + (fv >= 6)  # filter (+ rocksdb.index)
    assert r.meta_blocks == n_meta
    assert r.index_partitions == (5 if it == 2 else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("fv,ct,it,ri", [(5, 1, 0, 1), (6, 4, 2, 4), (6, 1, 3, 1), (2, 3, 0, 1)])
def test_verify_file_corruption(fv, ct, it, ri):
    name = "/db/000777.sst"
    w, f = make(fv, ct, it, ri, seed=9)
    data = blocks_of(w, "data")
    # data blocks 7 and 30 corrupted: the first is reported, both counted
    b = bytearray(f)
    for i in (7, 30):
        o, n = data[i]
        b[o + n // 2] ^= 0x20
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.status == 2 and r.n_failed == 2
    o, n = data[7]
    assert r.message.decode() == _expected_mismatch(w, bytes(b), o, n, name)
    # a stored checksum byte
    b = bytearray(f)
    o, n = data[39]
    b[o + n + 2] ^= 1
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.message.decode() == _expected_mismatch(w, bytes(b), o, n, name)
    # the filter (meta) block is checked before any data block
    b = bytearray(f)
    fo, fn = blocks_of(w, "filter")[0]
    b[fo + 3] ^= 4
    o, n = data[0]
    b[o] ^= 4
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.n_failed == 2
    assert r.message.decode() == _expected_mismatch(w, bytes(b), fo, fn, name)
    # the index block is read (and verified) before its entries are trusted
    b = bytearray(f)
    io, in_ = blocks_of(w, "index")[0]
    b[io + in_ - 6] ^= 0x80
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.status == 2
    assert r.message.decode() == _expected_mismatch(w, bytes(b), io, in_, name)


@pytest.mark.gpu
def test_verify_file_footer_checksum():
    name = "x.sst"
    for ct in (0, 1, 4):
        w, f = make(6, ct, 0, 1)
        b = bytearray(f)
        b[-30] ^= 1  # reserved (unchecked) padding, covered by the footer checksum
        r = sst.verify_file(bytes(b), file_name=name)
        if ct == 0:  # kNoChecksum: computed = 0 + modifier, padding not covered
            assert r.status == 0, r.message
            b = bytearray(f)
            b[-47] ^= 1  # the stored footer checksum itself
            r = sst.verify_file(bytes(b), file_name=name)
        assert r.status == 2
        assert r.message.decode() == (f"Corruption: Footer at {w.footer_offset} checksum "
                                      f"mismatch in {name}")


@pytest.mark.gpu
def test_verify_file_large():
    """2000 data blocks, partitioned index, fv6 kXXH3"""
    w, f = make(6, 4, 2, 1, seed=5, n_data=2000, partition_size=64)
    r = sst.verify_file(f, file_name="big.sst")
    assert r.status == 0 and r.data_blocks == 2000, r.message
    assert r.index_partitions == 32


def test_decoders_survive_random_corruption():
    """Random byte flips in the structural blocks: every decoder either
    returns an error or handles, never reads outside the block (the fuzz
    loop would crash the process otherwise) and never loops forever."""
    rng = np.random.default_rng(17)
    for fv, ct, it, ri in [(5, 1, 0, 1), (6, 4, 2, 4), (6, 1, 3, 1), (2, 3, 1, 1)]:
        w, f = make(fv, ct, it, ri)
        for kind in ("index", "metaindex", "properties", "partition"):
            blks = blocks_of(w, kind)
            if not blks:
                continue
            o, n = blks[0]
            for _ in range(300):
                b = bytearray(f[o:o + n])
                for _ in range(int(rng.integers(1, 6))):
                    b[int(rng.integers(0, n))] = int(rng.integers(0, 256))
                if rng.random() < 0.2:  # truncations too
                    b = b[:int(rng.integers(0, n + 1))]
                try:
                    if kind == "properties":
                        sst.properties(bytes(b))
                    else:
                        offs, sizes = sst.index_handles(bytes(b), fv >= 4, it == 3)
                        assert len(offs) <= n  # at least one byte per entry
                except sst.SstCorruption:
                    pass
        tail = bytearray(f[-53:])
        for _ in range(300):
            t = bytearray(tail)
            t[int(rng.integers(0, 53))] ^= 1 << int(rng.integers(0, 8))
            try:
                sst.decode_footer(bytes(f[:-53]) + bytes(t))
            except Exception as e:  # corruption / unsupported, never a crash
                assert isinstance(e, sst.ForstError) or "block-based" in str(e)


@pytest.mark.gpu
def test_verify_files_batch():
    """forst_sst_verify_files (DB::VerifyChecksum over many files, one bulk
    launch per checksum type) returns, per file, exactly what
    forst_sst_verify_file returns -- clean files and corrupted ones mixed."""
    files, names = [], []
    for k, (fv, ct, it, ri) in enumerate(CASES):
        w, f = make(fv, ct, it, ri, seed=20 + k)
        b = bytearray(f)
        if k % 3 == 1:  # a data block of every third file corrupted
            o, n = blocks_of(w, "data")[5 + k]
            b[o + n // 3] ^= 0x10
        elif k % 3 == 2 and fv >= 1:  # a filter (meta) block and a data block
            fo, fn = blocks_of(w, "filter")[0]
            b[fo + 1] ^= 2
            o, n = blocks_of(w, "data")[0]
            b[o] ^= 1
        files.append(bytes(b))
        names.append(f"/db/{100 + k:06d}.sst")
    files.append(b"\0" * 10)  # too short for a footer
    names.append("/db/short.sst")
    rs = sst.verify_files(files, names)
    assert len(rs) == len(files)
    for f, name, r in zip(files, names, rs):
        one = sst.verify_file(f, file_name=name)
        assert (r.status, r.message) == (one.status, one.message), name
        assert (r.n_failed, r.blocks_verified, r.data_blocks) == \
            (one.n_failed, one.blocks_verified, one.data_blocks), name
    assert sum(r.status == 2 for r in rs) >= 8


@pytest.mark.gpu
def test_verify_files_many():
    """64 files of 300 blocks each (every type, fv 5/6) in one call: all OK."""
    files = [make(5 + (k & 1), (k % 4) + 1, (0, 2, 3)[k % 3], 1, seed=100 + k, n_data=300)[1]
             for k in range(64)]
    rs = sst.verify_files(files)
    assert all(r.status == 0 for r in rs), [r.message for r in rs if r.status]
    assert all(r.data_blocks == 300 for r in rs)


@pytest.mark.gpu
def test_ingested_global_seqno_rewrite_still_verifies():
    """IngestExternalFile(write_global_seqno=true) rewrites the 8-byte
    global_seqno property value after the properties block checksum was taken;
    the reference retries that checksum with the value zeroed
    (ReadTablePropertiesHelper, meta_blocks.cc:401-417)"""
    name = "/db/000099.sst"
    for fv, ct in ((5, 1), (6, 4)):
        w, f = make(fv, ct, 0, 1, external=True)
        po, pn = blocks_of(w, "properties")[0]
        props = sst.properties(f[po:po + pn])
        at = po + props.global_seqno_value_offset
        assert props.global_seqno_value_offset > 0
        b = bytearray(f)
        b[at:at + 8] = struct.pack("<Q", 123456789)  # the ingested file's global seqno
        r = sst.verify_file(bytes(b), file_name=name)
        assert r.status == 0, r.message
        blk = bytes(b[po:po + pn])
        cmp_at = po + blk.index(b"leveldb.BytewiseComparator") + 3
        b2 = bytearray(b)
        b2[cmp_at] ^= 0x40  # any other byte of the block still fails its checksum
        r = sst.verify_file(bytes(b2), file_name=name)
        assert r.status == 2 and b"block checksum mismatch" in r.message, r.message
        # an entry that no longer parses: the block iterator's error, which
        # carries no file name (block.h:559 CorruptionError; the properties are
        # decoded before their checksum, meta_blocks.cc:256-262)
        b3 = bytearray(b)
        b3[po + 1] = 0xFF  # first entry's non_shared varint: runs past the block
        b3[po + 2] = 0xFF
        b3[po + 3] = 0x7F
        r = sst.verify_file(bytes(b3), file_name=name)
        assert r.status == 2 and r.message == b"Corruption: bad entry in block", r.message


@pytest.mark.gpu
def test_footer_checked_reserved_bytes_after_checksum():
    """fv6: the footer checksum is compared before the 8 checked reserved
    bytes (format.cc:421-448): a flip there is a checksum mismatch; non-zero
    reserved bytes under a valid checksum are NotSupported"""
    name = "x.sst"
    w, f = make(6, 1, 0, 1)
    b = bytearray(f)
    b[-20] ^= 1
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.message.decode() == f"Corruption: Footer at {w.footer_offset} checksum mismatch in {name}"
    ft = bytearray(b[-53:])
    ft[5:9] = bytes(4)
    c = O.compute_builtin_checksum(1, bytes(ft))
    c = (c + O.checksum_modifier_for_context(w.bcc, w.footer_offset)) & 0xFFFFFFFF
    b[-48:-44] = struct.pack("<I", c)
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.status == 3
    assert r.message.decode() == ("Not implemented: File uses a future feature not supported "
                                  f"in this version in {name}")


@pytest.mark.gpu
def test_short_file_message():
    r = sst.verify_file(bytes(10), file_name="/db/000001.sst")
    assert r.message.decode() == ("Corruption: file is too short (10 bytes) to be an sstable: "
                                  "/db/000001.sst")


# ---- Snappy-compressed files (ForSt's default compression) -----------------
SNAPPY_CASES = [(5, 1, 0, 1), (6, 4, 2, 4), (2, 1, 3, 1), (4, 4, 2, 1)]


def make_snappy(fv, ct, it, ri, seed=13, **kw):
    """index blocks, index partitions and data blocks written through the real
    snappy library (type byte 1), as a column family with ForSt's default
    compression (options/options.cc:123) and enable_index_compression (the
    default, include/rocksdb/table.h:526) writes them"""
    pytest.importorskip("pyarrow")
    w = sstgen.SstWriter(fv=fv, ctype=ct, index_type=it, base_context=0x5EED1234 + seed,
                         restart_interval=ri, seed=seed, compression="snappy",
                         compressible_values=True)
    return w, w.build(**kw)


@pytest.mark.parametrize("fv,ct,it,ri", SNAPPY_CASES)
def test_snappy_file_structure_decodes_on_the_host(fv, ct, it, ri):
    """every Snappy structural block of the file decodes through the
    product's decoder (forst_block_uncompress) to what the real snappy
    library makes of it, and the decoded index lists the data blocks"""
    import ctypes

    import sstwalk
    from forst_amd._lib import lib
    w, f = make_snappy(fv, ct, it, ri)
    blocks, foot = sstwalk.walk(f)
    assert sstwalk.tiles(blocks, foot)
    types = {(k, t) for k, _, _, t in blocks}
    assert ("index", 1) in types and ("data", 1) in types
    if it == 2:
        assert ("index_partition", 1) in types
    for k, o, n, t in blocks:
        if t != 1 or k == "data":
            continue
        want = sstwalk.contents(f, (o, n), fv)
        out = np.zeros(len(want) + 16, np.uint8)
        got_n = ctypes.c_uint64()
        err = ctypes.c_char_p()
        src = np.frombuffer(f[o:o + n], np.uint8)
        rc = lib().forst_block_uncompress(1, fv, src.ctypes.data, n, out.ctypes.data, len(out),
                                          ctypes.byref(got_n), ctypes.byref(err))
        assert rc == 0, err.value
        assert out[:got_n.value].tobytes() == want
    assert [(o, n) for k, o, n, _ in blocks if k == "data"] == blocks_of(w, "data")


@pytest.mark.gpu
@pytest.mark.parametrize("fv,ct,it,ri", SNAPPY_CASES)
def test_verify_snappy_file(fv, ct, it, ri):
    """forst_sst_verify_file walks a Snappy-compressed index (and its
    partitions) on the host and verifies every block on the GPU; a corrupted
    data block is named with the reference's text; a Snappy index whose
    checksum is intact but whose stream is broken gives UncompressBlockData's
    Status (table/format.cc:654-667)"""
    name = "/flink/db/000123.sst"
    w, f = make_snappy(fv, ct, it, ri)
    r = sst.verify_file(f, file_name=name)
    assert r.status == 0, r.message
    assert r.data_blocks == 40 and r.n_failed == 0
    assert r.index_partitions == (5 if it == 2 else 0)
    data = blocks_of(w, "data")
    b = bytearray(f)
    o, n = data[17]
    b[o + n // 3] ^= 0x10
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.status == 2 and r.n_failed == 1
    assert r.message.decode() == _expected_mismatch(w, bytes(b), o, n, name)
    # the index stream's length preamble off by one, trailer re-signed
    io, in_ = blocks_of(w, "index")[0]
    assert f[io + in_] == 1
    b = bytearray(f)
    b[io] ^= 0x01
    b[io + in_:io + in_ + 5] = sstgen.PyCodec().trailer(w.ctype, bytes(b[io:io + in_]), 1,
                                                        w.bcc, io)
    r = sst.verify_file(bytes(b), file_name=name)
    assert r.status != 0
    assert r.message.decode() == "Corruption: Corrupted compressed block contents: Snappy"
