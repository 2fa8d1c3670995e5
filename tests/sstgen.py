"""tests/sstgen.py -- TEST INFRASTRUCTURE ONLY: writes SST files in the
block-based table format for the whole-file verify tests.

Layout follows the reference writer (file:line below).  Every encoding goes
through a codec: PyCodec is this file's restatement; tests/golden/
gen_sst_golden.py runs the SAME writer with a codec that calls the
reference's own BlockBuilder, BlockHandle / IndexValue encoders,
PropertyBlockBuilder, MetaIndexBuilder, FooterBuilder and
ComputeBuiltinChecksumWithLastByte + ChecksumModifierForContext (compiled
from /root/reference, tests/golden/ref_sst_shim.cc) and commits the files as
tests/golden/sst/*.sst -- tests/test_sst_pinned.py checks that PyCodec writes
them byte for byte, which pins every file this module writes.  Followed:
  BlockBuilder            table/block_based/block_builder.cc:46-260
  IndexValue / handles    table/format.cc:60-121
  ShortenedIndexBuilder   table/block_based/index_builder.h:184-264
  PartitionedIndexBuilder table/block_based/index_builder.cc:180-280
  MetaIndexBuilder        table/meta_blocks.cc:38-54 (sorted, restart 1)
  PropertyBlockBuilder    table/meta_blocks.cc:56-140 (sorted, restart INT_MAX)
  Finish() order          block_based_table_builder.cc:1966-2024
  FooterBuilder::Build    table/format.cc:230-351
  trailer                 block_based_table_builder.cc:1311-1360
The block ORDER and which properties are written are this writer's choice
(a subset of the reference's properties); the encodings are pinned.
"""
import struct

import numpy as np

from oracle import oracle as O

MAGIC = 0x88E241B785F4CFF7          # block_based_table_builder.cc:201
LEGACY_MAGIC = 0xDB4775248B80FB57   # :204
EXT_MAGIC = b"\x3e\x00\x7a\x00"     # format.cc:226


def varint(v):
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def zigzag(v):
    return ((v << 1) ^ (v >> 63)) & (2**64 - 1)


def handle(off, size):
    return varint(off) + varint(size)


class BlockBuilder:
    def __init__(self, restart_interval=16, delta_keys=True, value_delta=False):
        self.ri, self.dk, self.vd = restart_interval, delta_keys, value_delta
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""

    def add(self, key, value, delta_value=None):
        shared = 0
        if self.counter >= self.ri:
            self.restarts.append(len(self.buf))
            self.counter = 0
        elif self.dk:
            n = min(len(key), len(self.last))
            while shared < n and key[shared] == self.last[shared]:
                shared += 1
        non_shared = len(key) - shared
        if self.vd:
            self.buf += varint(shared) + varint(non_shared)
        else:
            self.buf += varint(shared) + varint(non_shared) + varint(len(value))
        self.buf += key[shared:]
        self.buf += delta_value if (shared and self.vd) else value
        self.last = key
        self.counter += 1

    def finish(self):
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))


class PyCodec:
    """the encodings, restated (tests/golden/gen_sst_golden.py has the
    reference-backed twin)"""

    def block(self, restart_interval, delta_keys, value_delta, entries):
        b = BlockBuilder(restart_interval, delta_keys, value_delta)
        for key, value, delta in entries:
            b.add(key, value, delta)
        return b.finish()

    def handle(self, off, n):
        return handle(off, n)

    def index_value(self, off, n, first_key, have_first_key, prev):
        """IndexValue::EncodeTo: full (prev None) or delta-encoded"""
        if prev is None:
            out = handle(off, n)
        else:
            out = varint(zigzag(n - prev[1]))
        if have_first_key:
            out += varint(len(first_key)) + first_key
        return out

    def properties(self, props):
        """props: (name, "u64" | "str", value); sorted, restart INT_MAX"""
        return self.block(2**31 - 1, True, False,
                          [(k, varint(v) if kind == "u64" else v, None)
                           for k, kind, v in sorted(props)])

    def metaindex(self, entries):
        """entries: (name, (offset, size)); sorted, restart 1"""
        return self.block(1, True, False, [(k, handle(*h), None) for k, h in sorted(entries)])

    def trailer(self, ctype, contents, ctype_byte, bcc, off):
        c = O.compute_builtin_checksum_with_last_byte(ctype, contents, ctype_byte)
        c = (c + O.checksum_modifier_for_context(bcc, off)) & 0xFFFFFFFF
        return bytes([ctype_byte]) + struct.pack("<I", c)

    def footer(self, fv, ctype, footer_offset, mi, ix, bcc):  # FooterBuilder::Build
        if fv == 0:
            part2 = handle(*mi) + handle(*ix)
            return part2 + bytes(40 - len(part2)) + struct.pack("<Q", LEGACY_MAGIC)
        part3 = struct.pack("<IQ", fv, MAGIC)
        if fv < 6:
            part2 = handle(*mi) + handle(*ix)
            return bytes([ctype]) + part2 + bytes(40 - len(part2)) + part3
        body = bytearray(bytes([ctype]) + EXT_MAGIC + struct.pack("<III", 0, bcc, mi[1])
                         + bytes(24) + part3)
        c = O.compute_builtin_checksum(ctype, bytes(body))
        c = (c + O.checksum_modifier_for_context(bcc, footer_offset)) & 0xFFFFFFFF
        body[5:9] = struct.pack("<I", c)
        return bytes(body)


class SstWriter:
    """kinds of the recorded blocks: data, filter, index, partition, properties,
    metaindex"""

    def __init__(self, fv=5, ctype=1, index_type=0, base_context=0, restart_interval=1,
                 seed=1, codec=None, compression=None, compressible_values=False):
        """compression: None, or "snappy" -- data blocks, index blocks and
        index partitions go through the real snappy library (pyarrow's
        bundled copy, snappy::RawCompress as Snappy_Compress calls it,
        util/compression.h:713-727) and are kept compressed when the ratio is
        good (GoodCompressionRatio, block_based_table_builder.cc:108-114,
        with the default max_compressed_bytes_per_kb = 896), with compression type byte 1 (kSnappyCompression);
        metaindex and properties stay uncompressed as the reference writes
        them (block_based_table_builder.cc:1728, :2010)"""
        self.codec = codec or PyCodec()
        self.compression = compression
        self.compressible_values = compressible_values
        self.fv, self.ctype, self.index_type = fv, ctype, index_type
        self.bcc = base_context if fv >= 6 else 0
        self.ri = restart_interval
        self.value_delta = fv >= 4
        self.f = bytearray()
        self.blocks = []  # (kind, offset, size)
        self.rng = np.random.default_rng(seed)

    def _maybe_compress(self, contents):
        if self.compression is None:
            return contents, 0
        assert self.compression == "snappy", self.compression
        import pyarrow as pa
        c = pa.Codec("snappy").compress(contents, asbytes=True)
        if len(c) <= (896 * len(contents)) >> 10:
            return c, 1
        return contents, 0

    def write_block(self, contents, kind, ctype_byte=0):
        if kind in ("data", "index", "partition") and self.compression and ctype_byte == 0:
            contents, ctype_byte = self._maybe_compress(contents)
        off = len(self.f)
        n = len(contents)
        self.f += contents + self.codec.trailer(self.ctype, contents, ctype_byte, self.bcc, off)
        self.blocks.append((kind, off, n))
        return off, n

    def data_block(self, nkeys, first):
        ents = []
        keys = []
        for k in range(nkeys):
            key = b"user%010d" % (first + k) + struct.pack("<Q", (first + k) << 8 | 1)
            val = self.rng.integers(0, 256, int(self.rng.integers(10, 300)), np.uint8).tobytes()
            if self.compressible_values:  # Flink-state-like values: repetitive
                val = (b"flink-state:%06d;" % (first + k)) * (1 + len(val) // 18)
            ents.append((key, val, None))
            keys.append(key)
        return self.codec.block(16, True, False, ents), keys

    def _index_block(self, entries, first_keys):
        """an index block (ShortenedIndexBuilder / a partition): separator ->
        IndexValue, delta-encoded after the first entry when the format
        version has value delta encoding"""
        ents = []
        prev = None
        for sep, (off, n), first_key in entries:
            full = self.codec.index_value(off, n, first_key, first_keys, None)
            delta = (self.codec.index_value(off, n, first_key, first_keys, prev)
                     if prev is not None else None)
            ents.append((sep, full, delta))
            prev = (off, n)
        return self.codec.block(self.ri, True, self.value_delta, ents)

    def build(self, n_data=40, filter_block=True, partition_size=8, compress_type_bytes=None,
              external=False):
        entries = []
        k = 0
        for i in range(n_data):
            nk = int(self.rng.integers(1, 40))
            contents, keys = self.data_block(nk, k)
            k += nk
            ct = 0 if compress_type_bytes is None else int(compress_type_bytes[i])
            h = self.write_block(contents, "data", ct)
            entries.append((keys[-1], h, keys[0]))
        meta = {}
        if filter_block:  # contents opaque to the checksum walk
            fb = self.rng.integers(0, 256, 777, np.uint8).tobytes()
            meta[b"fullfilter.rocksdb.BuiltinBloomFilter"] = self.write_block(fb, "filter")
        # index (block_based_table_builder.cc:1576-1644)
        if self.index_type == 2:
            parts = [entries[i:i + partition_size] for i in range(0, len(entries), partition_size)]
            tops = []
            for p in parts:
                tops.append((p[-1][0], self.write_block(self._index_block(p, False), "partition"),
                             b""))
            ix = self.write_block(self._index_block(tops, False), "index")
        else:
            ix = self.write_block(self._index_block(entries, self.index_type == 3), "index")
        if self.fv >= 6:
            meta[b"rocksdb.index"] = ix
        # properties (sorted, restart interval INT_MAX)
        props = [
            # (BlockBasedTablePropertiesCollector, block_based_table_builder.cc:226-262)
            (b"rocksdb.block.based.table.index.type", "str", struct.pack("<I", self.index_type)),
            (b"rocksdb.index.value.is.delta.encoded", "u64", 1 if self.value_delta else 0),
            (b"rocksdb.index.key.is.user.key", "u64", 0),
            (b"rocksdb.num.data.blocks", "u64", n_data),
            (b"rocksdb.format.version", "u64", self.fv),
            (b"rocksdb.data.size", "u64", entries[-1][1][0] + entries[-1][1][1] + 5),
            (b"rocksdb.comparator", "str", b"leveldb.BytewiseComparator"),
            (b"rocksdb.column.family.name", "str", b""),
        ]
        if self.index_type == 2:
            props.append((b"rocksdb.index.partitions", "u64", len(parts)))
        if external:  # SstFileWriter's collector (sst_file_writer_collectors.h): version 2, seqno 0
            props.append((b"rocksdb.external_sst_file.version", "str", struct.pack("<I", 2)))
            props.append((b"rocksdb.external_sst_file.global_seqno", "str", struct.pack("<Q", 0)))
        meta[b"rocksdb.properties"] = self.write_block(self.codec.properties(props), "properties")
        mi = self.write_block(self.codec.metaindex(list(meta.items())), "metaindex")
        self.meta_names = sorted(meta)
        self.footer_offset = len(self.f)
        self.f += self.codec.footer(self.fv, self.ctype, self.footer_offset, mi, ix, self.bcc)
        return bytes(self.f)

    def verify_order(self):
        """(offset, size) in the order VerifyChecksum checks them: meta blocks
        in metaindex order (properties separately), then data blocks"""
        return [b for b in self.blocks if b[0] == "data"]
