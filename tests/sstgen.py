"""tests/sstgen.py -- TEST INFRASTRUCTURE ONLY: writes SST files in the
block-based table format for the whole-file verify tests.

A restatement of the reference's WRITER side (parity unpinned at the file
level: the reference SST builder does not compile from a few source files --
FooterBuilder needs the magic-number definitions of
block_based_table_builder.cc / plain_table_builder.cc and BlockBuilder needs
db/dbformat.cc and monitoring/perf_context.cc -- so no reference-written SST
can be produced here; block checksums themselves are the oracle's, which is
pinned to the reference vectors).  Followed:
  BlockBuilder            table/block_based/block_builder.cc:46-260
  IndexValue / handles    table/format.cc:60-121
  ShortenedIndexBuilder   table/block_based/index_builder.h:184-264
  PartitionedIndexBuilder table/block_based/index_builder.cc:180-280
  MetaIndexBuilder        table/meta_blocks.cc:38-54 (sorted, restart 1)
  PropertyBlockBuilder    table/meta_blocks.cc:56-140 (sorted, restart INT_MAX)
  Finish() order          block_based_table_builder.cc:1966-2024
  FooterBuilder::Build    table/format.cc:230-351
  trailer                 block_based_table_builder.cc:1311-1360
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


class SstWriter:
    """kinds of the recorded blocks: data, filter, index, partition, properties,
    metaindex"""

    def __init__(self, fv=5, ctype=1, index_type=0, base_context=0, restart_interval=1,
                 seed=1):
        self.fv, self.ctype, self.index_type = fv, ctype, index_type
        self.bcc = base_context if fv >= 6 else 0
        self.ri = restart_interval
        self.value_delta = fv >= 4
        self.f = bytearray()
        self.blocks = []  # (kind, offset, size)
        self.rng = np.random.default_rng(seed)

    def write_block(self, contents, kind, ctype_byte=0):
        off = len(self.f)
        n = len(contents)
        c = O.compute_builtin_checksum_with_last_byte(self.ctype, contents, ctype_byte)
        c = (c + O.checksum_modifier_for_context(self.bcc, off)) & 0xFFFFFFFF
        self.f += contents + bytes([ctype_byte]) + struct.pack("<I", c)
        self.blocks.append((kind, off, n))
        return off, n

    def data_block(self, nkeys, first):
        b = BlockBuilder(16)
        keys = []
        for k in range(nkeys):
            key = b"user%010d" % (first + k) + struct.pack("<Q", (first + k) << 8 | 1)
            val = self.rng.integers(0, 256, int(self.rng.integers(10, 300)), np.uint8).tobytes()
            b.add(key, val)
            keys.append(key)
        return b.finish(), keys

    def _index_entries(self, builder, entries):
        prev = None
        for sep, (off, n), first_key in entries:
            full = handle(off, n)
            if self.index_type == 3:
                full += varint(len(first_key)) + first_key
            delta = None
            if prev is not None:
                delta = varint(zigzag(n - prev[1]))
                if self.index_type == 3:
                    delta += varint(len(first_key)) + first_key
            builder.add(sep, full, delta)
            prev = (off, n)

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
                pb = BlockBuilder(self.ri, True, self.value_delta)
                self._index_entries(pb, p)
                tops.append((p[-1][0], self.write_block(pb.finish(), "partition"), b""))
            tb = BlockBuilder(self.ri, True, self.value_delta)
            saved, self.index_type = self.index_type, 0
            self._index_entries(tb, tops)
            self.index_type = saved
            ix = self.write_block(tb.finish(), "index")
        else:
            ib = BlockBuilder(self.ri, True, self.value_delta)
            self._index_entries(ib, entries)
            ix = self.write_block(ib.finish(), "index")
        if self.fv >= 6:
            meta[b"rocksdb.index"] = ix
        # properties (sorted, restart interval INT_MAX)
        props = {
            b"rocksdb.block.based.table.index.type": struct.pack("<I", self.index_type),
            b"rocksdb.index.value.is.delta.encoded": varint(1 if self.value_delta else 0),
            b"rocksdb.index.key.is.user.key": varint(0),
            b"rocksdb.num.data.blocks": varint(n_data),
            b"rocksdb.format.version": varint(self.fv),
            b"rocksdb.data.size": varint(entries[-1][1][0] + entries[-1][1][1] + 5),
            b"rocksdb.comparator": b"leveldb.BytewiseComparator",
            b"rocksdb.column.family.name": b"",
        }
        if self.index_type == 2:
            props[b"rocksdb.index.partitions"] = varint(len(parts))
        if external:  # SstFileWriter's collector (sst_file_writer_collectors.h): version 2, seqno 0
            props[b"rocksdb.external_sst_file.version"] = struct.pack("<I", 2)
            props[b"rocksdb.external_sst_file.global_seqno"] = struct.pack("<Q", 0)
        pbld = BlockBuilder(2**31 - 1)
        for name in sorted(props):
            pbld.add(name, props[name])
        meta[b"rocksdb.properties"] = self.write_block(pbld.finish(), "properties")
        mb = BlockBuilder(1)
        for name in sorted(meta):
            mb.add(name, handle(*meta[name]))
        mi = self.write_block(mb.finish(), "metaindex")
        self.meta_names = sorted(meta)
        self.footer_offset = len(self.f)
        self.f += self.footer(mi, ix)
        return bytes(self.f)

    def footer(self, mi, ix):  # FooterBuilder::Build, format.cc:230-351
        if self.fv == 0:
            part2 = handle(*mi) + handle(*ix)
            return part2 + bytes(40 - len(part2)) + struct.pack("<Q", LEGACY_MAGIC)
        part3 = struct.pack("<IQ", self.fv, MAGIC)
        if self.fv < 6:
            part2 = handle(*mi) + handle(*ix)
            return bytes([self.ctype]) + part2 + bytes(40 - len(part2)) + part3
        body = bytearray(bytes([self.ctype]) + EXT_MAGIC + struct.pack("<III", 0, self.bcc, mi[1])
                         + bytes(24) + part3)
        c = O.compute_builtin_checksum(self.ctype, bytes(body))
        c = (c + O.checksum_modifier_for_context(self.bcc, self.footer_offset)) & 0xFFFFFFFF
        body[5:9] = struct.pack("<I", c)
        return bytes(body)

    def verify_order(self):
        """(offset, size) in the order VerifyChecksum checks them: meta blocks
        in metaindex order (properties separately), then data blocks"""
        return [b for b in self.blocks if b[0] == "data"]
