"""tests/sstwalk.py -- TEST INFRASTRUCTURE: a small reader of block-based SST
files that lists every block the way the reference's structures name them.

Used to locate blocks in SST files written by the reference's own
SstFileWriter (tests/golden/gen_sst_golden.py) -- to corrupt a chosen block,
and to feed GpuTrailerWriter the file's blocks in order for a byte-for-byte
rewrite.  Follows:
  footer      table/format.cc:334-463 (Footer::DecodeFrom)
  blocks      table/block_based/block.cc (entries, restarts), block_builder.cc
  index value table/format.cc:105-148 (IndexValue, delta-encoded sizes)
  metaindex   table/meta_blocks.cc (name -> BlockHandle)
  compression util/compression.h: compress_format_version 2 (fv >= 2) puts a
              varint32 uncompressed size in front; zlib is raw deflate
              (windowBits -14), as Zlib_Compress writes it; Snappy keeps its
              own length prefix in both versions (compression.h:711) and is
              decoded by the real snappy library bundled with pyarrow
"""
import struct
import zlib

MAGIC = 0x88e241b785f4cff7
LEGACY_MAGIC = 0xdb4775248b80fb57
TRAILER = 5


def varint(b, p):
    r = s = 0
    while True:
        x = b[p]
        p += 1
        r |= (x & 127) << s
        if not x & 128:
            return r, p
        s += 7


def footer(data):
    size = len(data)
    magic = struct.unpack_from("<Q", data, size - 8)[0]
    if magic == LEGACY_MAGIC:
        p = size - 48
        mo, p = varint(data, p)
        ms, p = varint(data, p)
        io, p = varint(data, p)
        is_, p = varint(data, p)
        return {"fv": 0, "checksum": 1, "footer_offset": size - 48, "metaindex": (mo, ms),
                "index": (io, is_), "bcc": 0}
    assert magic == MAGIC, hex(magic)
    fv = struct.unpack_from("<I", data, size - 12)[0]
    fo = size - 53
    ct = data[fo]
    if fv >= 6:
        bcc = struct.unpack_from("<I", data, fo + 9)[0]
        ms = struct.unpack_from("<I", data, fo + 13)[0]
        return {"fv": fv, "checksum": ct, "footer_offset": fo,
                "metaindex": (fo - TRAILER - ms, ms), "index": None, "bcc": bcc}
    p = fo + 1
    mo, p = varint(data, p)
    ms, p = varint(data, p)
    io, p = varint(data, p)
    is_, p = varint(data, p)
    return {"fv": fv, "checksum": ct, "footer_offset": fo, "metaindex": (mo, ms),
            "index": (io, is_), "bcc": 0}


def contents(data, h, fv):
    """the block's uncompressed contents (what BlockFetcher hands the reader)"""
    off, n = h
    raw = bytes(data[off:off + n])
    t = data[off + n]
    if t == 0:
        return raw
    if t == 1:
        import pyarrow as pa
        n_out, _ = varint(raw, 0)
        return pa.Codec("snappy").decompress(raw, decompressed_size=n_out, asbytes=True)
    assert t == 2, f"codec {t} (zlib or snappy in the fixtures)"
    p = 0
    if fv >= 2:
        _, p = varint(raw, 0)
    return zlib.decompress(raw[p:], -14)


def entries(blk, value_delta=False, value_fn=None):
    nr = struct.unpack_from("<I", blk, len(blk) - 4)[0] & 0x7FFFFFFF
    lim = len(blk) - 4 * (nr + 1)
    p, key = 0, b""
    while p < lim:
        shared, p = varint(blk, p)
        non_shared, p = varint(blk, p)
        vlen = None
        if not value_delta:
            vlen, p = varint(blk, p)
        key = key[:shared] + blk[p:p + non_shared]
        p += non_shared
        if value_delta:
            used = value_fn(key, shared != 0, blk, p)
            p += used
        else:
            yield key, blk[p:p + vlen]
            p += vlen
            continue
        yield key, None


def index_handles(blk, value_delta, first_key):
    out = []

    def fn(key, shared, b, p):
        q = p
        if shared:
            z, q = varint(b, q)
            delta = (z >> 1) ^ -(z & 1)
            po, ps = out[-1]
            out.append((po + ps + TRAILER, ps + delta))
        else:
            o, q = varint(b, q)
            n, q = varint(b, q)
            out.append((o, n))
        if first_key:
            kl, q = varint(b, q)
            q += kl
        return q - p

    if value_delta:
        for _ in entries(blk, True, fn):
            pass
        return out
    for _, v in entries(blk):
        q = 0
        o, q = varint(v, q)
        n, q = varint(v, q)
        out.append((o, n))
    return out


def properties(blk):
    out = {}
    for k, v in entries(blk):
        out[k.decode(errors="replace")] = v
    return out


def walk(data):
    """every block of the file: [(kind, offset, size, compression type byte)]
    plus the footer dict.  kinds: metaindex, properties, index, index_partition,
    filter, filter_index, filter_partition, rangedel, dict, data"""
    f = footer(data)
    fv = f["fv"]
    blocks = [("metaindex",) + f["metaindex"]]
    meta = {k.decode(): varint_handle(v) for k, v in entries(contents(data, f["metaindex"], fv))}
    props = properties(contents(data, meta["rocksdb.properties"], fv))
    u = lambda k: varint(props[k], 0)[0] if k in props else 0  # noqa: E731
    index_type = struct.unpack("<I", props["rocksdb.block.based.table.index.type"])[0]
    delta = u("rocksdb.index.value.is.delta.encoded") != 0
    ix = f["index"] or meta["rocksdb.index"]
    for name, h in meta.items():
        kind = ("properties" if name == "rocksdb.properties" else
                "index" if name == "rocksdb.index" else
                "rangedel" if name == "rocksdb.range_del" else
                "dict" if name == "rocksdb.compression_dict" else
                "filter_index" if name.startswith("partitionedfilter.") else
                "filter" if name.startswith("fullfilter.") else name)
        blocks.append((kind,) + h)
        if kind == "filter_index":  # PartitionedFilterBlockBuilder's index
            for p in index_handles(contents(data, h, fv), fv >= 4, False):
                blocks.append(("filter_partition",) + p)
    if f["index"]:
        blocks.append(("index",) + ix)
    top = index_handles(contents(data, ix, fv), delta, index_type == 3)
    if index_type == 2:
        data_h = []
        for p in top:
            blocks.append(("index_partition",) + p)
            data_h += index_handles(contents(data, p, fv), delta, index_type == 3)
    else:
        data_h = top
    blocks += [("data",) + h for h in data_h]
    out = sorted({(o, n, k) for k, o, n in blocks})
    return [(k, o, n, data[o + n]) for o, n, k in out], f


def varint_handle(v):
    o, p = varint(v, 0)
    n, _ = varint(v, p)
    return (o, n)


def tiles(blocks, f):
    """the blocks (+ trailers) cover [0, footer_offset) exactly"""
    pos = 0
    for _, o, n, _ in blocks:
        if o != pos:
            return False
        pos = o + n + TRAILER
    return pos == f["footer_offset"]
