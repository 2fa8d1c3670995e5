#!/usr/bin/env python3
"""tests/golden/gen_kv_golden.py -- TEST INFRASTRUCTURE ONLY: per-KV protection
fixtures (a15) at the reference's own call sites, from the REFERENCE's code.

The veneer tests/golden/ref_kv_shim.cc is linked against the reference archive
of tests/golden/refbuild.py (g++ over src.mk's LIB_SOURCES where they lie, in a
throwaway directory outside the repository; `-z defs` proves nothing is stood
in for) and driven through ctypes:

  memtable   MemTable::Add with memtable_protection_bytes_per_key 1/2/4/8
             (db/memtable.cc:696-732), entries read back through the
             memtable's iterator; MemTable::VerifyEntryChecksum
             (memtable.cc:273-307) on every intact entry, on single-byte
             corruptions of key / tag / value / checksum bytes, and on crafted
             headers (5-byte varint32, internal key shorter than 8, bad value
             length varint) -- its Status text recorded per case.
  writebatch WriteBatch reps of every record kind ReadRecordFromWriteBatch
             parses (write_batch.cc:361-475), default and other column
             families, iterated by the reference's WriteBatch::Iterate with a
             handler doing ProtectionInfoUpdater's ProtectKVO(...).ProtectC(cf)
             (write_batch.cc:3016-3080); truncated reps, wrong counts and
             every tag byte 0-255 in front of a record, with the Status text.
  blocks     data / index / metaindex blocks of the committed reference-written
             SSTs (tests/golden/sst/builder_*.sst), their kv_checksum_ from
             Block::Initialize{Data,Index,MetaIndex}BlockProtectionInfo
             (table/block_based/block.cc:1113-1235, TEST_GetKVChecksum).

Committed: tests/golden/kv_sites.npz (arrays only: numpy.load with
allow_pickle=False) + kv_sites.json (case lists, Status texts).

Re-run:  python tests/golden/gen_kv_golden.py   (needs /root/reference + g++)
"""
import ctypes
import json
import os
import struct
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, TESTS)
import refbuild  # noqa: E402

OUT_NPZ = os.path.join(HERE, "kv_sites.npz")
OUT_JSON = os.path.join(HERE, "kv_sites.json")
ull, sz, vp, c_int = ctypes.c_ulonglong, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int


def load(path):
    L = ctypes.CDLL(path)
    L.ref_memtable_build.argtypes = [c_int, c_int, ull, vp, sz, vp, ctypes.POINTER(sz)]
    L.ref_memtable_build.restype = c_int
    L.ref_memtable_verify.argtypes = [vp, c_int, c_int, ctypes.c_char_p, sz]
    L.ref_memtable_verify.restype = c_int
    L.ref_write_batch_build.argtypes = [c_int, ull, vp, sz, ctypes.POINTER(sz)]
    L.ref_write_batch_build.restype = c_int
    L.ref_write_batch_protect.argtypes = [vp, sz, vp, sz, ctypes.POINTER(sz), ctypes.c_char_p, sz]
    L.ref_write_batch_protect.restype = c_int
    L.ref_block_kv_checksum.argtypes = [vp, sz, c_int, c_int, c_int, c_int, vp, sz]
    L.ref_block_kv_checksum.restype = ctypes.c_long
    return L


def ptr(a):
    return a.ctypes.data


def mem_verify(L, buf, off, pb):
    """VerifyEntryChecksum on buf[off:] (buf padded: the reference reads up to
    5 bytes past a varint's start regardless)"""
    msg = ctypes.create_string_buffer(4096)
    ok = L.ref_memtable_verify(ptr(buf) + off, pb, 0, msg, 4096)
    return msg.value.decode()


def varint(b, p):
    r = s = 0
    while True:
        x = int(b[p])
        p += 1
        r |= (x & 127) << s
        if not x & 128:
            return r, p
        s += 7


def gen_memtable(L, arrays, meta):
    cases = []
    for pb, n, seed in ((8, 150, 0xA15001), (1, 60, 0xA15002), (2, 60, 0xA15003),
                        (4, 60, 0xA15004)):
        cap = 1 << 23
        raw = np.zeros(cap, np.uint8)
        offs = np.zeros(n, np.uint64)
        nb = sz()
        k = L.ref_memtable_build(pb, n, seed, ptr(raw), cap, ptr(offs), ctypes.byref(nb))
        assert k == n, k
        base = raw[:nb.value + 64].copy()  # + readable padding
        tag = f"mem{pb}"
        status = [mem_verify(L, base, int(o), pb) for o in offs]
        assert all(s == "OK" for s in status), status[:3]
        # corruptions: one byte of key / tag / value / checksum of chosen entries
        corrupt = []
        rng = np.random.default_rng(seed)
        for j in range(0, n, 3):
            o = int(offs[j])
            ikl, kp = varint(base, o)
            vl, vp_ = varint(base, kp + ikl)
            region = [("key", kp, ikl - 8), ("tag", kp + ikl - 8, 8), ("value", vp_, vl),
                      ("checksum", vp_ + vl, pb)][j % 4]
            if region[2] == 0:
                region = ("tag", kp + ikl - 8, 8)
            at = region[1] + int(rng.integers(0, region[2]))
            bit = 1 << int(rng.integers(0, 8))
            b2 = base.copy()
            b2[at] ^= bit
            corrupt.append({"entry": j, "region": region[0], "at": at, "xor": bit,
                            "status": mem_verify(L, b2, o, pb)})
        arrays[tag + "_base"] = base
        arrays[tag + "_offs"] = offs
        cases.append({"tag": tag, "prot_bytes": pb, "n": n, "corrupt": corrupt})
    # crafted headers (pb 8): each a small buffer of its own
    crafted = []
    pads = bytes(32)
    for name, head in (("klen_5_continuation", b"\x80\x80\x80\x80\x80\x01"),
                       ("klen_below_8", b"\x07" + b"k" * 7 + b"\x00" * 8),
                       ("klen_0", b"\x00\x00" + b"v" * 9),
                       ("vlen_5_continuation", b"\x0b" + b"abc" + struct.pack("<Q", (9 << 8) | 1)
                        + b"\xff\xff\xff\xff\xff\x00"),
                       ("vlen_multibyte_ok", b"\x0b" + b"abc" + struct.pack("<Q", (9 << 8) | 1)
                        + b"\x81\x01" + b"w" * 129 + b"\x00" * 8),
                       ("klen_5_bytes_ok", b"\x8b\x80\x80\x80\x00" + b"abc" +
                        struct.pack("<Q", (5 << 8) | 2) + b"\x02xy" + b"\x00" * 8)):
        buf = np.frombuffer(head + pads, np.uint8).copy()
        crafted.append({"name": name, "hex": (head + pads).hex(), "len": len(head),
                        "status": mem_verify(L, buf, 0, 8)})
    meta["memtable"] = {"cases": cases, "crafted": crafted}


def wb_protect(L, rep):
    buf = np.frombuffer(rep + bytes(16), np.uint8).copy()
    out = np.zeros(4096, np.uint64)
    n = sz()
    msg = ctypes.create_string_buffer(4096)
    ok = L.ref_write_batch_protect(ptr(buf), len(rep), ptr(out), 4096, ctypes.byref(n), msg, 4096)
    return msg.value.decode(), out[:n.value].copy()


def gen_writebatch(L, arrays, meta):
    reps, batches = [], []

    def add(name, rep):
        st, prot = wb_protect(L, rep)
        batches.append({"name": name, "status": st, "n_prot": len(prot), "len": len(rep)})
        reps.append(rep)
        arrays[f"wb_prot_{len(batches) - 1}"] = prot

    cap = 1 << 22
    raw = np.zeros(cap, np.uint8)
    n = sz()
    for i, nrec in enumerate((0, 1, 2, 5, 9, 17, 40, 40, 120)):
        cnt = L.ref_write_batch_build(nrec, 0xB0001 + i, ptr(raw), cap, ctypes.byref(n))
        assert cnt >= 0
        rep = raw[:n.value].tobytes()
        add(f"random_{nrec}_{i}", rep)
        if nrec >= 2:
            add(f"truncated_{i}", rep[:len(rep) - 3])
            add(f"wrong_count_{i}", rep[:8] + struct.pack("<I", cnt + 1) + rep[12:])
            add(f"short_header_{i}", rep[:11])
    # every tag byte in front of one well-formed-looking record
    body = b"\x03abc\x04wxyz"
    for t in range(256):
        add(f"tag_{t:02x}", struct.pack("<QI", 77, 1) + bytes([t]) + b"\x05" + body)
    meta["writebatch"] = batches
    blob = b"".join(reps)
    offs = np.cumsum([0] + [len(r) for r in reps[:-1]]).astype(np.uint64)
    arrays["wb_base"] = np.frombuffer(blob + bytes(64), np.uint8).copy()
    arrays["wb_offs"] = offs
    arrays["wb_lens"] = np.array([len(r) for r in reps], np.uint32)


def gen_blocks(L, arrays, meta):
    """the blocks of the committed reference-written SSTs, uncompressed (the
    contents the reader builds Block from), with the kind / value flags the
    table reader gives them, plus crafted damaged blocks; Block::Initialize*
    ProtectionInfo's kv_checksum_ for protection bytes 8 and 2"""
    import sstwalk

    man = json.load(open(os.path.join(HERE, "sst", "builder_manifest.json")))
    blobs, cases = [], []
    for f in man["files"]:
        data = open(os.path.join(HERE, "sst", f["file"]), "rb").read()
        blocks, foot = sstwalk.walk(data)
        fv, ix = f["format_version"], f["index_type"]
        taken = {}
        for kind, o, n, _t in blocks:
            if kind in ("filter", "filter_partition", "dict"):
                continue  # not in block format
            if taken.get(kind, 0) >= 6:
                continue
            taken[kind] = taken.get(kind, 0) + 1
            try:
                blk = sstwalk.contents(data, (o, n), fv)
            except Exception:  # zlib with a compression dictionary: not decodable here
                continue
            if kind in ("data", "rangedel"):
                k = 0
            elif kind == "properties":
                continue  # never protected: MetaBlockIter assumes restart interval 1 (block.h:826-829)
            elif kind == "metaindex":
                k = 2
            else:  # index, index_partition, filter_index (index-block format)
                full = fv < 4
                first = ix == 3 and kind != "filter_index"
                k = 1 | (4 if full else 0) | (8 if first else 0)
            cases.append({"src": f["file"], "kind_name": kind, "kind": k, "bytes": blk})
    # damaged blocks: too small, restart count that wraps the offset, a first
    # entry sharing bytes with no previous key, an entry running past the block,
    # and a data block whose last value runs into the restart array
    good = next(c for c in cases if c["kind"] == 0)["bytes"]
    nr = struct.unpack_from("<I", good, len(good) - 4)[0]
    cases.append({"src": "crafted", "kind_name": "tiny", "kind": 0, "bytes": b"\x00" * 5})
    cases.append({"src": "crafted", "kind_name": "restarts_wrap", "kind": 0,
                  "bytes": good[:-4] + struct.pack("<I", 0x00ffffff)})
    cases.append({"src": "crafted", "kind_name": "first_shared", "kind": 0,
                  "bytes": b"\x05" + good[1:]})
    cases.append({"src": "crafted", "kind_name": "meta_slice_past_limit", "kind": 2,
                  "bytes": b"\x00\x04\x7f" + b"abcd" + b"\x00" * 4 + struct.pack("<II", 0, 1)})
    cases.append({"src": "crafted", "kind_name": "data_value_into_restarts", "kind": 0,
                  "bytes": b"\x00\x04\x05" + b"abcd" + b"xy" + struct.pack("<II", 0, 1)})
    cases.append({"src": "crafted", "kind_name": "empty_restarts", "kind": 0,
                  "bytes": struct.pack("<II", 0, 0)})
    for c in cases:
        blk = c.pop("bytes")
        buf = np.frombuffer(blk + bytes(64), np.uint8).copy()
        c["size"] = len(blk)
        if os.environ.get("GEN_DEBUG"):
            print(c["src"], c["kind_name"], c["kind"], len(blk), flush=True)
        for pb in (8, 2):
            out = np.zeros(1 << 20, np.uint8)
            nk = L.ref_block_kv_checksum(ptr(buf), len(blk), c["kind"] & 3, pb,
                                         1 if c["kind"] & 4 else 0, 1 if c["kind"] & 8 else 0,
                                         ptr(out), out.nbytes)
            c[f"keys_{pb}"] = int(nk)
            c[f"kv_checksum_{pb}"] = out[:max(0, nk) * pb].tobytes().hex()
        blobs.append(blk)
    offs, pos, parts = [], 0, []
    for b in blobs:
        pos += (-pos) % 4 + 3  # unaligned block starts
        parts.append(pos)
        pos += len(b)
    base = np.zeros(pos + 64, np.uint8)
    for o, b in zip(parts, blobs):
        base[o:o + len(b)] = np.frombuffer(b, np.uint8)
    arrays["blk_base"] = base
    arrays["blk_offs"] = np.array(parts, np.uint64)
    meta["blocks"] = cases


def main():
    with tempfile.TemporaryDirectory() as td:
        so = refbuild.link_veneer([os.path.join(HERE, "ref_kv_shim.cc")],
                                  os.path.join(td, "libref_kv.so"))
        L = load(so)
        arrays, meta = {}, {"generator": "tests/golden/gen_kv_golden.py"}
        gen_memtable(L, arrays, meta)
        gen_writebatch(L, arrays, meta)
        gen_blocks(L, arrays, meta)
        np.savez_compressed(OUT_NPZ, **arrays)
        with open(OUT_JSON, "w") as f:
            json.dump(meta, f, indent=1)
    print(OUT_NPZ, os.path.getsize(OUT_NPZ), OUT_JSON)


if __name__ == "__main__":
    main()
