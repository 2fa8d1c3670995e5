"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU restatement in oracle/oracle.c.  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the
product package (forst_amd/), which has no CPU fallback.
"""
import ctypes
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

kNoChecksum, kCRC32c, kxxHash, kxxHash64, kXXH3 = 0, 1, 2, 3, 4

_u8p = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32, u64, sz, vp, i = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t,
                               ctypes.c_void_p, ctypes.c_int)
        sigs = {
            "oracle_crc32c_extend": (u32, [u32, vp, sz]),
            "oracle_crc32c_extend_fast": (u32, [u32, vp, sz]),
            "oracle_crc32c_value": (u32, [vp, sz]),
            "oracle_crc32c_combine": (u32, [u32, u32, sz]),
            "oracle_crc32c_mask": (u32, [u32]),
            "oracle_crc32c_unmask": (u32, [u32]),
            "oracle_crc32c_shift": (u32, [u32, u64]),
            "oracle_xxh3_64": (u64, [vp, sz]),
            "oracle_xxh32": (u32, [vp, sz, u32]),
            "oracle_xxh64": (u64, [vp, sz, u64]),
            "oracle_compute_builtin_checksum": (u32, [i, vp, sz]),
            "oracle_compute_builtin_checksum_with_last_byte": (u32, [i, vp, sz, ctypes.c_uint8]),
            "oracle_checksum_modifier_for_context": (u32, [u32, u64]),
            "oracle_verify_block_checksum": (i, [i, vp, sz, u32, vp, vp]),
            "oracle_block_checksum_batch": (None, [i, vp, vp, vp, vp, vp, vp, sz, i]),
            "oracle_block_verify_batch": (u64, [i, vp, vp, vp, vp, vp, vp, sz, i]),
            "oracle_crc32c_batch": (None, [vp, vp, vp, vp, sz, i]),
            "oracle_xxh3_batch": (None, [vp, vp, vp, vp, sz, i]),
            "oracle_wal_record_crc": (u32, [i, u32, vp, sz]),
            "oracle_wal_record_xxh3_batch": (None, [vp, vp, vp, u64, u32, vp, vp, sz, i]),
            "oracle_wal_framed_size": (u64, [vp, sz, i]),
            "oracle_wal_frame": (u64, [vp, vp, sz, i, u32, vp, vp, vp, vp]),
            "oracle_wal_verify": (u64, [vp, u64, vp, u64, vp, i]),
            "oracle_wal_verify_blocks": (None, [vp, u64, u32, vp, vp, vp, i]),
            "oracle_hash64": (u64, [vp, sz, u64]),
            "oracle_kv_protect": (u64, [vp, sz, vp, sz, i, i, u64, i, u32]),
            "oracle_kv_verify": (i, [u64, u32, vp]),
            "oracle_hash64_batch": (None, [vp, vp, vp, vp, u64, vp, sz]),
            "oracle_kv_protect_batch": (None, [vp, vp, vp, vp, vp, vp, vp, vp, vp, sz]),
            "oracle_memtable_verify_batch": (None, [vp, sz, vp, sz, u32, vp, vp]),
            "oracle_splitmix64": (u64, [u64]),
            "oracle_fill_stream": (None, [vp, u64, u64, u64]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(a)), ctypes.c_void_p).value
    return a.ctypes.data


def _buf(data):
    """Return (pointer, length, keepalive) for bytes / numpy uint8 data."""
    if isinstance(data, np.ndarray):
        return data.ctypes.data, data.nbytes, data
    b = ctypes.create_string_buffer(bytes(data), len(data) or 1)
    return ctypes.addressof(b), len(data), b


def crc32c_value(data):
    p, n, _k = _buf(data)
    return lib().oracle_crc32c_value(p, n)


def crc32c_extend(crc, data, fast=False):
    p, n, _k = _buf(data)
    f = lib().oracle_crc32c_extend_fast if fast else lib().oracle_crc32c_extend
    return f(crc, p, n)


def crc32c_combine(a, b, blen):
    return lib().oracle_crc32c_combine(a, b, blen)


def crc32c_shift(state, nbytes):
    return lib().oracle_crc32c_shift(state, nbytes)


def mask(c):
    return lib().oracle_crc32c_mask(c)


def unmask(c):
    return lib().oracle_crc32c_unmask(c)


def xxh3_64(data):
    p, n, _k = _buf(data)
    return lib().oracle_xxh3_64(p, n)


def xxh32(data, seed=0):
    p, n, _k = _buf(data)
    return lib().oracle_xxh32(p, n, seed)


def xxh64(data, seed=0):
    p, n, _k = _buf(data)
    return lib().oracle_xxh64(p, n, seed)


def compute_builtin_checksum(ctype, data):
    p, n, _k = _buf(data)
    return lib().oracle_compute_builtin_checksum(ctype, p, n)


def compute_builtin_checksum_with_last_byte(ctype, data, last):
    p, n, _k = _buf(data)
    return lib().oracle_compute_builtin_checksum_with_last_byte(ctype, p, n, last & 0xFF)


def checksum_modifier_for_context(base, offset):
    return lib().oracle_checksum_modifier_for_context(base, offset)


def verify_block_checksum(ctype, data, block_size, modifier=0):
    p, _n, _k = _buf(data)
    c = ctypes.c_uint32()
    s = ctypes.c_uint32()
    ok = lib().oracle_verify_block_checksum(ctype, p, block_size, modifier,
                                            ctypes.byref(c), ctypes.byref(s))
    return bool(ok), c.value, s.value


def block_checksum_batch(ctype, base, offsets, sizes, last_bytes=None, modifiers=None,
                         nthreads=1):
    out = np.zeros(len(offsets), dtype=np.uint32)
    lib().oracle_block_checksum_batch(ctype, _ptr(base), _ptr(offsets), _ptr(sizes),
                                      _ptr(last_bytes), _ptr(modifiers), _ptr(out),
                                      len(offsets), nthreads)
    return out


def block_verify_batch(ctype, base, offsets, sizes, modifiers=None, nthreads=1):
    computed = np.zeros(len(offsets), dtype=np.uint32)
    ok = np.zeros(len(offsets), dtype=np.uint8)
    bad = lib().oracle_block_verify_batch(ctype, _ptr(base), _ptr(offsets), _ptr(sizes),
                                          _ptr(modifiers), _ptr(computed), _ptr(ok),
                                          len(offsets), nthreads)
    return computed, ok, bad


def crc32c_batch(base, offsets, lengths, nthreads=1):
    out = np.zeros(len(offsets), dtype=np.uint32)
    lib().oracle_crc32c_batch(_ptr(base), _ptr(offsets), _ptr(lengths), _ptr(out),
                              len(offsets), nthreads)
    return out


def xxh3_batch(base, offsets, lengths, nthreads=1):
    out = np.zeros(len(offsets), dtype=np.uint64)
    lib().oracle_xxh3_batch(_ptr(base), _ptr(offsets), _ptr(lengths), _ptr(out),
                            len(offsets), nthreads)
    return out


def wal_record_xxh3_batch(log, phys_offsets, phys_lengths, first, hs=7, nthreads=1):
    """XXH3 of every logical record: record j = payloads of physical records
    [first[j], first[j+1]) (db/log_reader.cc:95-165)"""
    po = np.ascontiguousarray(phys_offsets, np.uint64)
    pl = np.ascontiguousarray(phys_lengths, np.uint32)
    fi = np.ascontiguousarray(first, np.uint64)
    out = np.zeros(len(fi), dtype=np.uint64)
    lib().oracle_wal_record_xxh3_batch(_ptr(log), _ptr(po), _ptr(pl), len(po), hs, _ptr(fi),
                                       _ptr(out), len(fi), nthreads)
    return out


def host_threads():
    """CPU threads this process may use: the cgroup cpu.max quota where one is
    set (the GPU box: 16), else the affinity mask"""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def wal_record_crc(rtype, log_number, payload):
    p, n, _k = _buf(payload)
    return lib().oracle_wal_record_crc(rtype, log_number, p, n)


def wal_frame(payloads, lengths, recyclable=False, log_number=0):
    """Frame logical records like log::Writer::AddRecord.  Returns
    (buffer, phys_offsets, phys_lengths)."""
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    payloads = np.ascontiguousarray(payloads, dtype=np.uint8)
    total = lib().oracle_wal_framed_size(_ptr(lengths), len(lengths), int(recyclable))
    dst = np.zeros(total, dtype=np.uint8)
    # upper bound on physical records: one per 32 KiB block + one per record
    cap = len(lengths) + total // 32768 + 2
    offs = np.zeros(cap, dtype=np.uint64)
    lens = np.zeros(cap, dtype=np.uint32)
    nphys = ctypes.c_uint64()
    lib().oracle_wal_frame(_ptr(payloads), _ptr(lengths), len(lengths), int(recyclable),
                           log_number, _ptr(dst), _ptr(offs), _ptr(lens),
                           ctypes.byref(nphys))
    n = nphys.value
    return dst, offs[:n].copy(), lens[:n].copy()


def wal_verify(buf, nthreads=1):
    bad = ctypes.c_uint64()
    n = lib().oracle_wal_verify(_ptr(buf), buf.nbytes, None, 0, ctypes.byref(bad), nthreads)
    return n, bad.value


def wal_verify_blocks(buf, log_number=0, nthreads=1):
    """per 32 KiB log block: (status, records verified before the first
    failure, offset of the failing header / end of parsing), as
    forst_wal_verify_batch reports them (db/log_reader.cc:450-531)"""
    nb = (buf.nbytes + 32767) // 32768
    st = np.zeros(nb, np.uint8)
    nr = np.zeros(nb, np.uint32)
    fo = np.zeros(nb, np.uint32)
    lib().oracle_wal_verify_blocks(_ptr(buf), buf.nbytes, log_number, _ptr(st), _ptr(nr), _ptr(fo),
                                   nthreads)
    return st, nr, fo


KV_SEED_K, KV_SEED_V = 0, 0xD28AAD72F49BD50B  # db/kv_checksum.h:84-88
KV_SEED_O, KV_SEED_S, KV_SEED_C = 0xA5155AE5E937AA16, 0x77A00858DDD37F21, 0x4A2AB5CBD26F542C


def hash64(data, seed=0):
    """util/hash.cc:81 Hash64 = XXPH3_64bits_withSeed (util/xxph3.h:1733)"""
    p, n, _k = _buf(data)
    return lib().oracle_hash64(p, n, seed & (2**64 - 1))


def kv_protect(key, value, op_type=None, seq=None, cf=None):
    """ProtectionInfo64().ProtectKV[O](...)[.ProtectS(seq)][.ProtectC(cf)]"""
    kp, kn, _k1 = _buf(key)
    vp, vn, _k2 = _buf(value)
    return lib().oracle_kv_protect(kp, kn, vp, vn, -1 if op_type is None else op_type,
                                   seq is not None, seq or 0, cf is not None, cf or 0)


def hash64_batch(base, offsets, lengths, seeds=None, seed=0):
    out = np.zeros(len(offsets), dtype=np.uint64)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lengths = np.ascontiguousarray(lengths, np.uint32)
    lib().oracle_hash64_batch(_ptr(base), _ptr(offsets), _ptr(lengths),
                              _ptr(None if seeds is None else np.ascontiguousarray(seeds, np.uint64)),
                              seed, _ptr(out), len(offsets))
    return out


def kv_protect_batch(base, key_offsets, key_sizes, value_offsets, value_sizes, op_types=None,
                     seqnos=None, cf_ids=None):
    n = len(key_offsets)
    out = np.zeros(n, dtype=np.uint64)
    arrs = [np.ascontiguousarray(key_offsets, np.uint64), np.ascontiguousarray(key_sizes, np.uint32),
            np.ascontiguousarray(value_offsets, np.uint64),
            np.ascontiguousarray(value_sizes, np.uint32)]
    opt = [None if op_types is None else np.ascontiguousarray(op_types, np.uint8),
           None if seqnos is None else np.ascontiguousarray(seqnos, np.uint64),
           None if cf_ids is None else np.ascontiguousarray(cf_ids, np.uint32)]
    lib().oracle_kv_protect_batch(_ptr(base), *[_ptr(a) for a in arrs], *[_ptr(a) for a in opt],
                                  _ptr(out), n)
    return out


def memtable_verify_batch(base, base_len, offsets, prot_bytes):
    """MemTable::VerifyEntryChecksum per encoded entry (db/memtable.cc:273-307):
    (computed, status) -- status codes as include/forst_checksum.h"""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets)
    comp = np.zeros(n, np.uint64)
    st = np.zeros(n, np.uint8)
    lib().oracle_memtable_verify_batch(_ptr(base), base_len, _ptr(offsets), n, prot_bytes,
                                       _ptr(comp), _ptr(st))
    return comp, st


MEM_STATUS = {0: "OK",
              1: "Corruption: Unable to parse internal key length",
              2: "Corruption: Memtable entry internal key length too short.",
              3: "Corruption: Unable to parse internal key value",
              4: "Corruption: Corrupted memtable entry, per key-value checksum verification "
                 "failed."}  # db/memtable.cc:280-306

WB_STATUS = {0: "OK", 1: "Corruption: malformed WriteBatch (too small)",
             2: "Corruption: bad WriteBatch Put", 3: "Corruption: bad WriteBatch Delete",
             4: "Corruption: bad WriteBatch DeleteRange", 5: "Corruption: bad WriteBatch Merge",
             6: "Corruption: bad WriteBatch BlobIndex", 7: "Corruption: bad WriteBatch Blob",
             8: "Corruption: bad EndPrepare XID", 9: "Corruption: bad commit timestamp",
             10: "Corruption: bad Commit XID", 11: "Corruption: bad Rollback XID",
             12: "Corruption: bad WriteBatch PutEntity", 13: "Corruption: unknown WriteBatch tag",
             14: "Corruption: WriteBatch has wrong count"}  # db/write_batch.cc:361-716

# ReadRecordFromWriteBatch (write_batch.cc:361-475): tag -> (has cf, parts, error,
# ProtectionInfoUpdater op type (write_batch.cc:3023-3052) or None)
_WB_TAGS = {0x05: (1, "kv", 2, 0x01), 0x01: (0, "kv", 2, 0x01),
            0x04: (1, "k", 3, 0x00), 0x08: (1, "k", 3, 0x07), 0x00: (0, "k", 3, 0x00),
            0x07: (0, "k", 3, 0x07), 0x0E: (1, "kv", 4, 0x0F), 0x0F: (0, "kv", 4, 0x0F),
            0x06: (1, "kv", 5, 0x02), 0x02: (0, "kv", 5, 0x02), 0x10: (1, "kv", 6, 0x11),
            0x11: (0, "kv", 6, 0x11), 0x17: (1, "kv", 12, 0x16), 0x16: (0, "kv", 12, 0x16),
            0x03: (0, "x", 7, None), 0x0D: (0, "", 0, None), 0x09: (0, "", 0, None),
            0x12: (0, "", 0, None), 0x13: (0, "", 0, None), 0x0A: (0, "x", 8, None),
            0x0B: (0, "x", 10, None), 0x15: (0, "kx", 9, None), 0x0C: (0, "x", 11, None)}


def _wb_varint(b, p, end):
    """GetVarint32 over input [p, end): (value, next p) or None"""
    r = 0
    for j in range(5):
        if p + j >= end:
            return None
        x = b[p + j]
        r |= (x & 127) << (7 * j)
        if not x & 128:
            return r & 0xFFFFFFFF, p + j + 1
    return None


def write_batch_protect(rep):
    """WriteBatchInternal::UpdateProtectionInfo(wb, 8) restated
    (write_batch.cc:3164-3181, Iterate :477-716, ReadRecordFromWriteBatch
    :361-475): (status code as WB_STATUS, [protection values of the data
    records in order])"""
    b = bytes(rep)
    if len(b) < 12:
        return 1, []
    count = struct.unpack_from("<I", b, 8)[0]
    p, end, out = 12, len(b), []
    while p < end:
        tag = b[p]
        p += 1
        if tag not in _WB_TAGS:
            return 13, out
        has_cf, parts, err, op = _WB_TAGS[tag]
        cf, sl = 0, []
        if has_cf:
            v = _wb_varint(b, p, end)
            if v is None:
                return err, out
            cf, p = v
        for i, part in enumerate(parts):
            v = _wb_varint(b, p, end)
            if v is None or end - v[1] < v[0]:
                return (10 if tag == 0x15 and i == 1 else err), out
            sl.append(b[v[1]:v[1] + v[0]])
            p = v[1] + v[0]
        if op is not None:
            out.append(kv_protect(sl[0], sl[1] if len(sl) > 1 else b"", op, cf=cf))
    return (14 if len(out) != count else 0), out


def splitmix64(x):
    return lib().oracle_splitmix64(x)


def fill_stream(start, nbytes, seed):
    out = np.empty(nbytes, dtype=np.uint8)
    lib().oracle_fill_stream(_ptr(out), start, nbytes, seed)
    return out
