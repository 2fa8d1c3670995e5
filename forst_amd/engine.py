"""Python mirror of the reference's checksum interface over the HIP engine.

Names follow the reference (table/format.h, table/block_based/reader_common.h,
util/crc32c.h, util/xxhash.h, db/log_reader.cc); every function is the batched
GPU form of the reference's per-block CPU call and runs the gfx950 kernels in
forst_amd/lib/libforst_checksum.so.  Device buffers are torch CUDA tensors
(torch is only plumbing for device memory and streams).  Calls are enqueued on
torch's current stream.
"""
import ctypes
import enum

import torch

from ._lib import check, lib


class ChecksumType(enum.IntEnum):
    """include/rocksdb/table.h:54-60"""
    kNoChecksum = 0
    kCRC32c = 1
    kxxHash = 2
    kxxHash64 = 3
    kXXH3 = 4


class WalStatus(enum.IntEnum):
    """per-log-block outcome of forst_wal_verify_batch"""
    OK = 0
    BAD_CHECKSUM = 1
    BAD_LENGTH = 2
    ZERO_RECORD = 3
    OLD_RECORD = 4


def _p(t):
    return None if t is None else t.data_ptr()


def _stream(stream):
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, torch.cuda.Stream):
        return stream.cuda_stream
    return stream


def _dev_u8(base):
    assert base.is_cuda and base.dtype == torch.uint8 and base.is_contiguous()
    return base


def _desc(offsets, sizes):
    assert offsets.is_cuda and offsets.dtype in (torch.int64, torch.uint64)
    assert sizes.is_cuda and sizes.dtype in (torch.int32, torch.uint32)
    assert offsets.is_contiguous() and sizes.is_contiguous()
    assert offsets.numel() == sizes.numel()
    return offsets.numel()


def init_device():
    check(lib().forst_init_device())


def version():
    return lib().forst_version().decode()


def last_kernel():
    return lib().forst_last_kernel().decode()


def block_checksum_batch(ctype, base, offsets, sizes, last_bytes=None, modifiers=None,
                         out=None, stream=None):
    """ComputeBuiltinChecksumWithLastByte + ChecksumModifierForContext per block
    (table/format.cc:594, table/format.h:119) -> uint32 tensor."""
    n = _desc(offsets, sizes)
    _dev_u8(base)
    if out is None:
        out = torch.empty(n, dtype=torch.uint32, device=base.device)
    check(lib().forst_block_checksum_batch(int(ctype), base.data_ptr(), base.numel(),
                                           offsets.data_ptr(), sizes.data_ptr(),
                                           _p(last_bytes), _p(modifiers), out.data_ptr(),
                                           n, _stream(stream)))
    return out


def block_trailer_batch(ctype, base, offsets, sizes, last_bytes, modifiers=None, out=None,
                        stream=None):
    """Writes [type][LE32 checksum] after each block in place, as
    BlockBasedTableBuilder::WriteMaybeCompressedBlock appends it."""
    n = _desc(offsets, sizes)
    _dev_u8(base)
    check(lib().forst_block_trailer_batch(int(ctype), base.data_ptr(), base.numel(),
                                          offsets.data_ptr(), sizes.data_ptr(),
                                          _p(last_bytes), _p(modifiers), _p(out),
                                          n, _stream(stream)))
    return out


def block_verify_batch(ctype, base, offsets, sizes, modifiers=None, computed=True,
                       stored=True, ok=True, mismatches=None, stream=None):
    """VerifyBlockChecksum per block (table/block_based/reader_common.cc:26).
    Returns (computed, stored, ok, mismatches) tensors (None where not asked)."""
    n = _desc(offsets, sizes)
    _dev_u8(base)
    dev = base.device
    c = torch.empty(n, dtype=torch.uint32, device=dev) if computed is True else computed
    s = torch.empty(n, dtype=torch.uint32, device=dev) if stored is True else stored
    o = torch.empty(n, dtype=torch.uint8, device=dev) if ok is True else ok
    if mismatches is None:
        mismatches = torch.zeros(1, dtype=torch.int64, device=dev)
    check(lib().forst_block_verify_batch(int(ctype), base.data_ptr(), base.numel(),
                                         offsets.data_ptr(), sizes.data_ptr(), _p(modifiers),
                                         _p(c), _p(s), _p(o), _p(mismatches), n,
                                         _stream(stream)))
    return c, s, o, mismatches


def crc32c_batch(base, offsets, lengths, init_crcs=None, out=None, stream=None):
    """crc32c::Extend(init, data, n) per buffer (util/crc32c.h:25), unmasked."""
    n = _desc(offsets, lengths)
    _dev_u8(base)
    if out is None:
        out = torch.empty(n, dtype=torch.uint32, device=base.device)
    check(lib().forst_crc32c_batch(base.data_ptr(), base.numel(), offsets.data_ptr(),
                                   lengths.data_ptr(), _p(init_crcs), out.data_ptr(), n,
                                   _stream(stream)))
    return out


def crc32c_buffer(base, init=0, out=None, stream=None):
    """crc32c::Extend(init, base) over one device buffer of any size
    (FileChecksumGenCrc32c, util/file_checksum_helper.h:22).  Returns a
    1-element uint32 device tensor."""
    _dev_u8(base)
    if out is None:
        out = torch.empty(1, dtype=torch.uint32, device=base.device)
    check(lib().forst_crc32c_buffer(base.data_ptr(), base.numel(), init & 0xFFFFFFFF,
                                    out.data_ptr(), _stream(stream)))
    return out


def crc32c_combine_batch(crc1, crc2, len2, out=None, stream=None):
    """crc32c::Crc32cCombine per element (util/crc32c.h:32), device arrays."""
    n = crc1.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.uint32, device=crc1.device)
    check(lib().forst_crc32c_combine_batch(crc1.data_ptr(), crc2.data_ptr(), len2.data_ptr(),
                                           out.data_ptr(), n, _stream(stream)))
    return out


def crc32c_combine(crc1, crc2, len2):
    """host crc32c::Crc32cCombine (no GPU call)."""
    return lib().forst_crc32c_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, len2)


def xxh3_64_batch(base, offsets, lengths, out=None, stream=None):
    """XXH3_64bits per buffer (util/xxhash.h:5311)."""
    n = _desc(offsets, lengths)
    _dev_u8(base)
    if out is None:
        out = torch.empty(n, dtype=torch.uint64, device=base.device)
    check(lib().forst_xxh3_64_batch(base.data_ptr(), base.numel(), offsets.data_ptr(),
                                    lengths.data_ptr(), out.data_ptr(), n, _stream(stream)))
    return out


def wal_verify_batch(log, log_number=0, first_block=0, n_blocks=None, bad_blocks=None,
                     stream=None):
    """Physical-record CRC verification of 32 KiB log blocks
    (db/log_reader.cc:450-531).  Returns (status, nrec, fail_off, bad_blocks)."""
    _dev_u8(log)
    total = (log.numel() + 32767) // 32768
    if n_blocks is None:
        n_blocks = total - first_block
    dev = log.device
    status = torch.empty(n_blocks, dtype=torch.uint8, device=dev)
    nrec = torch.empty(n_blocks, dtype=torch.uint32, device=dev)
    fail = torch.empty(n_blocks, dtype=torch.uint32, device=dev)
    if bad_blocks is None:
        bad_blocks = torch.zeros(1, dtype=torch.int64, device=dev)
    check(lib().forst_wal_verify_batch(log.data_ptr(), log.numel(), first_block, n_blocks,
                                       log_number, status.data_ptr(), nrec.data_ptr(),
                                       fail.data_ptr(), bad_blocks.data_ptr(), _stream(stream)))
    return status, nrec, fail, bad_blocks


def wal_record_crc_batch(log, header_offsets, write_in_place=True, out=None, stream=None,
                         payload_lengths=None, recyclable=False):
    """log::Writer::EmitPhysicalRecord CRC (db/log_writer.cc:228-263) for
    headers already laid out in `log`.  With payload_lengths (device int32,
    the lengths the writer laid out: forst_wal_record_crc_lengths) the
    descriptors come from the arrays instead of a pass over the headers."""
    _dev_u8(log)
    n = header_offsets.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.uint32, device=log.device)
    if payload_lengths is not None:
        assert payload_lengths.numel() == n and payload_lengths.element_size() == 4
        check(lib().forst_wal_record_crc_lengths(log.data_ptr(), log.numel(),
                                                 header_offsets.data_ptr(),
                                                 payload_lengths.data_ptr(), n, int(recyclable),
                                                 int(write_in_place), out.data_ptr(),
                                                 _stream(stream)))
        return out
    check(lib().forst_wal_record_crc_batch(log.data_ptr(), log.numel(),
                                           header_offsets.data_ptr(), n, int(write_in_place),
                                           out.data_ptr(), _stream(stream)))
    return out


def wal_record_xxh3_batch(log, header_offsets, stream=None):
    """XXH3_64bits per logical record (log_reader.cc:95-165).  Returns
    (hashes int64 [n_logical], first physical record index [n_logical])."""
    _dev_u8(log)
    n = header_offsets.numel()
    hashes = torch.empty(max(n, 1), dtype=torch.int64, device=log.device)
    first = torch.empty(max(n, 1), dtype=torch.int64, device=log.device)
    nl = ctypes.c_uint64()
    check(lib().forst_wal_record_xxh3_batch(log.data_ptr(), log.numel(), header_offsets.data_ptr(),
                                            n, hashes.data_ptr(), first.data_ptr(),
                                            ctypes.byref(nl), _stream(stream)))
    return hashes[:nl.value], first[:nl.value]


class WalRecords(ctypes.Structure):
    """forst_wal_records (device array pointers)"""
    _fields_ = [("offset", ctypes.c_void_p), ("length", ctypes.c_void_p),
                ("hash", ctypes.c_void_p), ("n_fragments", ctypes.c_void_p)]


class WalReports(ctypes.Structure):
    """forst_wal_reports (device array pointers)"""
    _fields_ = [("offset", ctypes.c_void_p), ("bytes", ctypes.c_void_p),
                ("reason", ctypes.c_void_p), ("type", ctypes.c_void_p)]


class WalRecoverResult(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("n_reports", ctypes.c_uint64),
                ("n_physical", ctypes.c_uint64), ("stop_offset", ctypes.c_uint64),
                ("stop_reason", ctypes.c_uint32), ("truncated", ctypes.c_uint32),
                ("unsupported", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


# forst_wal_report_reason -> the reader's Reporter::Corruption text (log_reader.cc)
WAL_REASONS = {1: "partial record without end(1)", 2: "partial record without end(2)",
               3: "missing start of fragmented record(1)",
               4: "missing start of fragmented record(2)", 5: "error in middle of record",
               6: "checksum mismatch", 7: "bad record length", 8: "truncated header",
               9: "error reading trailing data", 10: "truncated record body",
               11: "unknown record type %u"}
WAL_STOPS = {0: "eof", 1: "old_record", 2: "truncated_header", 3: "truncated_body",
             4: "recycled_tail"}
# WALRecoveryMode (include/rocksdb/options.h)
kTolerateCorruptedTailRecords, kAbsoluteConsistency, kPointInTimeRecovery, \
    kSkipAnyCorruptedRecords = 0, 1, 2, 3


def _recover_sig(L):
    f = L.forst_wal_recover_batch
    if f.argtypes is None:
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        f.restype = ctypes.c_int
        f.argtypes = [vp, u64, ctypes.c_uint32, ctypes.c_int, WalRecords, u64, WalReports, u64,
                      vp, vp]


def wal_recover_batch(log, log_number=0, mode=kPointInTimeRecovery, record_capacity=None,
                      report_capacity=1024, stream=None):
    """log::Reader::ReadRecord over a whole device log image (log_reader.cc:69-320):
    returns (records dict of device tensors offset/length/hash/n_fragments,
    reports dict of device tensors offset/bytes/reason/type, result)."""
    _dev_u8(log)
    _recover_sig(lib())
    if record_capacity is None:
        record_capacity = max(1024, log.numel() // 1024)
    while True:
        dev = log.device
        rec = {"offset": torch.empty(record_capacity, dtype=torch.int64, device=dev),
               "length": torch.empty(record_capacity, dtype=torch.int64, device=dev),
               "hash": torch.empty(record_capacity, dtype=torch.int64, device=dev),
               "n_fragments": torch.empty(record_capacity, dtype=torch.int32, device=dev)}
        rep = {"offset": torch.empty(report_capacity, dtype=torch.int64, device=dev),
               "bytes": torch.empty(report_capacity, dtype=torch.int64, device=dev),
               "reason": torch.empty(report_capacity, dtype=torch.int32, device=dev),
               "type": torch.empty(report_capacity, dtype=torch.int32, device=dev)}
        res = WalRecoverResult()
        check(lib().forst_wal_recover_batch(
            log.data_ptr(), log.numel(), log_number, mode,
            WalRecords(*[rec[k].data_ptr() for k in ("offset", "length", "hash", "n_fragments")]),
            record_capacity,
            WalReports(*[rep[k].data_ptr() for k in ("offset", "bytes", "reason", "type")]),
            report_capacity, ctypes.byref(res), _stream(stream)))
        if not res.truncated:
            break
        record_capacity = max(record_capacity, res.n_records)
        report_capacity = max(report_capacity, res.n_reports)
    rec = {k: v[:res.n_records] for k, v in rec.items()}
    rep = {k: v[:res.n_reports] for k, v in rep.items()}
    return rec, rep, res


def hash64_batch(base, offsets, lengths, seeds=None, seed=0, out=None, stream=None):
    """Hash64 / NPHash64 per buffer (util/hash.cc:81, XXPH3 0.7.2 preview)."""
    n = _desc(offsets, lengths)
    _dev_u8(base)
    if out is None:
        out = torch.empty(n, dtype=torch.uint64, device=base.device)
    check(lib().forst_hash64_batch(base.data_ptr(), base.numel(), offsets.data_ptr(),
                                   lengths.data_ptr(), _p(seeds), seed & (2**64 - 1),
                                   out.data_ptr(), n, _stream(stream)))
    return out


def kv_protect_batch(base, key_offsets, key_sizes, value_offsets, value_sizes, op_types=None,
                     seqnos=None, cf_ids=None, out=None, stream=None):
    """ProtectionInfo64 ProtectKV / ProtectKVO [+S] [+C] per entry (db/kv_checksum.h)."""
    n = _desc(key_offsets, key_sizes)
    assert _desc(value_offsets, value_sizes) == n
    _dev_u8(base)
    if out is None:
        out = torch.empty(n, dtype=torch.uint64, device=base.device)
    check(lib().forst_kv_protect_batch(base.data_ptr(), base.numel(), key_offsets.data_ptr(),
                                       key_sizes.data_ptr(), value_offsets.data_ptr(),
                                       value_sizes.data_ptr(), _p(op_types), _p(seqnos),
                                       _p(cf_ids), out.data_ptr(), n, _stream(stream)))
    return out


def kv_verify_batch(base, key_offsets, key_sizes, value_offsets, value_sizes, protection_bytes,
                    checksum_offsets, op_types=None, seqnos=None, cf_ids=None, computed=True,
                    ok=True, mismatches=None, stream=None):
    """ProtectionInfo<T>::Verify per entry (db/kv_checksum.h:117-133), e.g.
    MemTable::VerifyEntryChecksum.  Returns (computed, ok, mismatches)."""
    n = _desc(key_offsets, key_sizes)
    _dev_u8(base)
    dev = base.device
    c = torch.empty(n, dtype=torch.uint64, device=dev) if computed is True else computed
    o = torch.empty(n, dtype=torch.uint8, device=dev) if ok is True else ok
    if mismatches is None:
        mismatches = torch.zeros(1, dtype=torch.int64, device=dev)
    check(lib().forst_kv_verify_batch(base.data_ptr(), base.numel(), key_offsets.data_ptr(),
                                      key_sizes.data_ptr(), value_offsets.data_ptr(),
                                      value_sizes.data_ptr(), _p(op_types), _p(seqnos),
                                      _p(cf_ids), protection_bytes, checksum_offsets.data_ptr(),
                                      _p(c), _p(o), _p(mismatches), n, _stream(stream)))
    return c, o, mismatches


def memtable_verify_batch(base, entry_offsets, protection_bytes, computed=True, status=True,
                          mismatches=None, stream=None):
    """MemTable::VerifyEntryChecksum per encoded entry (db/memtable.cc:273-307),
    decoded on the device.  Returns (computed, status, mismatches); status
    codes as in include/forst_checksum.h."""
    _dev_u8(base)
    n = entry_offsets.numel()
    dev = base.device
    c = torch.empty(n, dtype=torch.uint64, device=dev) if computed is True else computed
    s = torch.empty(n, dtype=torch.uint8, device=dev) if status is True else status
    if mismatches is None:
        mismatches = torch.zeros(1, dtype=torch.int64, device=dev)
    check(lib().forst_memtable_verify_batch(base.data_ptr(), base.numel(), entry_offsets.data_ptr(),
                                            n, protection_bytes, _p(c), _p(s), _p(mismatches),
                                            _stream(stream)))
    return c, s, mismatches


def memtable_protect_batch(base, entry_offsets, protection_bytes, write_in_place=True, out=True,
                           status=True, stream=None):
    """MemTable::UpdateEntryChecksum per encoded entry (db/memtable.cc:676-693):
    the protection value, written in place as Encode(protection_bytes).
    Returns (out, status)."""
    _dev_u8(base)
    n = entry_offsets.numel()
    dev = base.device
    o = torch.empty(n, dtype=torch.uint64, device=dev) if out is True else out
    s = torch.empty(n, dtype=torch.uint8, device=dev) if status is True else status
    check(lib().forst_memtable_protect_batch(base.data_ptr(), base.numel(),
                                             entry_offsets.data_ptr(), n, protection_bytes,
                                             1 if write_in_place else 0, _p(o), _p(s),
                                             _stream(stream)))
    return o, s


def write_batch_protect_batch(base, rep_offsets, rep_sizes, capacity=None, stream=None):
    """WriteBatchInternal::UpdateProtectionInfo per WriteBatch rep
    (db/write_batch.cc:3164-3181), parsed on the device.  Returns
    (prot, first_entry, status, n_protected): rep b's protection values are
    prot[first_entry[b]:first_entry[b+1]].  Synchronous (one count read-back)."""
    _dev_u8(base)
    n = _desc(rep_offsets, rep_sizes)
    dev = base.device
    first = torch.empty(n + 1, dtype=torch.int64, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    nprot = torch.empty(n, dtype=torch.int32, device=dev)
    total = ctypes.c_uint64()
    if capacity is None:  # size from the header counts: a first call with capacity 0
        rc = lib().forst_write_batch_protect_batch(base.data_ptr(), base.numel(),
                                                   rep_offsets.data_ptr(), rep_sizes.data_ptr(),
                                                   n, first.data_ptr(), None, 0, None, None,
                                                   ctypes.byref(total), _stream(stream))
        if rc != 0 and total.value == 0:
            check(rc)
        capacity = total.value
    prot = torch.empty(max(1, capacity), dtype=torch.uint64, device=dev)
    check(lib().forst_write_batch_protect_batch(base.data_ptr(), base.numel(),
                                                rep_offsets.data_ptr(), rep_sizes.data_ptr(), n,
                                                first.data_ptr(), prot.data_ptr(), capacity,
                                                status.data_ptr(), nprot.data_ptr(),
                                                ctypes.byref(total), _stream(stream)))
    return prot[:total.value], first, status, nprot


class BlockKind(enum.IntFlag):
    """kinds[] of block_kv_checksum_batch (include/forst_checksum.h)"""
    DATA = 0
    INDEX = 1
    META = 2
    VALUE_IS_FULL = 4
    HAS_FIRST_KEY = 8


def block_kv_checksum_batch(base, block_offsets, block_sizes, kinds, protection_bytes,
                            capacity=None, stream=None):
    """Block::Initialize{Data,Index,MetaIndex}BlockProtectionInfo per block
    (table/block_based/block.cc:1113-1235), decoded on the device.  Returns
    (kv_checksums u8, prot u64, first_key, status): block b's kv_checksum_ is
    kv_checksums[first_key[b] * pb : first_key[b+1] * pb].  Synchronous."""
    _dev_u8(base)
    n = _desc(block_offsets, block_sizes)
    dev = base.device
    first = torch.empty(n + 1, dtype=torch.int64, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    total = ctypes.c_uint64()
    args = (base.data_ptr(), base.numel(), block_offsets.data_ptr(), block_sizes.data_ptr(),
            kinds.data_ptr(), n, protection_bytes, first.data_ptr())
    if capacity is None:
        rc = lib().forst_block_kv_checksum_batch(*args, None, None, 0, None, ctypes.byref(total),
                                                 _stream(stream))
        if rc != 0 and total.value == 0:
            check(rc)
        capacity = total.value
    enc = torch.empty(max(1, capacity) * protection_bytes, dtype=torch.uint8, device=dev)
    prot = torch.empty(max(1, capacity), dtype=torch.uint64, device=dev)
    check(lib().forst_block_kv_checksum_batch(*args, enc.data_ptr(), prot.data_ptr(), capacity,
                                              status.data_ptr(), ctypes.byref(total),
                                              _stream(stream)))
    m = total.value
    return enc[:m * protection_bytes], prot[:m], first, status


def fill_stream(dev_u8, start, seed, stream=None):
    """Synthetic splitmix64 byte stream written on the device."""
    _dev_u8(dev_u8)
    check(lib().forst_fill_stream(dev_u8.data_ptr(), start, dev_u8.numel(), seed,
                                  _stream(stream)))
    return dev_u8
