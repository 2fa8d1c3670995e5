"""oracle/wal_reader.py -- TEST INFRASTRUCTURE ONLY.

Serial CPU restatement of the reference WAL reader for the fused recovery
pass (forst_wal_recover_batch): log::Reader::ReadRecord
(db/log_reader.cc:69-320), ReadPhysicalRecord (:450-531) and ReadMore
(:404-448), no WAL compression, with the XXH3 record checksum of every
logical record (:95-165) and the reporter's Corruption(bytes, reason) calls in
order.  Record types db/log_format.h:20-41; recovery modes
include/rocksdb/options.h (WALRecoveryMode).  CRC32C and XXH3 come from the
pinned C oracle (oracle/oracle.c).
"""
from . import oracle as O

kBlockSize, kHeaderSize, kRecyclableHeaderSize = 32768, 7, 11  # log_format.h:45-52
kZeroType, kFullType, kFirstType, kMiddleType, kLastType = 0, 1, 2, 3, 4
kRecyclableFullType, kRecyclableLastType = 5, 8
kSetCompressionType, kUserDefinedTimestampSizeType = 9, 10
kRecyclableUserDefinedTimestampSizeType = 11
# ReadPhysicalRecord's extra results (log_reader.h)
kEof, kBadRecord, kBadHeader, kOldRecord, kBadRecordLen, kBadRecordChecksum = \
    "eof", "bad_record", "bad_header", "old_record", "bad_record_len", "bad_record_checksum"

# WALRecoveryMode (include/rocksdb/options.h)
kTolerateCorruptedTailRecords, kAbsoluteConsistency, kPointInTimeRecovery, \
    kSkipAnyCorruptedRecords = 0, 1, 2, 3


class Unsupported(Exception):
    pass


class Reader:
    def __init__(self, log, log_number=0):
        self.log = bytes(log)
        self.log_number = log_number
        self.file_pos = 0
        self.buf_lo = self.buf_hi = 0   # buffer_ = log[buf_lo:buf_hi]
        self.eof = False
        self.end_of_buffer_offset = 0
        self.recycled = False
        self.reports = []  # (bytes, reason, reader position of the physical record)
        self.cur_phys = 0

    def _size(self):
        return self.buf_hi - self.buf_lo

    def _report(self, nbytes, reason):
        self.reports.append((nbytes, reason, self.cur_phys))

    def read_more(self):  # log_reader.cc:404-448
        if not self.eof:
            n = min(kBlockSize, len(self.log) - self.file_pos)
            self.buf_lo, self.buf_hi = self.file_pos, self.file_pos + n
            self.file_pos += n
            self.end_of_buffer_offset += n
            if n < kBlockSize:
                self.eof = True
            return None, 0
        if self._size():
            drop = self._size()
            self.buf_lo = self.buf_hi
            return kBadHeader, drop
        self.buf_lo = self.buf_hi
        return kEof, 0

    def read_physical_record(self):  # log_reader.cc:450-531
        while True:
            if self._size() < kHeaderSize:
                r, drop = self.read_more()
                if r is not None:
                    return r, drop, None
                continue
            h = self.log[self.buf_lo:self.buf_lo + kRecyclableHeaderSize]
            length = h[4] | (h[5] << 8)
            rtype = h[6]
            header_size = kHeaderSize
            recyc = (kRecyclableFullType <= rtype <= kRecyclableLastType) or \
                rtype == kRecyclableUserDefinedTimestampSizeType
            if recyc:
                header_size = kRecyclableHeaderSize
                if self.end_of_buffer_offset - self._size() == 0:
                    self.recycled = True
                if self._size() < kRecyclableHeaderSize:
                    r, drop = self.read_more()
                    if r is not None:
                        return r, drop, None
                    continue
            if header_size + length > self._size():
                drop = self._size()
                self.buf_lo = self.buf_hi
                return kBadRecordLen, drop, None
            if recyc:
                log_num = int.from_bytes(h[7:11], "little")
                if log_num != self.log_number:
                    self.buf_lo += header_size + length
                    return kOldRecord, 0, None
            if rtype == kZeroType and length == 0:
                self.buf_lo = self.buf_hi
                return kBadRecord, 0, None
            expected = O.unmask(int.from_bytes(h[0:4], "little"))
            hdr = self.log[self.buf_lo + 6:self.buf_lo + header_size + length]
            if O.crc32c_value(hdr) != expected:
                drop = self._size()
                self.buf_lo = self.buf_hi
                return kBadRecordChecksum, drop, None
            frag = self.log[self.buf_lo + header_size:self.buf_lo + header_size + length]
            self.buf_lo += header_size + length
            if rtype in (kSetCompressionType, kUserDefinedTimestampSizeType,
                         kRecyclableUserDefinedTimestampSizeType):
                raise Unsupported("WAL compression / timestamp-size records")
            return rtype, 0, frag

    def read_record(self, mode):  # log_reader.cc:69-320
        scratch = b""
        in_frag = False
        prospective = 0
        while True:
            phys = self.end_of_buffer_offset - self._size()
            self.cur_phys = phys
            rt, drop, frag = self.read_physical_record()
            if rt in (kFullType, kRecyclableFullType):
                if in_frag and scratch:
                    self._report(len(scratch), "partial record without end(1)")
                return phys, frag
            if rt in (kFirstType, kFirstType + 4):
                if in_frag and scratch:
                    self._report(len(scratch), "partial record without end(2)")
                prospective = phys
                scratch = frag
                in_frag = True
                continue
            if rt in (kMiddleType, kMiddleType + 4):
                if not in_frag:
                    self._report(len(frag), "missing start of fragmented record(1)")
                else:
                    scratch += frag
                continue
            if rt in (kLastType, kLastType + 4):
                if not in_frag:
                    self._report(len(frag), "missing start of fragmented record(2)")
                    continue
                return prospective, scratch + frag
            strict = mode in (kAbsoluteConsistency, kPointInTimeRecovery)
            if rt == kBadHeader:
                if strict:
                    self._report(drop, "truncated header")
                rt = kEof
            if rt == kEof:
                if in_frag and strict:
                    self._report(len(scratch), "error reading trailing data")
                return None
            if rt == kOldRecord:
                if mode != kSkipAnyCorruptedRecords:
                    if in_frag and strict:
                        self._report(len(scratch), "error reading trailing data")
                    return None
                rt = kBadRecord
            if rt == kBadRecord:
                if in_frag:
                    self._report(len(scratch), "error in middle of record")
                    in_frag, scratch = False, b""
                continue
            if rt == kBadRecordLen:
                if self.eof:
                    if strict:
                        self._report(drop, "truncated record body")
                    return None
            if rt in (kBadRecordLen, kBadRecordChecksum):
                if self.recycled and mode == kTolerateCorruptedTailRecords:
                    return None
                self._report(drop, "bad record length" if rt == kBadRecordLen
                             else "checksum mismatch")
                if in_frag:
                    self._report(len(scratch), "error in middle of record")
                    in_frag, scratch = False, b""
                continue
            # unknown record type (:308-316)
            self._report(len(frag) + (len(scratch) if in_frag else 0),
                         "unknown record type %u" % rt)
            in_frag, scratch = False, b""


def read_all(log, log_number=0, mode=kPointInTimeRecovery):
    """Every logical record ReadRecord returns, in order: (record offset =
    Reader::LastRecordOffset, length, XXH3_64bits), and the reporter's
    (bytes, reason, reader position) calls."""
    r = Reader(log, log_number)
    recs = []
    while True:
        got = r.read_record(mode)
        if got is None:
            break
        off, payload = got
        recs.append((off, len(payload), O.xxh3_64(payload)))
    return recs, r.reports
