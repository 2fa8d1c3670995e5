"""oracle/wal_reader.py -- TEST INFRASTRUCTURE ONLY.

Serial CPU restatement of the reference WAL reader for the fused recovery
pass (forst_wal_recover_batch): log::Reader::ReadRecord
(db/log_reader.cc:69-320), ReadPhysicalRecord (:450-592), ReadMore
(:404-448) and UpdateRecordedTimestampSize, with the XXH3 record checksum
(:73-79, :95-165) and the reporter's Corruption(bytes, reason) calls in order.
Record types db/log_format.h:20-43; recovery modes include/rocksdb/options.h
(WALRecoveryMode).  CRC32C and XXH3 come from the pinned C oracle
(oracle/oracle.c).

Pinned against the reference reader itself: tests/golden/gen_wal_golden.py
drives the reference's compiled log::Reader over the scenario logs of
tests/walcases.py and commits its transcripts (tests/golden/wal_reader.json);
tests/test_wal_golden.py checks this restatement against them.  Behaviours
the pinning brought out, restated here as the reference has them:
  * the record type is read from a `const char*` into `unsigned int`
    (:466-469), so a type byte >= 0x80 sign-extends ("unknown record type
    4294967295" for 0xFF);
  * ReadPhysicalRecord's own results share the type space (log_reader.h:173-
    186: kEof = kMaxRecordType + 1 = 12 ... kBadRecordChecksum = 17), so a
    physical record of type 12..17 with a valid CRC acts as that result (with
    drop_size 0 and the buffer NOT cleared);
  * the XXH3 state of a fragmented record is only reset at the start of
    ReadRecord and at "partial record without end(2)" (:73-79, :119-124), so
    after an aborted fragmented record (error in middle, unknown type, ...)
    the next fragmented record's checksum also covers the aborted fragments;
  * kSetCompressionType / timestamp-size records clear scratch but keep
    in_fragmented_record (:167-213).
WAL compression (a kSetCompressionType record naming kZSTD) is not restated:
it raises Unsupported, as forst_wal_recover_batch reports unsupported.
"""
from . import oracle as O

kBlockSize, kHeaderSize, kRecyclableHeaderSize = 32768, 7, 11  # log_format.h:45-52
kZeroType, kFullType, kFirstType, kMiddleType, kLastType = 0, 1, 2, 3, 4
kRecyclableFullType, kRecyclableFirstType, kRecyclableMiddleType, kRecyclableLastType = 5, 6, 7, 8
kSetCompressionType, kUserDefinedTimestampSizeType = 9, 10
kRecyclableUserDefinedTimestampSizeType = 11
kMaxRecordType = 11
# ReadPhysicalRecord's extra results (log_reader.h:173-186)
kEof, kBadRecord, kBadHeader, kOldRecord, kBadRecordLen, kBadRecordChecksum = range(12, 18)
kZSTD = 7

# WALRecoveryMode (include/rocksdb/options.h)
kTolerateCorruptedTailRecords, kAbsoluteConsistency, kPointInTimeRecovery, \
    kSkipAnyCorruptedRecords = 0, 1, 2, 3


class Unsupported(Exception):
    pass


class _Hash:
    """XXH3_64bits streaming state as a byte accumulator (xxhash.h)"""

    def __init__(self):
        self.data = bytearray()

    def reset(self):
        self.data = bytearray()

    def update(self, b):
        self.data += b

    def digest(self):
        return O.xxh3_64(bytes(self.data))


class Reader:
    def __init__(self, log, log_number=0):
        self.log = bytes(log)
        self.log_number = log_number
        self.file_pos = 0
        self.buf_lo = self.buf_hi = 0   # buffer_ = log[buf_lo:buf_hi]
        self.eof = False
        self.end_of_buffer_offset = 0
        self.recycled = False
        self.first_record_read = False
        self.compression_type_record_read = False
        self.recorded_ts = {}
        self.hash = _Hash()
        self.last_record_offset = 0
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

    def read_physical_record(self):  # log_reader.cc:450-592
        while True:
            if self._size() < kHeaderSize:
                r, drop = self.read_more()
                if r is not None:
                    return r, drop, None
                continue
            h = self.log[self.buf_lo:self.buf_lo + kRecyclableHeaderSize]
            length = h[4] | (h[5] << 8)
            rtype = h[6] if h[6] < 0x80 else h[6] | 0xFFFFFF00  # char -> unsigned int
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
            return rtype, 0, frag

    def read_record(self, mode):  # log_reader.cc:69-320
        scratch = b""
        self.hash.reset()
        in_frag = False
        prospective = 0
        strict = mode in (kAbsoluteConsistency, kPointInTimeRecovery)
        while True:
            phys = self.end_of_buffer_offset - self._size()
            self.cur_phys = phys
            rt, drop, frag = self.read_physical_record()
            if rt in (kFullType, kRecyclableFullType):
                if in_frag and scratch:
                    self._report(len(scratch), "partial record without end(1)")
                self.last_record_offset = phys
                self.first_record_read = True
                return phys, frag, O.xxh3_64(frag)
            if rt in (kFirstType, kRecyclableFirstType):
                if in_frag and scratch:
                    self._report(len(scratch), "partial record without end(2)")
                    self.hash.reset()
                self.hash.update(frag)
                prospective = phys
                scratch = frag
                in_frag = True
                continue
            if rt in (kMiddleType, kRecyclableMiddleType):
                if not in_frag:
                    self._report(len(frag), "missing start of fragmented record(1)")
                else:
                    self.hash.update(frag)
                    scratch += frag
                continue
            if rt in (kLastType, kRecyclableLastType):
                if not in_frag:
                    self._report(len(frag), "missing start of fragmented record(2)")
                    continue
                self.hash.update(frag)
                self.last_record_offset = prospective
                self.first_record_read = True
                return prospective, scratch + frag, self.hash.digest()
            if rt == kSetCompressionType:
                if self.compression_type_record_read:
                    self._report(len(frag), "read multiple SetCompressionType records")
                if self.first_record_read:
                    self._report(len(frag), "SetCompressionType not the first record")
                prospective = phys
                scratch = b""
                self.last_record_offset = prospective
                # CompressionTypeRecord::DecodeFrom (util/compression.h:1716):
                # GetFixed32 consumes 4 bytes; CompressionType is an 8-bit enum
                if len(frag) < 4:
                    self._report(len(frag), "could not decode SetCompressionType record")
                    continue
                ct = frag[0]  # static_cast<CompressionType>(uint32) keeps the low byte
                if ct == kZSTD:
                    raise Unsupported("WAL compression (kZSTD)")
                if ct != 0:
                    self._report(len(frag) - 4, "could not decode SetCompressionType record")
                    continue
                self.compression_type_record_read = True  # InitCompression: no decoder
                continue
            if rt in (kUserDefinedTimestampSizeType, kRecyclableUserDefinedTimestampSizeType):
                if in_frag and scratch:
                    self._report(len(scratch), "user-defined timestamp size record "
                                 "interspersed partial record")
                prospective = phys
                scratch = b""
                self.last_record_offset = prospective
                # UserDefinedTimestampSizeRecord::DecodeFrom (util/udt_util.h:46)
                if len(frag) % 6:
                    self._report(len(frag), "could not decode user-defined timestamp size record")
                    continue
                err = None
                for k in range(0, len(frag), 6):  # UpdateRecordedTimestampSize
                    cf = int.from_bytes(frag[k:k + 4], "little")
                    ts = int.from_bytes(frag[k + 4:k + 6], "little")
                    if ts == 0:
                        err = "User-defined timestamp size record contains zero timestamp size."
                        break
                    if cf in self.recorded_ts:
                        err = ("User-defined timestamp size record contains update to "
                               "recorded column family.")
                        break
                    self.recorded_ts[cf] = ts
                if err:
                    self._report(0, err)
                continue
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


def resume_at(reader, pos, recycled=False):
    """TEST-INFRASTRUCTURE shortcut (no reference counterpart): put `reader`
    in the state ReadRecord leaves behind after returning a complete record
    whose last fragment ends at `pos` -- the 32 KiB block holding `pos` in the
    buffer, consumed up to `pos`, no fragment in progress, a first record
    read.  The next read_record starts at the physical record at `pos`, so a
    window of a large log (starting at the block boundary below `pos`) can be
    checked against the serial reader without replaying everything before
    it.  Valid only when the log before `pos` holds no control records
    (SetCompressionType, timestamp-size); `recycled` = whether the log's
    first header is a recyclable one (the reader's recycled_ flag,
    log_reader.cc:476-479)."""
    blk = pos // kBlockSize * kBlockSize
    reader.file_pos = blk
    reader.end_of_buffer_offset = blk
    reader.eof = False
    reader.read_more()
    reader.buf_lo = pos
    reader.first_record_read = True
    reader.recycled = recycled
    return reader


def read_all(log, log_number=0, mode=kPointInTimeRecovery):
    """Every logical record ReadRecord returns, in order: (record offset =
    Reader::LastRecordOffset, length, record checksum), and the reporter's
    (bytes, reason, reader position) calls."""
    r = Reader(log, log_number)
    recs = []
    while True:
        got = r.read_record(mode)
        if got is None:
            break
        off, payload, h = got
        recs.append((off, len(payload), h))
    return recs, r.reports
