"""SST- and WAL-shaped synthetic batches on the device.

Blocks are packed back-to-back exactly as BlockBasedTableBuilder writes them
(payload n_i bytes, compression-type byte, LE32 checksum; offset_{i+1} =
offset_i + n_i + 5), so block starts are deliberately unaligned.  Payload
bytes are the splitmix64 stream of the config's seed (byte i of the buffer is
byte i of the stream); trailers are written by the engine's own trailer kernel
(write side) and then read back by the verify kernel (read side).
"""
import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import engine
from ._lib import check, lib

TRAILER = 5  # table/block_based/block_based_table_reader.h:75 kBlockTrailerSize

# BASELINE.json configs (seeds from SURVEY.md §8d)
SEEDS = {"C1": 0xF0E5700001, "C2": 0xF0E5700002, "C3": 0xF0E5700003,
         "C4": 0xF0E5700004, "C5": 0xF0E5700005}


def _splitmix(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def block_sizes(n, spec, seed):
    """n block payload sizes.
    spec: int            -> all equal
          tuple of ints  -> equal shares of each class, shuffled (C3)
          ("dev", b)     -> uniform in [0.9 b, b] (block_size_deviation=10, C3b)
          ("logu", lo, hi) -> log-uniform in [lo, hi] (the C5 record mix)
          ("sorted", (a, b, ..)) -> the shuffled mix sorted largest first (C3S:
                             the same blocks as C3, clustered by size)
    """
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        keys = _splitmix(np.uint64(seed ^ 0x5EED5EED5EED) + idx * np.uint64(0x9E3779B97F4A7C15))
    if isinstance(spec, int):
        return np.full(n, spec, dtype=np.uint32)
    if isinstance(spec, tuple) and spec and spec[0] == "logu":  # log-uniform [lo, hi] (C5-like)
        return log_uniform_lengths(n, int(spec[1]), int(spec[2]), seed)
    if isinstance(spec, tuple) and spec and spec[0] == "sorted":
        return np.sort(block_sizes(n, tuple(spec[1]), seed))[::-1].copy()
    if isinstance(spec, tuple) and spec and spec[0] == "dev":
        b = int(spec[1])
        lo = (b * 9) // 10
        return (lo + (keys % np.uint64(b - lo + 1))).astype(np.uint32)
    classes = np.array(spec, dtype=np.uint32)
    perm = np.argsort(keys, kind="stable")
    out = np.empty(n, dtype=np.uint32)
    out[perm] = classes[np.arange(n) % len(classes)]
    return out


@dataclass
class SstBatch:
    base: torch.Tensor      # uint8 [total]  (device)
    offsets: torch.Tensor   # int64 [n]      (device)
    sizes: torch.Tensor     # int32 [n]      (device)
    types: torch.Tensor     # uint8 [n]      (device) compression type bytes
    n: int
    total: int
    payload_bytes: int      # sum of sizes
    seed: int

    @property
    def checksummed_bytes(self):
        """bytes covered by the block checksums: payload + type byte"""
        return self.payload_bytes + self.n


def make_sst_batch(n, spec, seed, ctype=engine.ChecksumType.kCRC32c, device="cuda",
                   write_trailers=True, modifiers=None, sizes=None, stream_start=0):
    """n SST-packed blocks on the device.  stream_start = byte offset of the
    first block in a larger described batch (a rank's shard, shard.rank_slice):
    the payload bytes are then exactly that batch's bytes."""
    if sizes is None:
        sizes = block_sizes(n, spec, seed)
    sizes = np.asarray(sizes, dtype=np.uint32)
    n = len(sizes)
    offs = np.zeros(n, dtype=np.int64)
    if n > 1:
        offs[1:] = np.cumsum(sizes[:-1].astype(np.int64) + TRAILER)
    total = int(offs[-1]) + int(sizes[-1]) + TRAILER if n else 0
    alloc = max(16, (total + 255) // 256 * 256)
    base = torch.empty(alloc, dtype=torch.uint8, device=device)
    engine.fill_stream(base, stream_start, seed)
    base = base[:total] if total else base[:0]
    d_offs = torch.from_numpy(offs).to(device)
    d_sizes = torch.from_numpy(sizes.astype(np.int32)).to(device)
    types = torch.zeros(n, dtype=torch.uint8, device=device)  # kNoCompression
    b = SstBatch(base, d_offs, d_sizes, types, n, total, int(sizes.astype(np.int64).sum()), seed)
    if write_trailers and n:
        engine.block_trailer_batch(ctype, base, d_offs, d_sizes, types, modifiers)
    return b


def log_uniform_lengths(n, lo, hi, seed):
    """WAL record lengths, log-uniform in [lo, hi] (config C5)."""
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        k = _splitmix(np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15))
    u = (k >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    return np.exp(np.log(lo) + u * (np.log(hi) - np.log(lo))).astype(np.uint32)


@dataclass
class WalBatch:
    log: torch.Tensor        # uint8 [total] (device): the log image
    rec_offsets: np.ndarray  # uint64 header offsets of the physical records (host)
    rec_lengths: np.ndarray  # uint32 payload lengths
    rec_types: np.ndarray    # uint8 RecordType
    n_records: int           # logical records
    total: int
    seed: int

    @property
    def n_log_blocks(self):
        return (self.total + 32767) // 32768


def wal_layout(lengths, recyclable=False):
    """log::Writer::AddRecord's physical-record layout (forst_wal_layout).
    Returns (rec_offsets, rec_lengths, rec_types, pad_offsets, pad_lengths, total)."""
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = len(lengths)
    np_, npad, tot = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    L = lib()
    check(L.forst_wal_layout(lengths.ctypes.data, n, int(recyclable), None, None, None, 0, None,
                             None, 0, ctypes.byref(np_), ctypes.byref(npad), ctypes.byref(tot)))
    offs = np.empty(np_.value, np.uint64)
    lens = np.empty(np_.value, np.uint32)
    types = np.empty(np_.value, np.uint8)
    poffs = np.empty(max(1, npad.value), np.uint64)
    plens = np.empty(max(1, npad.value), np.uint32)
    check(L.forst_wal_layout(lengths.ctypes.data, n, int(recyclable), offs.ctypes.data,
                             lens.ctypes.data, types.ctypes.data, np_.value, poffs.ctypes.data,
                             plens.ctypes.data, npad.value, ctypes.byref(np_), ctypes.byref(npad),
                             ctypes.byref(tot)))
    return offs, lens, types, poffs[:npad.value], plens[:npad.value], tot.value


def make_wal_batch(n_records, seed, lo=32, hi=32768, recyclable=False, log_number=0,
                   device="cuda", lengths=None, block_range=None):
    """C5-shaped WAL image built on the device: logical record
    lengths log-uniform in [lo, hi], framed by log::Writer's rules
    (forst_wal_layout); payload bytes are the splitmix64 stream of `seed`,
    headers [crc:4 len:2 type:1 (lognum:4)] are written in place, block-tail
    pads zeroed and the CRCs filled by the writer-side kernel
    (forst_wal_record_crc_batch).  block_range = (b0, b1): only the 32 KiB
    log blocks [b0, b1) of that log, as their own buffer (physical records
    never straddle a block, log_writer.cc:86-102): a rank's shard of one log;
    offsets are then relative to block b0 and n_records counts the logical
    records whose first fragment lies in the range."""
    if lengths is None:
        lengths = log_uniform_lengths(n_records, lo, hi, seed)
    offs, lens, types, poffs, plens, total = wal_layout(lengths, recyclable)
    if block_range is not None:
        b0, b1 = block_range
        lo_b, hi_b = b0 * 32768, min(total, b1 * 32768)
        keep = (offs >= lo_b) & (offs < hi_b)
        offs, lens, types = offs[keep] - np.uint64(lo_b), lens[keep], types[keep]
        pk = (poffs >= lo_b) & (poffs < hi_b)
        poffs, plens = poffs[pk] - np.uint64(lo_b), plens[pk]
        total = hi_b - lo_b
        alloc = max(256, (total + 255) // 256 * 256)
        log = torch.empty(alloc, dtype=torch.uint8, device=device)
        engine.fill_stream(log, lo_b, seed)
        log = log[:total]
        n_rec = int(((types == 1) | (types == 2) | (types == 5) | (types == 6)).sum())
        return _frame_wal(log, offs, lens, types, poffs, plens, total, seed, n_rec, recyclable,
                          log_number, device)
    alloc = max(256, (total + 255) // 256 * 256)
    log = torch.empty(alloc, dtype=torch.uint8, device=device)
    engine.fill_stream(log, 0, seed)
    log = log[:total]
    return _frame_wal(log, offs, lens, types, poffs, plens, total, seed, len(lengths), recyclable,
                      log_number, device)


def _frame_wal(log, offs, lens, types, poffs, plens, total, seed, n_rec, recyclable, log_number,
               device):
    """headers, zeroed block tails and writer CRCs into a payload image"""
    d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
    hdr = [(4, (lens & 0xFF).astype(np.uint8)), (5, (lens >> 8).astype(np.uint8)), (6, types)]
    if recyclable:
        for k in range(4):
            hdr.append((7 + k, np.full(len(offs), (log_number >> (8 * k)) & 0xFF, np.uint8)))
    for k, v in hdr:
        log[d_offs + k] = torch.from_numpy(v).to(device)
    if len(poffs):  # zero-filled block tails (log_writer.cc:88-97)
        plens64 = plens.astype(np.int64)
        starts = np.repeat(poffs.astype(np.int64), plens64)
        within = np.arange(int(plens64.sum()), dtype=np.int64) - np.repeat(
            np.cumsum(plens64) - plens64, plens64)
        log[torch.from_numpy(starts + within).to(device)] = 0
    if len(offs):
        engine.wal_record_crc_batch(log, d_offs, write_in_place=True)
    return WalBatch(log, offs, lens, types, n_rec, total, seed)
