"""WAL logs whose multi-fragment records cross log-block boundaries at chosen
places -- the cases the fragment-aware XXH3 (forst_amd/csrc/wal_hash.h,
xxh3.hip xxh3_frag_kernel) maps logical offsets for.

A record whose header lands at block offset o has its first fragment end at
the block end, so its first boundary is l0 = 32768 - o - hs logical bytes in
(log_writer.cc:65-160).  frag_edge_log() places each target record at the
offset giving a chosen l0 by writing a pad record in front of it, and covers:
the boundary at every byte of a 16-byte lane slot and of a 64-byte stripe, at
1 KiB window edges, in the last stripe, the last fragment at 63 / 64 / 65
bytes, records of 241..300 bytes across a boundary, an empty first fragment
(leftover exactly hs), three- and four-fragment records, and short records
(<= 240 bytes) across a boundary (gathered)."""
import numpy as np

from oracle import oracle as O

BLOCK = 32768


def _advance(o, L, hs):
    """block offset after log::Writer::AddRecord of L bytes at offset o"""
    left = L
    first = True
    while first or left > 0:
        first = False
        if BLOCK - o < hs:
            o = 0
        avail = BLOCK - o - hs
        frag = min(left, avail)
        o += hs + frag
        left -= frag
    return o


def _pad_to(o, target, hs):
    """a record length that moves the writer from block offset o to target"""
    if BLOCK - o < hs:
        o = 0
    if target >= o + hs:
        return target - o - hs
    return (BLOCK - o - hs) + (target - hs)  # ends target bytes into the next block


def cases(rng):
    """(l0, L) pairs: first boundary l0 logical bytes in, record length L"""
    out = []
    for c in range(16):  # boundary at every byte of a lane slot, stripe positions
        for k in (0, 1, 5):
            l0 = 1024 * k + 16 * int(rng.integers(0, 64)) + c
            if l0 == 0:
                l0 = 16
            out.append((l0, l0 + int(rng.integers(64, 4000))))
    for l0 in (1024, 2048, 1023, 1025, 64, 63, 65, 1, 2, 3):  # window / stripe edges
        out.append((l0, l0 + 700))
    for last in (63, 64, 65, 66, 100):  # last fragment length
        out.append((3000, 3000 + last))
        out.append((5, 5 + last + 200))
    for L in range(241, 301, 3):  # just above the short-input limit
        out.append((int(rng.integers(1, L - 63)), L))
    for L in (100, 200, 240, 16):  # short records across a boundary (gathered)
        out.append((int(rng.integers(1, L)), L))
    for l0 in (7, 500, 1000, 30000):  # three and four fragments
        out.append((l0, l0 + 32761 + int(rng.integers(64, 30000))))
        out.append((l0, l0 + 2 * 32761 + int(rng.integers(64, 3000))))
    out.append((0, 5000))  # empty first fragment (header exactly at block end - hs)
    out.append((0, 32761 + 100))
    rng.shuffle(out)
    return out


def frag_edge_log(recyclable=False, seed=5, log_number=9, repeat=1):
    """(log, header offsets, payload, logical lengths, [(record index, l0)])"""
    rng = np.random.default_rng(seed)
    hs = 11 if recyclable else 7
    lens, targets = [], []
    o = 0
    for _ in range(repeat):
        for l0, L in cases(rng):
            want = BLOCK - hs - l0
            pad = _pad_to(o, want, hs)
            lens.append(pad)
            o = _advance(o, pad, hs)
            targets.append((len(lens), l0))
            lens.append(L)
            o = _advance(o, L, hs)
            if rng.integers(0, 3) == 0:  # a small full record between cases
                n = int(rng.integers(0, 300))
                lens.append(n)
                o = _advance(o, n, hs)
    lens = np.array(lens, np.uint32)
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), np.uint8)
    buf, po, pl = O.wal_frame(payload, lens, recyclable=recyclable, log_number=log_number)
    return buf, po, payload, lens, targets


def first_fragment_offsets(buf, po):
    """header offset of each logical record's first fragment (Full / First)"""
    t = buf[po.astype(np.int64) + 6]
    t = np.where((t >= 5) & (t <= 8), t - 4, t)
    return po[(t == 1) | (t == 2)]


def expected_hashes(payload, lens):
    starts = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    return np.array([O.xxh3_64(payload[starts[j]:starts[j + 1]].tobytes())
                     for j in range(len(lens))], np.uint64)
