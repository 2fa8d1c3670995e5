"""Fused WAL recovery (§8f-2, forst_wal_recover_batch): the whole reader --
header walk, physical-record CRCs, fragment assembly, reports and the XXH3
record checksum -- against the serial restatement of log::Reader::ReadRecord
(oracle/wal_reader.py, db/log_reader.cc:69-531) record for record and report
for report, in all four WALRecoveryModes, on clean, corrupted, re-typed
(missing starts, partial records, unknown types), zero-filled, truncated and
recycled logs with old records.

The CPU tests run the unmodified device code on the SIMT emulator
(tests/emu); the -m gpu tests run it on the MI355X, including a C5-shaped log
of 200 000 records with scattered corruption."""
import struct

import numpy as np
import pytest

from oracle import oracle as O
from oracle import wal_reader as R

MODES = [R.kTolerateCorruptedTailRecords, R.kAbsoluteConsistency, R.kPointInTimeRecovery,
         R.kSkipAnyCorruptedRecords]
REASONS = {1: "partial record without end(1)", 2: "partial record without end(2)",
           3: "missing start of fragmented record(1)",
           4: "missing start of fragmented record(2)", 5: "error in middle of record",
           6: "checksum mismatch", 7: "bad record length", 8: "truncated header",
           9: "error reading trailing data", 10: "truncated record body"}


def reason_text(code, rtype):
    return "unknown record type %u" % rtype if code == 11 else REASONS[code]


def frame(n, seed, recyclable=False, log_number=7, hi=70000):
    rng = np.random.default_rng(seed)
    lens = (np.exp(rng.uniform(0, np.log(hi), n))).astype(np.uint32)
    lens[:4] = [0, 32761, 5, 32750]
    pay = rng.integers(0, 256, int(lens.astype(np.int64).sum()), np.uint8)
    buf, po, pl = O.wal_frame(pay, lens, recyclable=recyclable, log_number=log_number)
    return buf.copy(), po, pl


def hdr_size(buf, off):
    t = buf[off + 6]
    return 11 if (5 <= t <= 8 or t == 11) else 7


def set_type(buf, off, t, log_number):
    """re-type a physical record and rewrite its CRC (log_writer.cc:240-263)"""
    buf[off + 6] = t
    hs = hdr_size(buf, off)
    n = int(buf[off + 4]) | (int(buf[off + 5]) << 8)
    c = O.mask(O.crc32c_value(bytes(buf[off + 6:off + hs + n])))
    buf[off:off + 4] = np.frombuffer(struct.pack("<I", c), np.uint8)


def scenarios(recyclable, seed):
    """(name, log bytes, log_number) cases with every reader outcome"""
    ln = 7
    buf, po, pl = frame(600, seed, recyclable, ln)
    rng = np.random.default_rng(seed + 1)
    types = buf[po.astype(np.int64) + 6]
    out = [("clean", buf, ln)]
    b = buf.copy()  # CRC mismatches (payload flips) in a few blocks
    for k in rng.choice(len(po), 6, replace=False):
        if pl[k]:
            b[int(po[k]) + hdr_size(b, int(po[k])) + int(rng.integers(0, pl[k]))] ^= 0x10
    out.append(("crc", b, ln))
    b = buf.copy()  # re-typed fragments: missing starts, partial records, unknown types
    base = 4 if recyclable else 0
    for k in rng.choice(len(po), 12, replace=False):
        t = int(types[k]) - base
        new = {1: 4, 2: 3, 3: 1, 4: 2}[t] if t in (1, 2, 3, 4) else 1
        if k % 5 == 0:
            new = 12 - base  # unknown type (12 here; 12-4 = 8 would be a valid one)
        set_type(b, int(po[k]), new + base if new < 9 else 12, ln)
    out.append(("retype", b, ln))
    b = buf.copy()  # a zero-filled region (kZeroType + length 0: preallocated space)
    z = int(po[len(po) // 3])
    b[z:z + 300] = 0
    out.append(("zero", b, ln))
    for cut in (3, 9, 5000):  # truncated tail: header / recyclable header / body
        e = int(po[-1]) + min(cut, int(pl[-1]) + 6)
        out.append((f"trunc{cut}", buf[:e].copy(), ln))
    b = buf.copy()  # bad length in a middle block
    k = len(po) // 2
    b[int(po[k]) + 4:int(po[k]) + 6] = 0xFF
    out.append(("badlen", b, ln))
    if recyclable:
        b = buf.copy()  # a record of an older log incarnation
        o = int(po[len(po) // 2])
        b[o + 7:o + 11] = np.frombuffer(struct.pack("<I", ln + 1), np.uint8)
        set_type(b, o, int(b[o + 6]), ln)
        out.append(("old", b, ln))
        b2 = b.copy()  # ... and a corrupt tail of a recycled log
        b2[int(po[-3]) + 12] ^= 1
        out.append(("old+crc", b2, ln))
    return out


def compare(got_recs, got_reps, res, log, log_number, mode, name):
    want_recs, want_reps = R.read_all(log, log_number, mode)
    go, gl, gh, gn = (np.asarray(x) for x in got_recs)
    assert len(go) == len(want_recs), (name, mode, len(go), len(want_recs))
    assert [(int(a), int(b), int(c) & (2**64 - 1)) for a, b, c in zip(go, gl, gh)] == \
        [(o, n, h) for o, n, h in want_recs], (name, mode)
    po, pb, pr, pt = (np.asarray(x) for x in got_reps)
    got = [(int(b), reason_text(int(r), int(t)), int(o)) for o, b, r, t in zip(po, pb, pr, pt)]
    assert got == [(b, r, p) for b, r, p in want_reps], (name, mode, got[:5], want_reps[:5])


def _emu():
    import importlib.util
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu", "emu.py")
    spec = importlib.util.spec_from_file_location("forst_emu", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("recyclable", [False, True])
def test_recover_on_emulator(recyclable):
    """the first 3 log blocks (+ a partial 4th: a truncated tail) of each
    scenario, every mode on the re-typed log, PIT recovery on the others"""
    E = _emu()
    for name, log, ln in scenarios(recyclable, 11):
        if name.startswith("trunc") or name == "badlen":
            continue  # (tail / middle-block events: GPU test on the full logs)
        small = log[:3 * 32768 + 1000]
        for mode in (MODES if name == "retype" else [R.kPointInTimeRecovery]):
            recs, reps, res = E.wal_recover(small, ln, mode)
            compare(recs, reps, res, small, ln, mode, name)


@pytest.mark.gpu
@pytest.mark.parametrize("recyclable", [False, True])
def test_recover_on_gpu(recyclable):
    import torch
    from forst_amd import engine
    for name, log, ln in scenarios(recyclable, 23):
        for mode in MODES:
            rec, rep, res = engine.wal_recover_batch(torch.from_numpy(log).cuda(), ln, mode,
                                                     record_capacity=64, report_capacity=4)
            recs = [rec[k].cpu().numpy() for k in ("offset", "length", "hash", "n_fragments")]
            reps = [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")]
            compare(recs, reps, res, log, ln, mode, name)


@pytest.mark.gpu
def test_recover_c5_shape_with_corruption():
    """200 000 C5-shaped records (log-uniform 32 B-32 KiB) from the writer
    kernels, 40 payload flips: every record before / after the dropped blocks
    and every report equal the serial reader's"""
    import torch
    from forst_amd import engine, workload
    w = workload.make_wal_batch(200_000, workload.SEEDS["C5"])
    rng = np.random.default_rng(9)
    cand = np.nonzero(w.rec_lengths > 0)[0]
    victims = rng.choice(cand, 40, replace=False)
    pos = w.rec_offsets[victims].astype(np.int64) + 7 + \
        rng.integers(0, w.rec_lengths[victims].astype(np.int64))
    w.log[torch.from_numpy(pos).cuda()] ^= 0x01
    log = w.log.cpu().numpy()
    rec, rep, res = engine.wal_recover_batch(w.log, 0, R.kPointInTimeRecovery)
    recs = [rec[k].cpu().numpy() for k in ("offset", "length", "hash", "n_fragments")]
    reps = [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")]
    compare(recs, reps, res, log, 0, R.kPointInTimeRecovery, "c5")
    assert res.n_physical == len(w.rec_offsets)
