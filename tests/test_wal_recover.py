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
import numpy as np
import pytest

import walcases as W
from oracle import wal_reader as R
from test_wal_golden import reason_text

MODES = [R.kTolerateCorruptedTailRecords, R.kAbsoluteConsistency, R.kPointInTimeRecovery,
         R.kSkipAnyCorruptedRecords]
scenarios = W.scenarios


def compare(got_recs, got_reps, res, log, log_number, mode, name):
    want_recs, want_reps = R.read_all(log, log_number, mode)
    go, gl, gh, gn = (np.asarray(x) for x in got_recs)
    assert len(go) == len(want_recs), (name, mode, len(go), len(want_recs))
    assert [(int(a), int(b), int(c) & (2**64 - 1)) for a, b, c in zip(go, gl, gh)] == \
        [(o, n, h) for o, n, h in want_recs], (name, mode)
    po, pb, pr, pt = (np.asarray(x) for x in got_reps)
    got = [(int(b), reason_text(int(r), int(t) & 0xFFFFFFFF), int(o))
           for o, b, r, t in zip(po, pb, pr, pt)]
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


def _short_lengths_log(recyclable, reps, seed):
    """Full records of every short length 0..240 (their CRC and XXH3 in
    wal_short_rows_kernel, a record per 16-lane row), each length at
    every payload alignment mod 4 over the repeats, between long records;
    one record's type byte flipped (a CRC mismatch on the raw path)"""
    rng = np.random.default_rng(seed)
    lens = []
    for r in range(reps):
        sh = np.arange(241, dtype=np.uint32)
        rng.shuffle(sh)
        lens += list(sh[:120]) + [int(rng.integers(3000, 9000))] + list(sh[120:]) + [r % 7 + 1]
    lens += [20000, 600]
    log, po, pl = W.frame_lens(lens, seed, recyclable=recyclable)
    short = [int(o) for o, l_ in zip(po, pl) if 0 < l_ <= 240 and (int(o) % 32768) < 32000]
    log[short[len(short) // 2] + 6] ^= 0x01
    return log


def test_recover_short_lengths_on_emulator():
    """(legacy headers; the GPU test below also runs recyclable ones)"""
    E = _emu()
    recyclable = False
    log = _short_lengths_log(recyclable, 1, 3)
    recs, reps, res = E.wal_recover(log, 7, R.kPointInTimeRecovery)
    compare(recs, reps, res, log, 7, R.kPointInTimeRecovery, "short")


@pytest.mark.gpu
@pytest.mark.parametrize("recyclable", [False, True])
def test_recover_short_lengths_on_gpu(recyclable):
    """the same on the GPU at scale (300 repeats): the Full records of
    <= 240 B are short candidates (head 2) and take wal_short_rows_kernel;
    they are not on the raw list, so this log does not reach the kRawFirst
    branch -- test_recover_many_raw_records_on_gpu covers that"""
    import torch
    from forst_amd import engine
    log = _short_lengths_log(recyclable, 300, 4)
    for mode in MODES:
        rec, rep, res = engine.wal_recover_batch(torch.from_numpy(log).cuda(), 7, mode)
        recs = [rec[k].cpu().numpy() for k in ("offset", "length", "hash", "n_fragments")]
        reps = [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")]
        compare(recs, reps, res, log, 7, mode, "short")


@pytest.mark.gpu
def test_recover_many_raw_records_on_gpu():
    """a raw list over 64 K entries (records no candidate covers: here
    re-typed to an unknown type with a valid CRC), so the raw path runs
    ahead of the fused kernel on its stream; a few of them with a wrong CRC;
    every record and report against the serial reader, every mode"""
    import torch
    from forst_amd import engine
    rng = np.random.default_rng(29)
    lens = rng.integers(20, 300, 150_000).astype(np.uint32)
    log, po, pl = W.frame_lens(lens, 6)
    for off in po[1::2]:
        W.set_type(log, int(off), 30)
    for off in rng.choice(po[1::2], 5, replace=False):
        log[int(off) + 7] ^= 0x04  # a payload byte of a re-typed record: a CRC mismatch
    for mode in MODES:
        rec, rep, res = engine.wal_recover_batch(torch.from_numpy(log).cuda(), 7, mode)
        recs = [rec[k].cpu().numpy() for k in ("offset", "length", "hash", "n_fragments")]
        reps = [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")]
        compare(recs, reps, res, log, 7, mode, "raw")


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


@pytest.mark.gpu
def test_recover_dense_tiny_records():
    """20 log blocks of records of 0-2 bytes (about 4 600 per block, so the
    first workgroup of the walk holds far more items than rw_fill's LDS stage:
    its direct-store path), then ordinary records, with a few flips: every
    record and report equal the serial reader's in every mode"""
    import time

    import torch
    from forst_amd import engine
    rng = np.random.default_rng(17)
    tiny = rng.integers(0, 3, 20 * 32768 // 9).astype(np.uint32)
    big = (np.exp(rng.uniform(np.log(32), np.log(20000), 400))).astype(np.uint32)
    log, po, pl = W.frame_lens(np.concatenate([tiny, big]), 5)
    for off in rng.choice(po[len(tiny) // 2:], 6, replace=False):
        log[int(off) + 6] ^= 0x10  # the type byte (in the CRC'd range): a checksum mismatch
    t0 = time.perf_counter()
    for mode in MODES:
        rec, rep, res = engine.wal_recover_batch(torch.from_numpy(log).cuda(), 7, mode)
        recs = [rec[k].cpu().numpy() for k in ("offset", "length", "hash", "n_fragments")]
        reps = [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")]
        compare(recs, reps, res, log, 7, mode, "dense")
    assert time.perf_counter() - t0 < 120



def clean_expectation(rec_offsets, rec_lengths, rec_types, hashes, hs=7):
    """the records a clean, writer-laid-out log recovers to: (offset, length,
    hash, n_fragments) per logical record, and the first-fragment indices
    (hs: the header size, 7 or 11 for recyclable headers)"""
    nphys = len(rec_offsets)
    starts = np.nonzero((rec_types == 1) | (rec_types == 2) | (rec_types == 5) |
                        (rec_types == 6))[0]
    ends = np.concatenate([starts[1:], [nphys]])
    cum = np.concatenate([[0], np.cumsum(rec_lengths.astype(np.int64))])
    # Reader::LastRecordOffset is where the reader stood when it went for the
    # record's first fragment: for a header at a log-block start that is the
    # end of the previous physical record, in front of the writer's zero pad
    # (log_reader.cc:89-92 computes physical_record_offset before
    # ReadPhysicalRecord skips the < 7-byte block tail)
    offs = rec_offsets.astype(np.int64)
    hdr = offs[starts]
    prev = np.maximum(starts - 1, 0)
    prev_end = np.where(starts > 0, offs[prev] + hs + rec_lengths[prev].astype(np.int64), 0)
    # -- a tail of 7..10 bytes (recyclable logs pad < 11) is first read as a
    # zero-type header (kBadRecord, log_reader.cc:509-518) that consumes it, so
    # there the offset is the block start again
    reported = np.where((hdr % 32768 == 0) & (hdr - prev_end < 7), prev_end, hdr)
    return {"offset": reported,
            "length": cum[ends] - cum[starts],
            "hash": np.asarray(hashes).view(np.int64),
            "n_fragments": (ends - starts).astype(np.int32)}, starts, ends


def windowed_expectation(read_window, exp, starts, victims, vblocks, total, mode, log_number=0,
                         recycled=False):
    """What the serial reader returns on a writer-laid-out log after one
    payload flip in each of the log blocks `vblocks` (physical records
    `victims`, >= 8 blocks apart): the clean records outside the damaged
    windows, and inside each window what oracle/wal_reader.py returns when
    replayed from the start of the logical record holding the flip
    (wal_reader.resume_at) to four blocks past it, cut at the first record
    start at least two blocks past the flip (where the reader's state is
    clean again).  On a recycled log in kTolerateCorruptedTailRecords the
    first mismatch ends the log (log_reader.cc:291-296 / :265 of the
    restatement): then only the records in front of it remain.  Returns
    (offsets, lengths, hashes as uint64, reports, outside mask)."""
    n = len(exp["offset"])
    windows = []
    for i, v in zip(victims, vblocks):
        li = int(np.searchsorted(starts, i, side="right")) - 1
        o_start = int(exp["offset"][li])
        j = int(np.searchsorted(exp["offset"], (int(v) + 2) * 32768, side="left"))
        cutoff = int(exp["offset"][j]) if j < n else total
        windows.append((o_start, cutoff, min(total, (int(v) + 4) * 32768)))
    assert all(windows[k][1] <= windows[k + 1][0] for k in range(len(windows) - 1))
    stop_first = recycled and mode == R.kTolerateCorruptedTailRecords
    outside = np.ones(n, bool)
    if stop_first:
        windows = windows[:1]
        outside[exp["offset"] >= windows[0][0]] = False
    for o_start, cutoff, _ in windows:
        outside[(exp["offset"] >= o_start) & (exp["offset"] < cutoff)] = False
    win_recs, want_reps = [], []
    for o_start, cutoff, end in windows:
        b0 = o_start // 32768 * 32768
        r = R.resume_at(R.Reader(read_window(b0, end), log_number), o_start - b0,
                        recycled=recycled)
        while True:
            got = r.read_record(mode)
            if got is None:
                break
            off, payload, h = got
            if off + b0 < cutoff:
                win_recs.append((off + b0, len(payload), h))
        want_reps += [(nb_, why, p + b0) for nb_, why, p in r.reports if p + b0 < cutoff]
    wo = np.concatenate([exp["offset"][outside], np.array([t[0] for t in win_recs], np.int64)])
    wl = np.concatenate([exp["length"][outside], np.array([t[1] for t in win_recs], np.int64)])
    wh = np.concatenate([exp["hash"][outside].view(np.uint64),
                         np.array([t[2] for t in win_recs], np.uint64)])
    order = np.argsort(wo, kind="stable")
    return wo[order], wl[order], wh[order], want_reps, outside


def pick_flips(rng, rec_offsets, rec_lengths, n_log_blocks, k, hs=7):
    """k log blocks >= 8 apart, a physical record with payload in each, and
    one payload byte of it: (victims, blocks, byte positions)"""
    vblocks = np.sort(rng.choice(np.arange(4, n_log_blocks - 8, 8), k, replace=False))
    blk_of = (rec_offsets // 32768).astype(np.int64)
    victims = np.array([int(rng.choice(np.nonzero((blk_of == v) & (rec_lengths > 0))[0]))
                        for v in vblocks])
    pos = rec_offsets[victims].astype(np.int64) + hs + \
        rng.integers(0, rec_lengths[victims].astype(np.int64))
    return victims, vblocks, pos


@pytest.mark.parametrize("recyclable", [False, True])
@pytest.mark.parametrize("mode", MODES)
def test_windowed_expectation_equals_full_replay(mode, recyclable):
    """the composition the full-size GPU test relies on, checked on a log the
    serial reader replays whole: clean records + per-flip windows replayed
    from resume_at == read_all over the entire corrupted log (legacy and
    recyclable headers, every WALRecoveryMode); the clean log replays to the
    clean expectation with no report"""
    from oracle import oracle as O
    rng = np.random.default_rng(8)
    ln = 0x5EED if recyclable else 0
    hs = 11 if recyclable else 7
    lens = (np.exp(rng.uniform(np.log(32), np.log(32768), 2500))).astype(np.uint32)
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), np.uint8)
    log, po, pl = O.wal_frame(payload, lens, recyclable=recyclable, log_number=ln)
    types = np.array([log[int(o) + 6] for o in po], np.uint8)
    starts0 = np.nonzero((types == 1) | (types == 2) | (types == 5) | (types == 6))[0]
    hashes = O.wal_record_xxh3_batch(log, po, pl, starts0, hs=hs)
    cuml = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    assert all(int(hashes[j]) == O.xxh3_64(payload[cuml[j]:cuml[j + 1]].tobytes())
               for j in range(0, len(lens), 97))
    exp, starts, _ = clean_expectation(po.astype(np.uint64), pl, types, hashes, hs)
    recs, want_reps = R.read_all(log, ln, mode)
    assert want_reps == [] and recs == [(int(a), int(b), int(c) & (2**64 - 1)) for a, b, c in
                                        zip(exp["offset"], exp["length"], exp["hash"])]
    nblk = (len(log) + 32767) // 32768
    victims, vblocks, pos = pick_flips(rng, po.astype(np.uint64), pl, nblk, 6, hs)
    bad = log.copy()
    bad[pos] ^= 1
    wo, wl, wh, reps, _ = windowed_expectation(lambda a, b: bad[a:b], exp, starts, victims,
                                               vblocks, len(bad), mode, ln, recyclable)
    recs, want_reps = R.read_all(bad, ln, mode)
    assert [(int(a), int(b), int(c)) for a, b, c in zip(wo, wl, wh)] == recs
    assert reps == want_reps


@pytest.mark.gpu
@pytest.mark.parametrize("recyclable", [False, True])
def test_full_size_c5_recovery(recyclable):
    """f2 at the bench's size (C5: 10 M logical records, ~44 GiB log, the log
    bench.py times; and the same records with recyclable 11-byte headers, as
    recycle_log_file_num > 0 writes them, options.h:806, log_format.h:52).
    Clean log, all four WALRecoveryModes (options.h:1192): every record's
    (offset, length, XXH3, fragment count) equals the writer's layout and the
    threaded oracle's XXH3 of EVERY record over a host copy of the log.  Then
    one payload byte flipped in each of 48 log blocks (>= 8 blocks apart),
    all four modes again: every record and every report equals the serial
    reader's (oracle/wal_reader.py, db/log_reader.cc:69-531) -- around each
    flip the reader is replayed from the start of the logical record holding
    it to past the recovery point, elsewhere the clean expectation holds (on
    the recycled log in kTolerateCorruptedTailRecords the first mismatch ends
    the log)."""
    import torch
    from forst_amd import engine, workload
    from oracle import oracle as O
    n = 10_000_000
    ln = 0x5EED if recyclable else 0
    hs = 11 if recyclable else 7
    w = workload.make_wal_batch(n, workload.SEEDS["C5"], recyclable=recyclable, log_number=ln)
    DEV = w.log.device
    nphys = len(w.rec_offsets)
    logh = w.log[:w.total].cpu().numpy()
    rt = w.rec_types
    starts0 = np.nonzero((rt == 1) | (rt == 2) | (rt == 5) | (rt == 6))[0]
    hashes = O.wal_record_xxh3_batch(logh, w.rec_offsets, w.rec_lengths, starts0, hs=hs,
                                     nthreads=O.host_threads())
    exp, starts, ends = clean_expectation(w.rec_offsets, w.rec_lengths, rt, hashes, hs)
    assert len(starts) == n
    keys = ("offset", "length", "hash", "n_fragments")

    def recover(mode):
        rec, rep, res = engine.wal_recover_batch(w.log, ln, mode, record_capacity=n + 1024)
        assert res.n_physical == nphys
        return ({k: rec[k].cpu().numpy() for k in keys},
                [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")], res)

    for mode in MODES:
        got, _, res = recover(mode)
        assert res.n_records == n and res.n_reports == 0, (mode, res.n_records, res.n_reports)
        for k in keys:
            assert (got[k] == exp[k]).all(), (mode, k)

    # ---- 48 flipped payload bytes, one per chosen log block ----------------
    rng = np.random.default_rng(3)
    victims, vblocks, pos = pick_flips(rng, w.rec_offsets, w.rec_lengths, w.n_log_blocks, 48, hs)
    w.log[torch.from_numpy(pos).to(DEV)] ^= 0x01
    logh[pos] ^= 0x01
    for mode in MODES:
        wo, wl, wh, want_reps, outside = windowed_expectation(
            lambda a, b: logh[a:b], exp, starts, victims, vblocks, w.total, mode, ln, recyclable)
        got, reps, res = recover(mode)
        assert len(got["offset"]) == len(wo), (mode, len(got["offset"]), len(wo))
        assert np.array_equal(got["offset"], wo), mode
        assert np.array_equal(got["length"], wl), mode
        assert np.array_equal(got["hash"].view(np.uint64), wh), mode
        # outside the windows the fragment counts are the clean layout's
        sel = np.isin(got["offset"], exp["offset"][outside])
        assert (got["n_fragments"][sel] == exp["n_fragments"][outside]).all()
        po, pb, pr, pt = reps
        gr = [(int(b), reason_text(int(r_), int(t) & 0xFFFFFFFF), int(o))
              for o, b, r_, t in zip(po, pb, pr, pt)]
        assert gr == want_reps, (mode, gr[:4], want_reps[:4])
        n_mis = sum(1 for g in gr if g[1] == "checksum mismatch")
        assert n_mis == (0 if recyclable and mode == R.kTolerateCorruptedTailRecords
                         else len(victims)), mode


@pytest.mark.parametrize("recyclable", [False, True])
def test_long_control_runs_on_emulator(recyclable):
    """runs of 200 control records (beyond rw_live_kernel's walk-back cap:
    the linear liveness fallback) inside a fragmented record, after an
    unfinished First and between Full records, every mode"""
    E = _emu()
    for name, log, ln in W.long_control_runs(recyclable):
        for mode in MODES:
            recs, reps, res = E.wal_recover(log, ln, mode)
            compare(recs, reps, res, log, ln, mode, name)


@pytest.mark.gpu
@pytest.mark.parametrize("recyclable", [False, True])
def test_long_control_runs_on_gpu(recyclable):
    import torch
    from forst_amd import engine
    for name, log, ln in W.long_control_runs(recyclable):
        for mode in MODES:
            rec, rep, res = engine.wal_recover_batch(torch.from_numpy(log).cuda(), ln, mode)
            recs = [rec[k].cpu().numpy() for k in ("offset", "length", "hash", "n_fragments")]
            reps = [rep[k].cpu().numpy() for k in ("offset", "bytes", "reason", "type")]
            compare(recs, reps, res, log, ln, mode, name)
