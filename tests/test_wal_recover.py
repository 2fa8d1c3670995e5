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
