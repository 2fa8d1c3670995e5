"""WAL recovery pinned to the REFERENCE's own log::Reader.

tests/golden/wal_reader.json.gz holds the transcripts of the reference's
compiled log::Reader::ReadRecord (db/log_reader.cc:69-320, with the record
checksum) over the scenario logs of tests/walcases.py in all four
WALRecoveryModes (tests/golden/gen_wal_golden.py).  The CPU test checks the
oracle restatement (oracle/wal_reader.py) against them; the -m gpu test checks
forst_wal_recover_batch against them directly, record for record and report
for report (Status text included)."""
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

import walcases as W
from oracle import wal_reader as R

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "wal_reader.json.gz")

REASONS = {1: "partial record without end(1)", 2: "partial record without end(2)",
           3: "missing start of fragmented record(1)",
           4: "missing start of fragmented record(2)", 5: "error in middle of record",
           6: "checksum mismatch", 7: "bad record length", 8: "truncated header",
           9: "error reading trailing data", 10: "truncated record body",
           12: "read multiple SetCompressionType records",
           13: "SetCompressionType not the first record",
           14: "could not decode SetCompressionType record",
           15: "user-defined timestamp size record interspersed partial record",
           16: "could not decode user-defined timestamp size record",
           17: "User-defined timestamp size record contains zero timestamp size.",
           18: "User-defined timestamp size record contains update to recorded column family."}


def reason_text(code, rtype):
    return "unknown record type %u" % rtype if code == 11 else REASONS[code]


def load():
    with gzip.open(FIXTURE, "rt") as f:
        return json.load(f)["cases"]


def build_logs():
    """the fixture's logs, rebuilt from tests/walcases.py (same generator
    calls as tests/golden/gen_wal_golden.py), keyed (family, name, recyclable)"""
    logs = {}
    for rec in (False, True):
        for name, log, _ in W.scenarios(rec, 23, n=300):
            logs[("scenarios", name, rec)] = log
        for name, log, _ in W.pseudo_type_scenarios(rec, 41):
            logs[("pseudo", name, rec)] = log
        for name, log, _ in W.control_scenarios(rec, 43):
            logs[("control", name, rec)] = log
        logs[("zero_tail", "zero_tail", rec)] = W.zero_tail_log(rec)
    logs[("old_tail", "old_tail", True)] = W.old_tail_log()
    return logs


@pytest.fixture(scope="module")
def golden():
    cases = load()
    logs = build_logs()
    out = []
    for c in cases:
        log = np.ascontiguousarray(logs[(c["family"], c["name"], c["recyclable"])])
        assert hashlib.sha256(log.tobytes()).hexdigest() == c["log_sha256"], c["name"]
        out.append((c, log))
    return out


def want(c, mode):
    m = c["modes"][str(mode)]
    recs = [(o, n, int(h, 16)) for o, n, h in m["records"]]
    reps = [(b, t) for b, t in m["reports"]]
    return recs, reps


def test_fixture_covers_the_reader_outcomes(golden):
    """the transcripts exercise every report text the reader can produce"""
    texts = set()
    for c, _ in golden:
        for m in c["modes"].values():
            texts.update(t.split(": ", 1)[1] for _, t in m["reports"])
    for r in REASONS.values():
        assert r in texts, r
    for t in (18, 127, 4294967168, 4294967295):  # type bytes 0x80 / 0xFF sign-extend
        assert "unknown record type %u" % t in texts


def test_oracle_reader_matches_reference(golden):
    for c, log in golden:
        for mode in range(4):
            recs, reps = R.read_all(log.tobytes(), c["log_number"], mode)
            wr, wp = want(c, mode)
            assert recs == wr, (c["family"], c["name"], c["recyclable"], mode)
            assert [(b, "Corruption: " + t) for b, t, _ in reps] == wp, \
                (c["family"], c["name"], c["recyclable"], mode)


@pytest.mark.gpu
def test_gpu_recovery_matches_reference(golden):
    import torch
    from forst_amd import engine
    for c, log in golden:
        dev = torch.from_numpy(log).cuda()
        for mode in range(4):
            wr, wp = want(c, mode)
            rec, rep, res = engine.wal_recover_batch(dev, c["log_number"], mode,
                                                     record_capacity=len(wr) + 8,
                                                     report_capacity=len(wp) + 8)
            key = (c["family"], c["name"], c["recyclable"], mode)
            assert not res.unsupported, key
            got = list(zip(rec["offset"].cpu().tolist(), rec["length"].cpu().tolist(),
                           [h & (2**64 - 1) for h in rec["hash"].cpu().tolist()]))
            assert got == wr, key
            gp = [(b, "Corruption: " + reason_text(r, t & 0xFFFFFFFF)) for b, r, t in
                  zip(rep["bytes"].cpu().tolist(), rep["reason"].cpu().tolist(),
                      rep["type"].cpu().tolist())]
            assert gp == wp, key


EMU_CASES = [("scenarios", "crc", False), ("pseudo", "mixed", True), ("pseudo", "partials", False),
             ("pseudo", "type16eof", True), ("control", "ctl_frag", False),
             ("control", "ctl_frag", True), ("control", "ctl_ts", True),
             ("control", "ctl_comp", False)]


def test_emulated_recovery_matches_reference(golden):
    """the unmodified device code on the SIMT emulator (tests/emu), on the
    fixtures that exercise the stale record checksum, pseudo types, partial
    records and control records; PIT recovery (all reports)"""
    import importlib.util
    p = os.path.join(HERE, "emu", "emu.py")
    spec = importlib.util.spec_from_file_location("forst_emu", p)
    E = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(E)
    by_key = {(c["family"], c["name"], c["recyclable"]): (c, log) for c, log in golden}
    for key in EMU_CASES:
        c, log = by_key[key]
        (ro, rl, rh, _), (_, pb, pr, pt), res = E.wal_recover(log, c["log_number"], 2)
        wr, wp = want(c, 2)
        assert [(int(a), int(b), int(h)) for a, b, h in zip(ro, rl, rh)] == wr, key
        assert [(int(b), "Corruption: " + reason_text(int(r), int(t) & 0xFFFFFFFF))
                for b, r, t in zip(pb, pr, pt)] == wp, key
