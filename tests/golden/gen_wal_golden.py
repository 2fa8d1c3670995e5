#!/usr/bin/env python3
"""tests/golden/gen_wal_golden.py -- TEST INFRASTRUCTURE ONLY: WAL recovery
fixtures from the REFERENCE's own log::Reader.

The reference's db/log_reader.cc and its link closure are compiled from the
sources under /root/reference (tests/golden/refbuild.py: g++ over src.mk's
LIB_SOURCES into a throwaway archive outside the repository) and linked with
the veneer tests/golden/ref_wal_shim.cc, which feeds each log through an
in-memory FSSequentialFile (as db/log_test.cc's StringSource does) and drives
ReadRecord(&record, &scratch, mode, &record_checksum) to the end, as
DBImpl::RecoverLogFiles does (db/db_impl/db_impl_open.cc:1210).

The logs are the scenario builders of tests/walcases.py (deterministic from
their seeds; each log's SHA-256 is recorded so a test can prove it rebuilt
the same bytes).  Committed: tests/golden/wal_reader.json.gz -- per log and
WALRecoveryMode, every record (LastRecordOffset, length, record checksum),
every Reporter::Corruption(bytes, Status::ToString()) call in order, and the
reader position / EOF flag when ReadRecord returned false.

Re-run:  python tests/golden/gen_wal_golden.py   (needs /root/reference + g++)
"""
import ctypes
import gzip
import hashlib
import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, TESTS)
sys.path.insert(0, os.path.dirname(TESTS))
import refbuild  # noqa: E402
import walcases as W  # noqa: E402

OUT = os.path.join(HERE, "wal_reader.json.gz")
MODES = (0, 1, 2, 3)


def cases():
    """(family, name, recyclable, log, log_number, modes)"""
    for rec in (False, True):
        for name, log, ln in W.scenarios(rec, 23, n=300):
            yield "scenarios", name, rec, log, ln, MODES
        for name, log, ln in W.pseudo_type_scenarios(rec, 41):
            yield "pseudo", name, rec, log, ln, MODES
        for name, log, ln in W.control_scenarios(rec, 43):
            yield "control", name, rec, log, ln, MODES
        yield "zero_tail", "zero_tail", rec, W.zero_tail_log(rec), 7, MODES
    yield "old_tail", "old_tail", True, W.old_tail_log(), 8, MODES


def reader(path):
    L = ctypes.CDLL(path)
    L.ref_wal_read.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_ulonglong, ctypes.c_int,
                               ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    L.ref_wal_read.restype = ctypes.c_int

    def run(log, ln, mode):
        cap = 1 << 24
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t()
        rc = L.ref_wal_read(bytes(log), len(log), ln, mode, out, cap, ctypes.byref(n))
        assert rc == 0
        recs, reps, end = [], [], None
        for line in out.raw[:n.value].decode().splitlines():
            kind, rest = line[0], line[2:]
            if kind == "R":
                o, n_, h = rest.split(" ")
                recs.append([int(o), int(n_), h])
            elif kind == "C":
                b, text = rest.split(" ", 1)
                reps.append([int(b), text])
            else:
                p, eof = rest.split(" ")
                end = [int(p), int(eof)]
        return {"records": recs, "reports": reps, "end": end}
    return run


def main():
    tmp = tempfile.mkdtemp(prefix="forst_ref_wal_")
    try:
        so = refbuild.link_veneer([os.path.join(HERE, "ref_wal_shim.cc")],
                                  os.path.join(tmp, "libref_wal.so"))
        run = reader(so)
        out = []
        for fam, name, rec, log, ln, modes in cases():
            log = bytes(log)
            out.append({"family": fam, "name": name, "recyclable": rec, "log_number": ln,
                        "log_len": len(log), "log_sha256": hashlib.sha256(log).hexdigest(),
                        "modes": {str(m): run(log, ln, m) for m in modes}})
            print(fam, name, rec, len(log), [len(out[-1]["modes"][str(m)]["records"]) for m in modes])
        doc = {"generator": "tests/golden/gen_wal_golden.py",
               "reference": "db/log_reader.cc log::Reader::ReadRecord (compiled from "
                            "/root/reference by tests/golden/refbuild.py)",
               "cases": out}
        with gzip.open(OUT, "wt", compresslevel=9) as f:
            json.dump(doc, f, separators=(",", ":"))
        print(f"{len(out)} logs -> {OUT} ({os.path.getsize(OUT)} bytes)")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
