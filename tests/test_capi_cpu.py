"""CPU-side checks of the drop-in boundary (no GPU compute calls):
the C-ABI library builds for gfx950, loads, and exports every symbol that
include/forst_checksum.h declares; the host shim's pure helpers behave like
the reference's (Mask/Unmask, ChecksumModifierForContext, message format)."""
import ctypes
import os
import re
import subprocess

import pytest

import forst_amd
from forst_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(forst_amd.LIB_PATH), "run __graft_entry__.build() first"
    L = ctypes.CDLL(forst_amd.LIB_PATH)
    declared = forst_amd.exported_symbols()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", forst_amd.LIB_PATH], text=True)
    exported = set(re.findall(r" T (forst_\w+)", out))
    assert set(declared) <= exported
    # nothing else leaks into the C namespace
    assert {s for s in exported if s.startswith("forst_")} == set(declared)


def test_version_string_without_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.forst_version()


def test_code_object_targets_only_gfx950():
    # offload bundle entry ids embedded in the fat binary
    blob = open(forst_amd.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


@pytest.fixture(scope="module")
def shim_selftest(tmp_path_factory):
    """Compile tests/cpp/shim_selftest.cc (host-only parts of the C++ shim)."""
    d = tmp_path_factory.mktemp("shim")
    exe = str(d / "shim_selftest")
    src = os.path.join(ROOT, "tests", "cpp", "shim_selftest.cc")
    libdir = os.path.dirname(forst_amd.LIB_PATH)
    subprocess.check_call(["g++", "-std=c++17", "-O1", f"-I{ROOT}/include",
                           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", src, "-o", exe,
                           f"-L{libdir}", "-lforst_checksum", "-L/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{libdir}:/opt/rocm/lib"])
    return exe


def test_host_shim_pure_helpers(shim_selftest):
    out = subprocess.check_output([shim_selftest, "pure"], text=True)
    assert "PASS" in out, out


@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_layout_matches_writer_framing(recyclable):
    """forst_wal_layout (host utility, no GPU call) reproduces log::Writer's
    fragmentation (db/log_writer.cc:65-160) exactly as the oracle frames it:
    physical-record offsets, lengths, types, zero-filled block tails."""
    import numpy as np
    from forst_amd import workload
    from oracle import oracle as O
    hs = 11 if recyclable else 7
    rng = np.random.default_rng(8)
    lens = workload.log_uniform_lengths(3000, 32, 32768, 0xF0E5700005)
    lens[:6] = [0, 1, 7, 32761, 32762, 70000]
    # from a block start, each of these leaves a 1..hs-1 byte block tail -> padding
    tail = (32768 - hs - rng.integers(1, hs, 200)).astype(np.uint32)
    lens = np.concatenate([tail, lens, np.zeros(5, np.uint32), [200000]]).astype(np.uint32)
    offs, l, t, po, pl, tot = workload.wal_layout(lens, recyclable)
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, oo, ol = O.wal_frame(payload, lens, recyclable=recyclable, log_number=7)
    assert tot == len(buf)
    assert (offs == oo).all() and (l == ol).all()
    assert (t == buf[offs.astype(np.int64) + 6]).all()
    assert len(po) >= 100
    for o, n in zip(po, pl):
        assert 0 < n < hs and (int(o) + int(n)) % 32768 == 0
        assert not buf[int(o):int(o) + int(n)].any()
    # every byte is a header, a payload byte or a pad byte
    assert int(l.astype(np.int64).sum()) + hs * len(offs) + int(pl.astype(np.int64).sum()) == tot
    # no fragment straddles a log block
    assert ((offs % 32768) + hs + l <= 32768).all()


@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_layout_at_continues_a_writer(recyclable):
    """forst_wal_layout_at frames a write group from the writer's current
    block offset (log::Writer::block_offset_): the log framed in pieces --
    every split point, offsets shifted by the bytes already written -- is the
    log framed at once, and the end block offset is the next piece's start"""
    import numpy as np
    from forst_amd import workload
    L = _lib.lib()
    rng = np.random.default_rng(4)
    lens = np.concatenate([workload.log_uniform_lengths(400, 1, 70000, 0xF0E57000AA),
                           (32768 - 11 - rng.integers(0, 12, 40)).astype(np.uint32),
                           np.zeros(3, np.uint32)]).astype(np.uint32)
    rng.shuffle(lens)
    whole, wl, wt, _, _, wtot = workload.wal_layout(lens, recyclable)

    def piece(ls, bo):
        ls = np.ascontiguousarray(ls, np.uint32)
        cap = 4 * len(ls) + 8
        o = np.zeros(cap, np.uint64)
        ln = np.zeros(cap, np.uint32)
        t = np.zeros(cap, np.uint8)
        npad, nph, tot, end = (ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(),
                               ctypes.c_uint32())
        _lib.check(L.forst_wal_layout_at(ls.ctypes.data, len(ls), int(recyclable), bo,
                                         o.ctypes.data, ln.ctypes.data, t.ctypes.data, cap,
                                         None, None, 0, ctypes.byref(nph), ctypes.byref(npad),
                                         ctypes.byref(tot), ctypes.byref(end)))
        k = nph.value
        return o[:k], ln[:k], t[:k], tot.value, end.value

    cuts = np.unique(np.concatenate([[0, len(lens)], rng.integers(0, len(lens), 25)]))
    pos, bo = 0, 0
    got_o, got_l, got_t = [], [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        o, ln, t, tot, end = piece(lens[a:b], bo)
        got_o.append(o + np.uint64(pos))
        got_l.append(ln)
        got_t.append(t)
        pos += tot
        assert end % 32768 == pos % 32768
        bo = end
    assert pos == wtot
    assert (np.concatenate(got_o) == whole).all()
    assert (np.concatenate(got_l) == wl).all() and (np.concatenate(got_t) == wt).all()
    # block_offset = 0 is forst_wal_layout
    o, ln, t, tot, end = piece(lens, 0)
    assert (o == whole).all() and tot == wtot
    with pytest.raises(Exception):
        piece(lens[:3], 32769)


def test_wal_layout_capacity_errors():
    import numpy as np
    from forst_amd import ForstError
    L = _lib.lib()
    lens = np.array([40000, 5], np.uint32)
    offs = np.zeros(1, np.uint64)
    n = ctypes.c_uint64()
    rc = L.forst_wal_layout(lens.ctypes.data, 2, 0, offs.ctypes.data, None, None, 1, None, None,
                            0, ctypes.byref(n), None, None)
    assert rc != 0 and n.value == 3
    with pytest.raises(ForstError):
        _lib.check(L.forst_wal_layout(None, 2, 0, None, None, None, 0, None, None, 0, None, None,
                                      None))


def test_crc32c_combine_host_matches_reference_tests():
    """forst_crc32c_combine == crc32c::Crc32cCombine: util/crc32c_test.cc:128-170
    cases (basic, order matters, full cover over 0..4095-byte suffixes, big
    size) against the oracle's Extend."""
    import numpy as np
    from forst_amd import engine
    from oracle import oracle as O
    a, b = O.crc32c_value(b"hello "), O.crc32c_value(b"world")
    assert engine.crc32c_combine(a, b, 5) == O.crc32c_value(b"hello world")
    assert engine.crc32c_combine(b, a, 6) != O.crc32c_value(b"hello world")
    rng = np.random.default_rng(3)
    s1 = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    c1 = O.crc32c_value(s1)
    for n in list(range(0, 300)) + [1023, 1024, 4095, 65537]:
        s2 = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert engine.crc32c_combine(c1, O.crc32c_value(s2), n) == O.crc32c_extend(c1, s2)
    s2 = rng.integers(0, 256, 16 * 1024 * 1024 - 1, dtype=np.uint8).tobytes()
    assert engine.crc32c_combine(c1, O.crc32c_value(s2), len(s2)) == O.crc32c_extend(c1, s2)
    for n in (1 << 33, (1 << 40) + 7, (1 << 63) + 5):  # shift powers beyond memory sizes
        assert engine.crc32c_combine(0, 0, n) == 0
        assert engine.crc32c_combine(c1, 0, n) == O.crc32c_combine(c1, 0, n)


def test_sst_verify_files_argument_errors():
    """forst_sst_verify_files rejects missing arrays before any HIP call, and
    an empty file set is a no-op (no GPU needed for either)."""
    L = _lib.lib()
    n = 2
    out = (ctypes.c_char * 4096)()
    assert L.forst_sst_verify_files(None, None, None, None, 0, None, 0, out, None) == 0
    sizes = (ctypes.c_uint64 * n)(100, 100)
    offs = (ctypes.c_uint64 * n)(0, 256)
    ptrs = (ctypes.c_void_p * n)(None, None)
    assert L.forst_sst_verify_files(None, sizes, offs, ctypes.c_void_p(1), 512, None, n,
                                    out, None) == -1
    assert L.forst_sst_verify_files(ptrs, sizes, offs, None, 512, None, n, out, None) == -1
    assert L.forst_sst_verify_files(ptrs, sizes, offs, ctypes.c_void_p(1), 512, None, n,
                                    None, None) == -1
    # a null host file pointer inside the array
    assert L.forst_sst_verify_files(ptrs, sizes, offs, ctypes.c_void_p(1), 512, None, n,
                                    out, None) == -1
