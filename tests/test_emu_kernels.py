"""The HIP kernel sources, compiled unmodified against the CPU SIMT emulator
(tests/emu), vs the oracle on the golden vectors and edge layouts.  This checks
kernel lane/index logic on the CPU; the real parity gate is
tests/test_gpu_parity.py on the MI355X."""
import os
import shutil
import struct
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "emu"))

if shutil.which("/opt/rocm/llvm/bin/clang++") is None:
    pytest.skip("needs ROCm clang++ to build the emulator", allow_module_level=True)

import emu  # noqa: E402

from oracle import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def golden_arrays(ref_vectors):
    v, blob = ref_vectors
    arr = np.frombuffer(blob, dtype=np.uint8)
    offs = np.array([r["off"] for r in v["vectors"]], dtype=np.uint64)
    lens = np.array([r["n"] for r in v["vectors"]], dtype=np.uint32)
    return v, arr, offs, lens


def test_emu_crc32c_raw_and_verify(golden_arrays):
    v, arr, offs, lens = golden_arrays
    out = emu.crc32c(arr, offs, lens)
    assert (out == np.array([r["crc32c"] for r in v["vectors"]], np.uint32)).all()
    comp, st, ok, bad = emu.block_verify(1, arr, offs, lens)
    assert (comp == np.array([r["builtin_plus1"][1] for r in v["vectors"]], np.uint32)).all()


def test_emu_xxh3_and_blocks(golden_arrays):
    v, arr, offs, lens = golden_arrays
    out = emu.xxh3(arr, offs, lens)
    assert (out == np.array([r["xxh3"] for r in v["vectors"]], np.uint64)).all()
    for t in (1, 4):
        got = emu.block_checksum(t, arr, offs, lens)
        assert (got == np.array([r["with_last"][t] for r in v["vectors"]], np.uint32)).all()


def test_emu_xxhash_legacy_blocks(golden_arrays):
    # kxxHash / kxxHash64 (format.cc:573-576, :603-622) against the reference
    v, arr, offs, lens = golden_arrays
    for t in (2, 3):
        got = emu.block_checksum(t, arr, offs, lens)
        assert (got == np.array([r["with_last"][t] for r in v["vectors"]], np.uint32)).all()
        # virtual last byte (last_bytes[] given, type byte not in memory)
        last = np.array([arr[int(o) + int(n)] for o, n in zip(offs, lens)], np.uint8)
        got = emu.block_checksum(t, arr, offs, lens, last=last)
        assert (got == np.array([r["with_last"][t] for r in v["vectors"]], np.uint32)).all()
        comp, st, ok, bad = emu.block_verify(t, arr, offs, lens)
        assert (comp == np.array([r["builtin_plus1"][t] for r in v["vectors"]], np.uint32)).all()


def test_emu_trailer_roundtrip_mixed():
    rng = np.random.default_rng(8)
    sizes = rng.integers(0, 9000, 400).astype(np.uint32)
    offs = np.zeros(len(sizes), np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5)
    total = int(offs[-1]) + int(sizes[-1]) + 5
    base = rng.integers(0, 256, total, dtype=np.uint8)
    types = rng.integers(0, 8, len(sizes), dtype=np.uint8)
    mods = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    for t in (1, 2, 3, 4):
        b2, out = emu.block_trailer(t, base, offs, sizes, types, mods)
        want = O.block_checksum_batch(t, base, offs, sizes, last_bytes=types, modifiers=mods)
        assert (out == want).all()
        o, n = int(offs[5]), int(sizes[5])
        assert b2[o + n] == types[5]
        assert struct.unpack("<I", b2[o + n + 1:o + n + 5].tobytes())[0] == int(want[5])
        comp, st, ok, bad = emu.block_verify(t, b2, offs, sizes, mods)
        assert bad == 0 and ok.all()


def test_emu_lane_kernel_unaligned_and_corrupt():
    """kxxHash / kxxHash64 through the lane kernel (buffers >= 4 KiB): ragged
    sizes at unaligned offsets (the transposed 16-lane loads and the
    realignment dword), 16 KiB blocks, the tail slot's stored word in verify
    mode; then one flipped byte per 7th block is found exactly there"""
    rng = np.random.default_rng(61)
    sizes = np.concatenate([rng.integers(0, 9000, 200), rng.integers(0, 600, 60),
                            [16384] * 12, [255, 256, 257, 259, 260, 511, 512, 513]]).astype(np.uint32)
    offs = np.zeros(len(sizes), np.uint64)
    gaps = rng.integers(0, 4, len(sizes) - 1).astype(np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5 + gaps)
    total = int(offs[-1]) + int(sizes[-1]) + 5
    base = rng.integers(0, 256, total, dtype=np.uint8)
    types = rng.integers(0, 8, len(sizes), dtype=np.uint8)
    mods = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    for t in (2, 3):
        b2, out = emu.block_trailer(t, base, offs, sizes, types, mods)
        want = O.block_checksum_batch(t, base, offs, sizes, last_bytes=types, modifiers=mods)
        assert (out == want).all()
        got = emu.block_checksum(t, base, offs, sizes, last=types)
        assert (got == O.block_checksum_batch(t, base, offs, sizes, last_bytes=types)).all()
        comp, st, ok, bad = emu.block_verify(t, b2, offs, sizes, mods)
        assert bad == 0 and ok.all()
        b3 = b2.copy()
        hit = np.arange(0, len(sizes), 7)
        hit = hit[sizes[hit] > 0]
        for k in hit:
            b3[int(offs[k]) + int(rng.integers(0, int(sizes[k])))] ^= 0x10
        comp, st, ok, bad = emu.block_verify(t, b3, offs, sizes, mods)
        assert bad == len(hit) and (np.flatnonzero(ok == 0) == hit).all()


def test_emu_wal():
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 40000, 60).astype(np.uint32)
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens)
    st, nrec, fail, bad = emu.wal_verify(buf)
    assert bad == 0 and (st == 0).all() and int(nrec.sum()) == len(poffs)


@pytest.mark.parametrize("max_len", [200, 1100, 2000])
def test_emu_wal_dense_blocks(max_len, monkeypatch):
    """blocks of 30 to ~290 records (wal.hip wal_walk_kernel / wal_fill_kernel):
    CRC failures early and late in a block == the serial per-block reader
    (FORST_WAL_VARIANT=wave)."""
    rng = np.random.default_rng(max_len)
    lens = rng.integers(0, max_len, 32768 * 3 // (max_len // 2 + 7)).astype(np.uint32)
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens)
    blk = (poffs // 32768).astype(np.int64)
    per = np.bincount(blk)
    assert per.max() > 32 or max_len > 1000
    b = buf.copy()
    for k in (int(np.nonzero(blk == 0)[0][5]), int(np.nonzero(blk == 1)[0][-1])):
        if plens[k] > 0:
            b[int(poffs[k]) + 7] ^= 0x10
    got = emu.wal_verify(b)
    monkeypatch.setenv("FORST_WAL_VARIANT", "wave")
    want = emu.wal_verify(b)
    monkeypatch.delenv("FORST_WAL_VARIANT")
    for g, w in zip(got[:3], want[:3]):
        assert (g == w).all()
    assert got[3] == want[3]
    st, nrec, fail, bad = emu.wal_verify(buf)
    assert bad == 0 and int(nrec.sum()) == len(poffs)


@pytest.mark.parametrize("recyclable,split", [(False, "0"), (True, "0"), (False, "1"),
                                               (True, "1")])
def test_emu_wal_pipeline_statuses(recyclable, split, monkeypatch):
    """walk/scan/fill/raw-CRC/status pipeline == the serial per-block reader
    (FORST_WAL_VARIANT=wave) on every status: CRC failure, bad length, old
    record, zero padding, truncated tail; writer-side CRCs restore the image."""
    monkeypatch.setenv("FORST_WAL_SPLIT", split)  # 1: small / large records on two kernels
    rng = np.random.default_rng(2)
    lens = rng.integers(0, 9000, 90).astype(np.uint32)
    lens[:4] = [0, 32761, 5, 70000]
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=recyclable, log_number=9)
    hs = 11 if recyclable else 7
    b = buf.copy()
    nb = (len(b) + 32767) // 32768
    blk = (poffs // 32768).astype(np.int64)
    firsts = [int(np.nonzero(blk == k)[0][0]) for k in range(nb) if (blk == k).any()]
    k0, k1, k2, k3 = firsts[1], firsts[3], firsts[5], firsts[7]
    assert plens[k0] > 0
    b[int(poffs[k0]) + hs] ^= 0x40                        # CRC covers the payload
    b[int(poffs[k1]) + 4:int(poffs[k1]) + 6] = 0xff              # length past the block
    if recyclable:
        b[int(poffs[k2]) + 7] ^= 1                          # older log number
    b[int(poffs[k3]):int(poffs[k3]) + 7] = 0               # zero type/length
    b = b[:len(b) - 3]                                     # truncated tail
    got = emu.wal_verify(b, log_number=9)
    monkeypatch.setenv("FORST_WAL_VARIANT", "wave")
    want = emu.wal_verify(b, log_number=9)
    monkeypatch.delenv("FORST_WAL_VARIANT")
    for g, w in zip(got[:3], want[:3]):
        assert (g == w).all()
    assert got[3] == want[3] and got[3] >= 2
    # the oracle's per-block form (the full-size GPU tests' checker) agrees
    for g, w in zip(got[:3], O.wal_verify_blocks(b, 9, nthreads=2)):
        assert (np.asarray(g) == w).all()
    assert got[0][blk[k0]] == 1 and got[0][blk[k1]] == 2 and got[0][blk[k3]] == 3
    if recyclable:
        assert got[0][blk[k2]] == 4
    # writer side, with one out-of-range offset
    w = buf.copy()
    for o in poffs:
        w[int(o):int(o) + 4] = 0
    offs = np.concatenate([poffs.astype(np.uint64), [len(buf) - 3]])
    crcs, img = emu.wal_record_crc(w, offs)
    assert (img[:len(buf)] == buf).all() and crcs[-1] == 0
    assert (crcs[:-1] == np.frombuffer(b"".join(buf[int(o):int(o) + 4].tobytes()
                                                for o in poffs), np.uint32)).all()


def test_emu_crc_stream_batches_and_edges():
    """> 64 blocks per wave (descriptor/result batch switches), the 64-byte
    fast-path threshold, every start alignment, a block at the buffer start
    (head lane would underflow -> wave_crc32c path), all CRC modes."""
    rng = np.random.default_rng(21)
    n = 2600
    sizes = rng.integers(0, 700, n).astype(np.uint32)
    sizes[:40] = np.arange(40) + 40          # 40..79 around the threshold
    sizes[40:48] = [4091, 4092, 4093, 4094, 4095, 4096, 8191, 12000]
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5 + rng.integers(0, 4, n - 1))
    total = int(offs[-1]) + int(sizes[-1]) + 5 + 4096
    base = rng.integers(0, 256, total, dtype=np.uint8)
    types = rng.integers(0, 8, n, dtype=np.uint8)
    mods = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    # compute, type byte from memory and from last_bytes[]
    want = O.block_checksum_batch(1, base, offs, sizes, modifiers=mods)
    assert (emu.block_checksum(1, base, offs, sizes, mods=mods) == want).all()
    want = O.block_checksum_batch(1, base, offs, sizes, last_bytes=types, modifiers=mods)
    assert (emu.block_checksum(1, base, offs, sizes, last=types, mods=mods) == want).all()
    # trailer then verify (with a corruption)
    b2, out = emu.block_trailer(1, base, offs, sizes, types, mods)
    assert (out == want).all()
    b2[int(offs[7]) + 3] ^= 0x10
    comp, st, ok, bad = emu.block_verify(1, b2, offs, sizes, mods)
    assert bad == 1 and not ok[7] and ok.sum() == n - 1
    # raw crc32c::Extend with per-message init
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = emu.crc32c(base, offs, sizes, init=init)
    for k in range(0, n, 37):
        o, s = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.crc32c_extend(int(init[k]), base[o:o + s]), (k, s, o & 3)
    # the XXH3 stream kernel on the same layout (short and long inputs)
    want = O.block_checksum_batch(4, base, offs, sizes, last_bytes=types, modifiers=mods)
    assert (emu.block_checksum(4, base, offs, sizes, last=types, mods=mods) == want).all()
    want = O.block_checksum_batch(4, base, offs, sizes, modifiers=mods)
    assert (emu.block_checksum(4, base, offs, sizes, mods=mods) == want).all()
    b2, out = emu.block_trailer(4, base, offs, sizes, types, mods)
    b2[int(offs[41]) + 1000] ^= 0x01
    comp, st, ok, bad = emu.block_verify(4, b2, offs, sizes, mods)
    assert bad == 1 and not ok[41] and ok.sum() == n - 1
    got = emu.xxh3(base, offs, sizes)
    for k in range(0, n, 41):
        o, s = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.xxh3_64(base[o:o + s]), (k, s)
    # messages at the very start of the buffer (round-0 head would underflow)
    offs2 = np.array([0, 1, 2, 3, 70, 4100], np.uint64)
    sizes2 = np.array([5000, 4999, 64, 4093, 100, 9000], np.uint32)
    got = emu.crc32c(base, offs2, sizes2)
    for k in range(len(offs2)):
        o, s = int(offs2[k]), int(sizes2[k])
        assert int(got[k]) == O.crc32c_extend(0, base[o:o + s]), k


def test_emu_blocks_at_buffer_start():
    """Blocks whose first 32-byte lane segment would start in front of the
    buffer (offset < 28, head dword index > offset/4): the v2 CRC kernel loads
    that segment from offset 0 and re-aligns it in registers."""
    rng = np.random.default_rng(33)
    base = rng.integers(0, 256, 200000, dtype=np.uint8)
    offs, sizes = [], []
    for o in range(28):
        for d in (0, 4, 8, 12, 20, 28, 100, 2047, 2048, 2049, 4095):
            offs.append(o)
            sizes.append(4096 + d + (o * 7) % 5)
    offs = np.array(offs, np.uint64)
    sizes = np.array(sizes, np.uint32)
    init = rng.integers(0, 2**32, len(offs), dtype=np.uint64).astype(np.uint32)
    got = emu.crc32c(base, offs, sizes, init=init)
    for k in range(len(offs)):
        o, s = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.crc32c_extend(int(init[k]), base[o:o + s]), (o, s)
    want = O.block_checksum_batch(1, base, offs, sizes)
    assert (emu.block_checksum(1, base, offs, sizes) == want).all()
    comp, st, ok, bad = emu.block_verify(1, base, offs, sizes)
    ocomp, ook, obad = O.block_verify_batch(1, base, offs, sizes)
    assert (comp == ocomp).all() and bad == obad


def test_emu_offsets_above_2gib():
    """64-bit descriptor offsets (bit 31 set): readlane results must not be
    sign-extended when the offset is rebuilt (a GPU-only failure mode at the
    full C2 size, 1 M x 4 KiB = 4.3 GB)."""
    big = (1 << 31) + 3 * 65536
    base = np.zeros(big, dtype=np.uint8)  # lazily zero pages
    rng = np.random.default_rng(5)
    tail0 = (1 << 31) - 65536
    base[tail0:] = rng.integers(0, 256, big - tail0, dtype=np.uint8)
    offs = np.array([tail0 + 3, (1 << 31) + 1, (1 << 31) + 70001, (1 << 31) - 9000],
                    np.uint64)
    sizes = np.array([60000, 4096, 5000, 8999], np.uint32)
    got = emu.crc32c(base, offs, sizes)
    for k in range(len(offs)):
        o, s = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.crc32c_extend(0, base[o:o + s]), k


def test_emu_hash64_golden(golden_arrays):
    # Hash64 (XXPH3) kernel vs the reference's values, per-buffer seeds
    v, arr, offs, lens = golden_arrays
    got0 = emu.hash64(arr, offs, lens)
    assert (got0 == np.array([r["hash64_s0"] for r in v["vectors"]], np.uint64)).all()
    seeds = np.full(len(offs), O.KV_SEED_V, np.uint64)
    got1 = emu.hash64(arr, offs, lens, seeds=seeds)
    assert (got1 == np.array([r["hash64_s1"] for r in v["vectors"]], np.uint64)).all()


@pytest.mark.parametrize("prot_bytes,flags", [(8, (True, True, False)), (1, (False, False, False)),
                                              (4, (True, True, True)), (2, (True, False, True))])
def test_emu_kv_protect_verify(prot_bytes, flags):
    import kvdata
    d = kvdata.make_kv(150, 3 + prot_bytes, prot_bytes, *flags)
    got = emu.kv_protect(d["base"], d["ko"], d["ks"], d["vo"], d["vs"], d["ops"], d["seqs"],
                         d["cfs"])
    assert (got == d["prot"]).all()
    comp, ok, bad = emu.kv_verify(d["base"], d["ko"], d["ks"], d["vo"], d["vs"], prot_bytes,
                                  d["co"], d["ops"], d["seqs"], d["cfs"])
    assert bad == 0 and ok.all() and (comp == d["prot"]).all()
    b2 = d["base"].copy()
    b2[int(d["vo"][40]) + max(0, int(d["vs"][40]) - 1)] ^= 0x04  # value byte (or separator)
    b2[int(d["co"][77])] ^= 0x80                                  # stored checksum
    comp, ok, bad = emu.kv_verify(b2, d["ko"], d["ks"], d["vo"], d["vs"], prot_bytes, d["co"],
                                  d["ops"], d["seqs"], d["cfs"])
    want_bad = {77} | ({40} if int(d["vs"][40]) > 0 else set())
    assert set(np.nonzero(ok == 0)[0].tolist()) == want_bad and bad == len(want_bad)


def test_emu_kv_staged_and_direct_subtiles():
    """kv_kernel's sub-tiles: packed entries of small values (their 8-entry
    spans fit the LDS stage), entries with 3-6 KiB values (spans over it:
    global loads), entries in reverse buffer order, the buffer ending at the
    last entry's checksum (the last span may not be staged), and a base that
    is not 16-byte aligned (no staging) -- every hash equal to the oracle's"""
    rng = np.random.default_rng(77)
    n = 400
    ks = rng.integers(0, 90, n).astype(np.uint32)
    vs = rng.integers(0, 900, n).astype(np.uint32)
    vs[rng.integers(0, n, 25)] = rng.integers(3000, 6000, 25)
    ks[rng.integers(0, n, 5)] = rng.integers(241, 700, 5)
    ko = np.zeros(n, np.uint64)
    vo = np.zeros(n, np.uint64)
    pos = 3
    for i in range(n):
        ko[i] = pos
        pos += int(ks[i])
        vo[i] = pos
        pos += int(vs[i]) + 8
    base = rng.integers(0, 256, pos, dtype=np.uint8)
    ops = rng.integers(0, 26, n).astype(np.uint8)
    seqs = rng.integers(0, 2**63, n, dtype=np.uint64)
    want = O.kv_protect_batch(base, ko, ks, vo, vs, ops, seqs, None)
    assert (emu.kv_protect(base, ko, ks, vo, vs, ops, seqs) == want).all()
    r = np.arange(n)[::-1].copy()
    got = emu.kv_protect(base, ko[r], ks[r], vo[r], vs[r], ops[r], seqs[r])
    assert (got == want[r]).all()
    assert (emu.kv_protect(base, ko, ks, vo, vs, ops, seqs, misalign=4) == want).all()


def test_emu_crc32c_buffer():
    """whole-buffer CRC: 64 KiB chunk CRCs folded with the combine identity"""
    rng = np.random.default_rng(31)
    buf = rng.integers(0, 256, 3 * 65536 + 777, dtype=np.uint8)
    for n in (0, 1, 63, 65535, 65536, 65537, 2 * 65536 + 5, len(buf)):
        for init in (0, 0xDEADBEEF):
            assert emu.crc32c_buffer(buf[:n], init) == O.crc32c_extend(init, buf[:n].tobytes())


@pytest.mark.parametrize("recyclable", [False, True])
def test_emu_wal_record_xxh3(recyclable):
    """a14: XXH3 of each logical record = XXH3 of its payload, whether one
    fragment or First/Middle*/Last across log blocks"""
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 3000, 40).astype(np.uint32)
    lens[[3, 10, 20]] = [70000, 32761, 40000]
    lens[5] = 0
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=recyclable, log_number=3)
    h, first = emu.wal_record_xxh3(buf, poffs)
    assert len(h) == len(lens)
    starts = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    for j in range(len(lens)):
        assert int(h[j]) == O.xxh3_64(payload[starts[j]:starts[j + 1]].tobytes()), j


@pytest.mark.parametrize("recyclable", [False, True])
def test_emu_wal_record_xxh3_fragment_edges(recyclable):
    """a14 across log-block boundaries at every lane-slot byte, window and
    stripe edge, last fragments of 63-66 bytes, 241-300-byte records, empty
    first fragments, 3-4 fragments (tests/walcases.py): the in-place
    fragment-aware hash and the gathered fallback both equal XXH3 of the
    payload"""
    import walcases as W
    buf, po, payload, lens, targets = W.frag_edge_log(recyclable, seed=5 + recyclable)
    first = W.first_fragment_offsets(buf, po)
    hs = 11 if recyclable else 7
    for j, l0 in targets:  # the generator placed each case where it meant to
        assert int(first[j]) % W.BLOCK == W.BLOCK - hs - l0, (j, l0)
    h, f = emu.wal_record_xxh3(buf, po)
    assert len(h) == len(lens)
    assert (np.asarray(h).view(np.uint64) == W.expected_hashes(payload, lens)).all()


def test_emu_xxh3_short_inputs_on_rows():
    """every length 0..260 at every start alignment, and inputs ending in the
    buffer's first 16 bytes (the <= 16-byte window is then loaded from 0):
    the row-parallel short path (xxh3_short_row) in raw, compute and verify
    modes"""
    rng = np.random.default_rng(77)
    sizes, offs = [], []
    pos = 0
    for o in range(16):  # at the buffer start
        for L in (0, 1, 2, 3, 4, 7, 8, 9, 15, 16 - o if o < 16 else 1):
            if o + L <= 16:
                offs.append(o)
                sizes.append(L)
    pos = 64
    for L in range(0, 261):
        for m in range(4):
            pos += m
            offs.append(pos)
            sizes.append(L)
            pos += L + 5
    sizes += [241, 1000, 5000]  # long ones in the same launch
    for L in sizes[-3:]:
        offs.append(pos)
        pos += L + 5
    offs = np.array(offs, np.uint64)
    sizes = np.array(sizes, np.uint32)
    base = rng.integers(0, 256, pos + 8192, dtype=np.uint8)
    got = emu.xxh3(base, offs, sizes)
    for k in range(len(offs)):
        o, n = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.xxh3_64(base[o:o + n]), (k, o, n)
    keep = offs >= 64  # block modes need the 5 trailer bytes in front of the next block
    offs, sizes = offs[keep], sizes[keep]
    want = O.block_checksum_batch(4, base, offs, sizes)
    assert (emu.block_checksum(4, base, offs, sizes) == want).all()
    types = rng.integers(0, 8, len(offs), dtype=np.uint8)
    b2, out = emu.block_trailer(4, base, offs, sizes, types, None)
    comp, st, ok, bad = emu.block_verify(4, b2, offs, sizes)
    assert bad == 0 and (comp == out).all()


def test_emu_rows_extra_dword_windows():
    """4096- and 1024·k-byte blocks at every start alignment: the rows kernel
    ends windows that are one dword longer than whole rounds one dword early
    and steps that dword in the finish"""
    rng = np.random.default_rng(5)
    sizes = np.array([4096, 4096, 4096, 4096, 1024, 2048, 3072, 4095, 4097, 8192] * 8, np.uint32)
    offs = np.zeros(len(sizes), np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5 + rng.integers(0, 4, len(sizes) - 1))
    base = rng.integers(0, 256, int(offs[-1]) + int(sizes[-1]) + 4096, dtype=np.uint8)
    types = rng.integers(0, 8, len(sizes), dtype=np.uint8)
    for t in (1, 4):
        want = O.block_checksum_batch(t, base, offs, sizes)
        assert (emu.block_checksum(t, base, offs, sizes) == want).all()
        b2, out = emu.block_trailer(t, base, offs, sizes, types)
        comp, st, ok, bad = emu.block_verify(t, b2, offs, sizes)
        assert bad == 0 and ok.all()


@pytest.mark.parametrize("recyclable", [False, True])
def test_emu_raw_split_short_and_long(recyclable):
    """Raw batches big enough for the global feed (>= 64 descriptors per wave
    of the grid) are split by length (crc32c.hip FORST_RAW_SPLIT, 256 B):
    shorter messages one per lane (crc32c_raw_lane_kernel), the rest on the
    rows kernel, which drops the short ones from each batch as it loads it
    (crc32c_rows_raw_filt_kernel).  Every length around the split, every start
    alignment, per-message init, messages ending at the buffer end, and
    out-of-range descriptors on both sides (one at an offset >= 2^58, whose
    top bits the filter kernel reuses); then the WAL writer's lengths mode
    and the reader's verify (only mismatching CRCs stored) on > 2048
    physical records with corruptions in short and long ones."""
    rng = np.random.default_rng(52 + int(recyclable))
    n = 3000
    sizes = rng.integers(0, 1500, n).astype(np.uint32)
    split = 256  # FORST_RAW_SPLIT: the 64 lengths straddle it (split - 32 .. split + 31)
    sizes[:64] = split - 32 + np.arange(64)
    sizes[64:80] = np.arange(16)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + rng.integers(0, 4, n - 1).astype(np.uint64))
    total = int(offs[-1]) + int(sizes[-1])
    base = rng.integers(0, 256, total, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = emu.crc32c(base, offs, sizes, init=init)
    for k in range(n):
        o, s = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.crc32c_extend(int(init[k]), base[o:o + s]), (k, s, o & 3)
    o2, s2 = offs.copy(), sizes.copy()
    o2[5], s2[5] = total - 3, 10                 # short, past the end
    o2[6], s2[6] = total - 100, 600              # long, past the end
    o2[7], s2[7] = 1 << 59, 600                  # long, offset >= 2^58
    o2[8], s2[8] = (1 << 58) - 1, 700            # long, just below 2^58
    o2[9], s2[9] = total - 509, 509              # long, ends at the buffer end
    o2[10], s2[10] = total - 1300, 1300          # long, ends at the buffer end
    o2[11], s2[11] = total - 255, 255            # short (split - 1), ends at the buffer end:
    o2[12], s2[12] = total - 256, 256            # the lane kernel's end-of-buffer fallback,
    o2[13], s2[13] = total - 77, 77              # then the split itself
    got = emu.crc32c(base, o2, s2)
    for k in range(n):
        o, s = int(o2[k]), int(s2[k])
        want = 0 if k in (5, 6, 7, 8) else O.crc32c_extend(0, base[o:o + s])
        assert int(got[k]) == want, (k, o, s)
    # the WAL on both sides of the split
    lens = rng.integers(0, 1200, 2500).astype(np.uint32)
    lens[:30] = 505 - np.arange(30) % 12
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=recyclable, log_number=5)
    assert len(poffs) > 2048
    w = buf.copy()
    for o in poffs:
        w[int(o):int(o) + 4] = 0
    crcs, img = emu.wal_record_crc_lengths(w, poffs, plens, recyclable=recyclable)
    assert (img[:len(buf)] == buf).all()
    assert (crcs == np.frombuffer(b"".join(buf[int(o):int(o) + 4].tobytes() for o in poffs),
                                  np.uint32)).all()
    # in place only (no CRC array): the kernels' own header stores
    _, img = emu.wal_record_crc_lengths(w, poffs, plens, recyclable=recyclable, with_out=False)
    assert (img[:len(buf)] == buf).all()
    b = buf.copy()
    hs = 11 if recyclable else 7
    short = [k for k in range(len(poffs)) if 0 < plens[k] < 400]
    longr = [k for k in range(len(poffs)) if plens[k] > 900]
    for k in (short[3], short[-2], longr[4], longr[-3]):
        b[int(poffs[k]) + hs + int(plens[k]) // 2] ^= 0x08
    got = emu.wal_verify(b, log_number=5)
    ost = O.wal_verify_blocks(b, 5, nthreads=2)
    for g, want in zip(got[:3], ost):
        assert (np.asarray(g) == want).all()
    assert got[3] == int(((ost[0] != 0) & (ost[0] != 3)).sum()) >= 2


def test_emu_raw_split_sparse_long():
    """A raw batch whose long messages are sparse -- one in ~150, as a WAL
    recovery's raw list (short candidates plus a few irregular long records)
    -- so the compacted descriptor batches hold fewer entries than a wave has
    rows: rows wait for the next batch instead of skipping positions
    (crc32c.hip FILT), every message computed once, results exact."""
    rng = np.random.default_rng(77)
    n = 9000
    sizes = rng.integers(0, 200, n).astype(np.uint32)
    longs = rng.choice(n, 60, replace=False)
    sizes[longs] = rng.integers(256, 6000, len(longs))
    sizes[:3] = [300, 0, 5000]
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 7)
    total = int(offs[-1]) + int(sizes[-1]) + 7
    base = rng.integers(0, 256, total, dtype=np.uint8)
    got = emu.crc32c(base, offs, sizes)
    want = np.array([O.crc32c_extend(0, base[int(o):int(o) + int(s)]) for o, s in zip(offs, sizes)],
                    np.uint32)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (len(bad), bad[:8].tolist(), sizes[bad[:8]].tolist())


# ---- a15 at the reference's call sites (kv_sites fixtures, gen_kv_golden.py) --
def test_emu_memtable_entries_vs_reference(kv_sites):
    import kvsites

    for name, base, offs, pb, want in kvsites.memtable_cases(*kv_sites):
        comp, st, bad = emu.memtable_verify(base, offs, pb)
        assert [O.MEM_STATUS[int(s)] for s in st] == want, name
        ocomp, ost = O.memtable_verify_batch(base, len(base), offs, pb)
        assert (comp == ocomp).all() and bad == int((st != 0).sum()), name
        if not name.endswith("_corrupt") and name != "crafted":
            # MemTable::UpdateEntryChecksum in place over zeroed checksum bytes
            z = base.copy()
            for o in offs:
                c = kvsites.mem_checksum_pos(base, int(o))
                z[c:c + pb] = 0
            b2, out, pst = emu.memtable_protect(z, offs, pb)
            assert (out == comp).all() and (pst == 0).all()
            assert (b2[:len(base)] == base).all(), name


def test_emu_write_batch_vs_reference(kv_sites):
    import kvsites

    base, offs, lens, reps = kvsites.write_batch_case(*kv_sites)
    prot, first, st, nprot = emu.write_batch_protect(base, offs, lens)
    for j, (name, status, want) in enumerate(reps):
        assert O.WB_STATUS[int(st[j])] == status, name
        got = prot[int(first[j]):int(first[j]) + int(nprot[j])]
        assert [int(x) for x in got] == [int(x) for x in want][:len(got)], name
        if status == "OK":
            assert len(got) == len(want), name


def test_emu_block_kv_checksums_vs_reference(kv_sites):
    """Block::Initialize*BlockProtectionInfo's kv_checksum_ (block.cc:1113-1235)
    for data / index / metaindex blocks of reference-written SSTs"""
    import kvsites

    base, offs, sizes, kinds, cases = kvsites.block_case(*kv_sites)
    for pb in (8, 2):
        enc, prot, first, st = emu.block_kv_checksum(base, offs, sizes, kinds, pb)
        for j, c in enumerate(cases):
            nk = int(first[j + 1] - first[j])
            want = c[f"keys_{pb}"]
            if want < 0:
                assert st[j] != 0 and nk == 0, c
                continue
            assert st[j] == 0 and nk == want, (c["src"], c["kind_name"], nk, want)
            got = enc[int(first[j]) * pb:int(first[j + 1]) * pb].tobytes().hex()
            assert got == c[f"kv_checksum_{pb}"], (c["src"], c["kind_name"])


@pytest.mark.parametrize("recyclable", [False, True])
def test_emu_wal_record_xxh3_unpacked_form(recyclable):
    """a14's unpacked bookkeeping (wal_hash.h: the flag kernel, a second scan
    and gpos, taken beyond 2^24 records or a 2^40-byte log; the patch kernel
    then writes straight into out) forced on with FORST_WH_UNPACKED: the same
    fragment-edge log as above, every logical record's hash equals XXH3 of its
    payload"""
    import walcases as W
    buf, po, payload, lens, targets = W.frag_edge_log(recyclable, seed=9 + recyclable)
    with emu.variant("-DFORST_WH_UNPACKED"):
        h, f = emu.wal_record_xxh3(buf, po)
    assert len(h) == len(lens)
    assert (np.asarray(h).view(np.uint64) == W.expected_hashes(payload, lens)).all()
