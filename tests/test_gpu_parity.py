"""GPU parity: HIP kernels (through the C ABI) vs the pinned CPU oracle.

Bit-exact for every case (integer/byte work).  Covers the reference's edge
cases: empty batches and zero-length blocks, unaligned starts (every start
alignment), lengths around every internal boundary (16/32/64/240/1024/4096),
blocks at the very start/end of the buffer, context modifiers (fv6),
corruption detection, out-of-range descriptors, WAL framing with all record
types, and the full-size configs through size-independent properties.
"""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from forst_amd import engine, workload  # noqa: E402
from forst_amd.engine import ChecksumType as CT  # noqa: E402
from oracle import oracle as O  # noqa: E402
import stream  # noqa: E402,F401  (tests/golden on sys.path via conftest)

DEV = "cuda"
NT = O.host_threads()  # the oracle's threads: the CPUs this process may use


def d(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def host(t):
    return t.cpu().numpy()


@pytest.fixture(scope="module")
def golden(ref_vectors):
    v, blob = ref_vectors
    arr = np.frombuffer(blob, dtype=np.uint8).copy()
    offs = np.array([r["off"] for r in v["vectors"]], dtype=np.int64)
    lens = np.array([r["n"] for r in v["vectors"]], dtype=np.int32)
    return v, arr, d(arr), d(offs), d(lens)


ALL_TYPES = [CT.kCRC32c, CT.kXXH3, CT.kxxHash, CT.kxxHash64, CT.kNoChecksum]
HASH_TYPES = [CT.kCRC32c, CT.kXXH3, CT.kxxHash, CT.kxxHash64]


def test_library_loads_and_reports_gfx950():
    engine.init_device()
    assert "gfx950" in engine.version()


def test_crc32c_raw_golden(golden):
    v, arr, base, offs, lens = golden
    out = host(engine.crc32c_batch(base, offs, lens)).astype(np.uint64)
    want = np.array([r["crc32c"] for r in v["vectors"]], dtype=np.uint64)
    bad = np.nonzero(out != want)[0]
    assert bad.size == 0, [(v["vectors"][i]["n"], v["vectors"][i]["off"]) for i in bad[:10]]


def test_crc32c_extend_with_init(golden):
    v, arr, base, offs, lens = golden
    rng = np.random.default_rng(11)
    init = rng.integers(0, 2**32, len(v["vectors"]), dtype=np.uint64).astype(np.uint32)
    out = host(engine.crc32c_batch(base, offs, lens, init_crcs=d(init.view(np.int32))))
    for k, r in enumerate(v["vectors"]):
        want = O.crc32c_extend(int(init[k]), arr[r["off"]:r["off"] + r["n"]])
        assert int(out[k]) == want, (r["n"], r["off"])


@pytest.mark.parametrize("mean", [600, 5000, 40000])
def test_crc32c_extend_multi_round_with_init(mean):
    """crc32c::Extend(init, data, n) with a per-message init over messages of
    1..~3 x mean bytes at every alignment, from the buffer start on: the rows
    kernel (mean <= 20 KiB) and the v2 kernel take the init in round 0 of a
    message, many rounds before its finish"""
    rng = np.random.default_rng(mean)
    n = 3000
    sizes = rng.integers(1, 3 * mean, n).astype(np.uint32)
    sizes[:64] = np.arange(1, 65)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + rng.integers(0, 9, n - 1).astype(np.uint64))
    total = int(offs[-1]) + int(sizes[-1]) + 64
    base = rng.integers(0, 256, total, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = host(engine.crc32c_batch(d(base), d(offs.view(np.int64)), d(sizes.view(np.int32)),
                                   init_crcs=d(init.view(np.int32)))).view(np.uint32)
    for k in range(n):
        o, s = int(offs[k]), int(sizes[k])
        assert int(got[k]) == O.crc32c_extend(int(init[k]), base[o:o + s]), (k, o, s)


def test_xxh3_raw_golden(golden):
    v, arr, base, offs, lens = golden
    out = host(engine.xxh3_64_batch(base, offs, lens)).view(np.uint64)
    want = np.array([r["xxh3"] for r in v["vectors"]], dtype=np.uint64)
    bad = np.nonzero(out != want)[0]
    assert bad.size == 0, [v["vectors"][i]["n"] for i in bad[:10]]


@pytest.mark.parametrize("ctype", ALL_TYPES)
def test_block_checksum_with_last_byte_golden(golden, ctype):
    v, arr, base, offs, lens = golden
    # last byte read from memory (base[off+n]) and passed explicitly
    out_mem = host(engine.block_checksum_batch(ctype, base, offs, lens)).astype(np.uint64)
    lasts = np.array([arr[r["off"] + r["n"]] for r in v["vectors"]], dtype=np.uint8)
    out_arr = host(engine.block_checksum_batch(ctype, base, offs, lens,
                                               last_bytes=d(lasts))).astype(np.uint64)
    want = np.array([r["with_last"][int(ctype)] for r in v["vectors"]], dtype=np.uint64)
    assert (out_mem == want).all()
    assert (out_arr == want).all()


@pytest.mark.parametrize("ctype", HASH_TYPES)
def test_verify_computed_matches_builtin_golden(golden, ctype):
    v, arr, base, offs, lens = golden
    comp, stored, ok, bad = engine.block_verify_batch(ctype, base, offs, lens)
    comp = host(comp).astype(np.uint64)
    want = np.array([r["builtin_plus1"][int(ctype)] for r in v["vectors"]], dtype=np.uint64)
    assert (comp == want).all()
    # stored = LE32 at off+n+1 (random bytes here) -> ok iff equal
    st = host(stored).astype(np.uint64)
    exp_st = np.array([struct.unpack("<I", arr[r["off"] + r["n"] + 1:r["off"] + r["n"] + 5]
                                     .tobytes())[0] for r in v["vectors"]], dtype=np.uint64)
    assert (st == exp_st).all()
    assert (host(ok).astype(bool) == (exp_st == want)).all()
    assert int(host(bad)[0]) == int((exp_st != want).sum())


def test_table_test_kats_on_gpu(kats):
    k = kats["table_test"]
    for t_str, expected in k["expected_hex"].items():
        t = int(t_str)
        datas = []
        for name, ct in k["cases"]:
            b = k["inputs"][name].encode()
            if ct is not None:
                b = b[:-1] + bytes([ct])
            datas.append(b)
        # lay out as blocks: payload = data[:-1], type byte = data[-1]
        buf = bytearray()
        offs, sizes = [], []
        for b in datas[1:]:
            offs.append(len(buf))
            sizes.append(len(b) - 1)
            buf += b + b"\0\0\0\0"
        arr = np.frombuffer(bytes(buf), dtype=np.uint8).copy()
        comp, _, _, _ = engine.block_verify_batch(t, d(arr), d(np.array(offs, np.int64)),
                                                  d(np.array(sizes, np.int32)))
        got = [struct.pack("<I", int(x)).hex().upper() for x in host(comp)]
        assert got == expected[1:], t


def _host_layout(sizes, seed):
    sizes = np.asarray(sizes, dtype=np.uint32)
    offs = np.zeros(len(sizes), dtype=np.int64)
    if len(sizes) > 1:
        offs[1:] = np.cumsum(sizes[:-1].astype(np.int64) + 5)
    total = int(offs[-1]) + int(sizes[-1]) + 5
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, total, dtype=np.uint8)
    return base, offs, sizes


EDGE_SIZES = ([0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 30, 31, 32, 33, 63, 64, 65, 127, 128, 129,
               239, 240, 241, 255, 256, 1023, 1024, 1025, 4090, 4091, 4092, 4093, 4094, 4095,
               4096, 4097, 4098, 8191, 8192, 8193, 16383, 16384, 16385, 65535, 65536, 65537])


@pytest.mark.parametrize("ctype", ALL_TYPES)
def test_edge_sizes_every_alignment(ctype):
    # every size at every start alignment mod 16
    sizes = []
    for s in EDGE_SIZES:
        sizes += [s] * 16
    # perturb offsets so that starts walk through all alignments
    base, offs, sizes = _host_layout(sizes, 7)
    for i in range(len(offs)):
        offs[i] += 0  # packed layout already gives varied alignment
    rng = np.random.default_rng(1)
    lasts = rng.integers(0, 256, len(sizes), dtype=np.uint8)
    mods = rng.integers(0, 2**32, len(sizes), dtype=np.uint64).astype(np.uint32)
    want = O.block_checksum_batch(int(ctype), base, offs, sizes, last_bytes=lasts,
                                  modifiers=mods, nthreads=4)
    got = host(engine.block_checksum_batch(ctype, d(base), d(offs), d(sizes.astype(np.int32)),
                                           last_bytes=d(lasts), modifiers=d(mods.view(np.int32))))
    bad = np.nonzero(got.astype(np.uint64) != want.astype(np.uint64))[0]
    assert bad.size == 0, [(int(sizes[i]), int(offs[i]) & 15) for i in bad[:10]]
    assert {int(o) & 15 for o in offs} == set(range(16)) or len(offs) < 64


@pytest.mark.parametrize("ctype", ALL_TYPES)
def test_trailer_then_verify_roundtrip_and_corruption(ctype):
    rng = np.random.default_rng(2)
    sizes = rng.integers(0, 20000, 3000).astype(np.uint32)
    sizes[:len(EDGE_SIZES)] = EDGE_SIZES
    base, offs, sizes = _host_layout(sizes, 3)
    types = rng.integers(0, 8, len(sizes), dtype=np.uint8)
    base_ctx = 0x9E3779B1
    mods = np.array([O.checksum_modifier_for_context(base_ctx, int(o)) for o in offs],
                    dtype=np.uint32)
    dbase, doffs, dsz = d(base), d(offs), d(sizes.astype(np.int32))
    out = torch.empty(len(sizes), dtype=torch.uint32, device=DEV)
    engine.block_trailer_batch(ctype, dbase, doffs, dsz, d(types), d(mods.view(np.int32)), out)
    hb = host(dbase)
    # trailers exactly as WriteMaybeCompressedBlock would write them
    want = O.block_checksum_batch(int(ctype), base, offs, sizes, last_bytes=types,
                                  modifiers=mods, nthreads=4)
    assert (host(out).astype(np.uint64) == want.astype(np.uint64)).all()
    for i in range(0, len(sizes), 37):
        o, n = int(offs[i]), int(sizes[i])
        assert hb[o + n] == types[i]
        assert struct.unpack("<I", hb[o + n + 1:o + n + 5].tobytes())[0] == int(want[i])
    # verify: all ok, oracle agrees
    comp, st, ok, bad = engine.block_verify_batch(ctype, dbase, doffs, dsz,
                                                  modifiers=d(mods.view(np.int32)))
    assert int(host(bad)[0]) == 0 and host(ok).all()
    _, ook, obad = O.block_verify_batch(int(ctype), hb, offs, sizes, modifiers=mods, nthreads=4)
    assert obad == 0
    # corrupt a set of blocks (payload, type byte, stored checksum) -> exactly those fail
    victims = sorted(set(rng.integers(0, len(sizes), 40).tolist()))
    hb2 = hb.copy()
    for j, i in enumerate(victims):
        o, n = int(offs[i]), int(sizes[i])
        where = [o + n, o + n + 1 + (j % 4)]
        if n:
            where.append(o + (j * 7919) % n)
        hb2[where[j % len(where)]] ^= 1 << (j % 8)
    comp, st, ok, bad = engine.block_verify_batch(ctype, d(hb2), doffs, dsz,
                                                  modifiers=d(mods.view(np.int32)))
    okh = host(ok).astype(bool)
    ocomp, ook, obad = O.block_verify_batch(int(ctype), hb2, offs, sizes, modifiers=mods,
                                            nthreads=4)
    assert (okh == ook.astype(bool)).all()
    assert (host(comp).astype(np.uint64) == ocomp.astype(np.uint64)).all()
    assert int(host(bad)[0]) == obad
    if ctype != CT.kNoChecksum:
        assert set(np.nonzero(~okh)[0].tolist()) == set(victims)


@pytest.mark.parametrize("ctype", [CT.kxxHash, CT.kxxHash64])
def test_lane_kernel_trailer_staging_overflow(ctype):
    """4 M short kxxHash blocks: a workgroup of the lane kernel finishes more
    than its 8,192 staged trailers (xxhash_legacy.hip), so the overflow path
    stores directly -- every trailer byte and checksum against the oracle"""
    rng = np.random.default_rng(61)
    sizes = rng.integers(0, 120, 4 << 20).astype(np.uint32)
    base, offs, sizes = _host_layout(sizes, 7)
    types = rng.integers(0, 8, len(sizes), dtype=np.uint8)
    dbase = d(base)
    out = torch.empty(len(sizes), dtype=torch.uint32, device=DEV)
    engine.block_trailer_batch(ctype, dbase, d(offs), d(sizes.astype(np.int32)), d(types),
                               None, out)
    want = O.block_checksum_batch(int(ctype), base, offs, sizes, last_bytes=types,
                                  nthreads=O.host_threads())
    assert (host(out).astype(np.uint64) == want.astype(np.uint64)).all()
    hb = host(dbase)
    end = (offs + sizes.astype(np.int64))
    assert (hb[end] == types).all()
    stored = np.zeros(len(sizes), np.uint32)
    for k in range(4):
        stored |= hb[end + 1 + k].astype(np.uint32) << np.uint32(8 * k)
    assert (stored == want.astype(np.uint32)).all()


def test_out_of_range_descriptors_are_reported_not_read():
    base = d(np.zeros(1000, dtype=np.uint8))
    offs = d(np.array([0, 990, 5000, 100], dtype=np.int64))
    sizes = d(np.array([10, 10, 1, 0], dtype=np.int32))
    for ct in (CT.kCRC32c, CT.kXXH3):
        _, _, ok, bad = engine.block_verify_batch(ct, base, offs, sizes)
        okh = host(ok)
        assert okh[1] == 0 and okh[2] == 0
        assert int(host(bad)[0]) >= 2


def test_empty_batch_and_unsupported_type():
    base = d(np.zeros(64, dtype=np.uint8))
    e64 = torch.empty(0, dtype=torch.int64, device=DEV)
    e32 = torch.empty(0, dtype=torch.int32, device=DEV)
    engine.block_checksum_batch(CT.kCRC32c, base, e64, e32)
    from forst_amd import ForstError
    with pytest.raises(ForstError):
        engine.block_checksum_batch(9, base, d(np.array([0], np.int64)),
                                    d(np.array([4], np.int32)))


@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_verify_and_writer_crc(recyclable):
    lens = workload.log_uniform_lengths(4000, 32, 32768, 0xF0E5700005)
    lens[:6] = [0, 1, 7, 32761, 32762, 70000]
    rng = np.random.default_rng(4)
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=recyclable, log_number=0xABC)
    dlog = d(buf)
    status, nrec, fail, bad = engine.wal_verify_batch(dlog, log_number=0xABC)
    assert int(host(bad)[0]) == 0
    assert (host(status) == 0).all()
    assert int(host(nrec).astype(np.int64).sum()) == len(poffs)
    # corrupt one record payload in block b -> that block BAD_CHECKSUM with nrec = records
    # before it in the block
    k = len(poffs) // 2
    hs = 11 if recyclable else 7
    buf2 = buf.copy()
    buf2[int(poffs[k]) + hs + max(0, int(plens[k]) - 1)] ^= 0x80
    if plens[k] == 0:
        buf2[int(poffs[k]) + 6] ^= 0x01  # type byte is covered by the CRC
    status, nrec, fail, bad = engine.wal_verify_batch(d(buf2), log_number=0xABC)
    blk = int(poffs[k]) // 32768
    st = host(status)
    assert st[blk] == 1 and int(host(bad)[0]) == 1
    before = int((((poffs // 32768) == blk) & (poffs < poffs[k])).sum())
    assert int(host(nrec)[blk]) == before
    assert int(host(fail)[blk]) == int(poffs[k]) - blk * 32768
    # writer side: wipe all CRC fields, recompute in place -> identical image
    buf3 = buf.copy()
    for o in poffs:
        buf3[int(o):int(o) + 4] = 0
    d3 = d(buf3)
    crcs = engine.wal_record_crc_batch(d3, d(poffs.astype(np.int64)))
    assert (host(d3) == buf).all()
    want = [struct.unpack("<I", buf[int(o):int(o) + 4].tobytes())[0] for o in poffs]
    assert (host(crcs).astype(np.uint64) == np.array(want, dtype=np.uint64)).all()
    # ... and from the writer's own lengths (forst_wal_record_crc_lengths: the
    # rows kernel's WAL writer mode, descriptors from the arrays, CRCs masked
    # and stored in place by the kernel)
    d4 = d(buf3)
    crcs4 = engine.wal_record_crc_batch(d4, d(poffs.astype(np.int64)),
                                        payload_lengths=d(plens.astype(np.int32)),
                                        recyclable=recyclable)
    assert (host(d4) == buf).all()
    assert (host(crcs4) == host(crcs)).all()
    # without writing in place: only crc_out
    d5 = d(buf3)
    crcs5 = engine.wal_record_crc_batch(d5, d(poffs.astype(np.int64)), write_in_place=False,
                                        payload_lengths=d(plens.astype(np.int32)),
                                        recyclable=recyclable)
    assert (host(d5) == buf3).all() and (host(crcs5) == host(crcs)).all()


@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_writer_crc_with_lengths_edges(recyclable):
    """forst_wal_record_crc_lengths against the header-reading path on the
    write-group shapes a writer produces: records of 0..70000 bytes at every
    header alignment (in-place stores of 1, 2 or 3 pieces), a log shorter
    than one 4 KiB round (the fallback path), headers that do not fit the
    log (crc_out 0, nothing written), and a C5-sized batch"""
    hs = 11 if recyclable else 7
    rng = np.random.default_rng(31)
    lens = np.concatenate([np.arange(0, 40), rng.integers(0, 70000, 300),
                           [32761, 32762, 32757, 32758]]).astype(np.uint32)
    for sub in (lens, lens[:3]):  # (3 short records: a log under 4 KiB)
        payload = rng.integers(0, 256, int(sub.astype(np.int64).sum()), dtype=np.uint8)
        buf, poffs, plens = O.wal_frame(payload, sub, recyclable=recyclable, log_number=77)
        wiped = buf.copy()
        for o in poffs:
            wiped[int(o):int(o) + 4] = 0
        offs = poffs.astype(np.int64)
        lengths = plens.astype(np.int32)
        # two headers that do not fit: past the end, and a length overrunning it
        offs = np.concatenate([offs, [len(buf) + 5, int(offs[-1])]])
        lengths = np.concatenate([lengths, [3, len(buf)]]).astype(np.int32)
        dl = d(wiped)
        got = host(engine.wal_record_crc_batch(dl, d(offs), payload_lengths=d(lengths),
                                               recyclable=recyclable))
        assert (host(dl) == buf).all(), len(sub)
        want = [struct.unpack("<I", buf[int(o):int(o) + 4].tobytes())[0] for o in poffs]
        assert got[:len(poffs)].astype(np.uint64).tolist() == want
        assert got[-2:].tolist() == [0, 0]
    # C5 volume of records (the bench's writer call)
    w = workload.make_wal_batch(200_000, workload.SEEDS["C5"], recyclable=recyclable,
                                log_number=77)
    ref = host(w.log)
    o = torch.from_numpy(w.rec_offsets.view(np.int64)).to(DEV)
    wiped = w.log.clone()
    wiped[(o[:, None] + torch.arange(4, device=DEV)[None, :]).reshape(-1)] = 0
    got = engine.wal_record_crc_batch(wiped, o, payload_lengths=d(w.rec_lengths.astype(np.int32)),
                                      recyclable=recyclable)
    assert (host(wiped) == ref).all()
    assert (host(got) == host(engine.wal_record_crc_batch(w.log.clone(), o))).all()


def test_wal_old_record_and_zero_type():
    lens = np.array([100, 200, 300], dtype=np.uint32)
    payload = np.arange(600, dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=True, log_number=5)
    status, nrec, fail, bad = engine.wal_verify_batch(d(buf), log_number=6)
    assert host(status)[0] == 4 and host(nrec)[0] == 0
    z = np.zeros(32768, dtype=np.uint8)
    status, nrec, fail, bad = engine.wal_verify_batch(d(z))
    assert host(status)[0] == 3 and int(host(bad)[0]) == 0


@pytest.mark.parametrize("spec,ctype", [(4096, CT.kCRC32c), ((4096, 16384, 65536), CT.kXXH3),
                                        (("dev", 16384), CT.kCRC32c),
                                        (("dev", 4096), CT.kXXH3),
                                        ((4096, 16384), CT.kxxHash),
                                        (("dev", 4096), CT.kxxHash64)])
def test_sst_batches_vs_oracle(spec, ctype):
    n = 6000
    b = workload.make_sst_batch(n, spec, 0xF0E5700003, ctype=ctype)
    hb = host(b.base)
    offs = host(b.offsets)
    sizes = host(b.sizes).astype(np.uint32)
    comp, st, ok, bad = engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes)
    assert int(host(bad)[0]) == 0
    ocomp, ook, obad = O.block_verify_batch(int(ctype), hb, offs, sizes, nthreads=8)
    assert obad == 0
    assert (host(comp).astype(np.uint64) == ocomp.astype(np.uint64)).all()
    # payload is the splitmix stream of the seed
    import stream as S
    assert (hb[:4096] == S.stream(b.seed, 0, 4096)).all() or sizes[0] < 4096


FULL_SIZE = {  # bench.py CONFIGS: (blocks, size spec, checksum type, seed)
    "C2": (1 << 20, 4096, CT.kCRC32c, workload.SEEDS["C2"]),
    "C3": (1 << 20, (4096, 16384, 65536), CT.kXXH3, workload.SEEDS["C3"]),
    "C4": (1 << 19, 16384, CT.kCRC32c, workload.SEEDS["C4"]),
    "NS16": (1 << 20, 16384, CT.kCRC32c, workload.SEEDS["C2"]),
    "NS16X": (1 << 20, 16384, CT.kXXH3, workload.SEEDS["C2"]),
    # C3's blocks sorted by size: the byte-balanced workgroup ranges
    "C3S": (1 << 20, ("sorted", (4096, 16384, 65536)), CT.kXXH3, workload.SEEDS["C3"]),
    "C3S_CRC": (1 << 20, ("sorted", (4096, 16384, 65536)), CT.kCRC32c, workload.SEEDS["C3"]),
    # kxxHash / kxxHash64 at the benched 1 M x 16 KiB: the lane kernel and its
    # ticket-claimed batch feed (xxhash_legacy.hip), every block vs the oracle
    "NS16H32": (1 << 20, 16384, CT.kxxHash, workload.SEEDS["C2"]),
    "NS16H64": (1 << 20, 16384, CT.kxxHash64, workload.SEEDS["C2"]),
}


@pytest.mark.parametrize("cfg", list(FULL_SIZE))
def test_full_size_properties(cfg):
    """Every bench configuration at its full size (C2 1 M x 4 KiB, C3 1 M
    mixed 4/16/64 KiB XXH3, C4 512 K x 16 KiB, NS16 / NS16X 1 M x 16 KiB
    CRC32C / XXH3), the kernels the bench times: (1) round trip -- trailers
    written by the trailer kernel verify clean, (2) EVERY block's computed
    and stored value against the threaded oracle over a host copy of the
    whole batch (VerifyBlockChecksum, reader_common.cc:26-60), (3) exact
    detection of 64 injected corruptions, at the block start, middle and last
    byte."""
    n, spec, ctype, seed = FULL_SIZE[cfg]
    b = workload.make_sst_batch(n, spec, seed, ctype=ctype)
    comp, st, ok, bad = engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes)
    assert int(host(bad)[0]) == 0
    rng = np.random.default_rng(5)
    offs = host(b.offsets)
    sizes = host(b.sizes).astype(np.int64)
    hb = host(b.base)
    ocomp, ook, obad = O.block_verify_batch(int(ctype), hb, offs, sizes.astype(np.uint32),
                                            nthreads=NT)
    del hb
    assert obad == 0 and ook.all()
    assert np.array_equal(host(comp), ocomp), cfg
    assert np.array_equal(host(st), ocomp), cfg
    victims = rng.choice(n, 64, replace=False)
    pos = offs[victims].astype(np.int64) + np.where(
        np.arange(64) % 3 == 0, 0, np.where(np.arange(64) % 3 == 1, sizes[victims] // 2,
                                             sizes[victims] - 1))
    b.base[torch.from_numpy(pos).to(DEV)] ^= 0x10
    _, _, ok, bad = engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes)
    assert int(host(bad)[0]) == 64
    assert set(np.nonzero(host(ok) == 0)[0].tolist()) == set(victims.tolist())


@pytest.mark.parametrize("ctype", [CT.kCRC32c, CT.kXXH3])
def test_descriptors_in_any_order(ctype):
    """the workgroup ranges come from a counting search over offsets[]: exact
    cover for descriptors in any order (a random permutation of a mixed batch,
    and a reversed one) -- every block verified once, results in place"""
    n = 200_000
    b = workload.make_sst_batch(n, (4096, 16384, 65536), 0xF0E57000C1, ctype=ctype)
    want = host(engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes)[0])
    for perm in (np.random.default_rng(2).permutation(n), np.arange(n)[::-1].copy()):
        p = torch.from_numpy(perm).to(DEV)
        comp, _, ok, bad = engine.block_verify_batch(ctype, b.base, b.offsets[p].contiguous(),
                                                     b.sizes[p].contiguous())
        assert int(host(bad)[0]) == 0 and host(ok).all()
        assert (host(comp) == want[perm]).all()


# ---- a15: Hash64 (XXPH3) and per-KV protection (db/kv_checksum.h) ---------

def test_hash64_golden(golden):
    v, arr, base, offs, lens = golden
    got0 = host(engine.hash64_batch(base, offs, lens)).view(np.uint64)
    assert (got0 == np.array([r["hash64_s0"] for r in v["vectors"]], np.uint64)).all()
    seeds = d(np.full(len(v["vectors"]), O.KV_SEED_V, np.uint64).view(np.int64))
    got1 = host(engine.hash64_batch(base, offs, lens, seeds=seeds)).view(np.uint64)
    assert (got1 == np.array([r["hash64_s1"] for r in v["vectors"]], np.uint64)).all()
    got2 = host(engine.hash64_batch(base, offs, lens, seed=O.KV_SEED_V)).view(np.uint64)
    assert (got2 == got1).all()


def _kv_dev(kd):
    def opt(a, dt):
        return None if a is None else d(a.view(dt))
    return dict(base=d(kd["base"]), ko=d(kd["ko"].view(np.int64)), ks=d(kd["ks"].view(np.int32)),
                vo=d(kd["vo"].view(np.int64)), vs=d(kd["vs"].view(np.int32)),
                co=d(kd["co"].view(np.int64)), ops=opt(kd["ops"], np.uint8),
                seqs=opt(kd["seqs"], np.int64), cfs=opt(kd["cfs"], np.int32))


@pytest.mark.parametrize("prot_bytes,flags", [(8, (True, True, False)), (1, (False, False, False)),
                                              (4, (True, True, True)), (2, (True, False, True))])
def test_kv_protect_and_verify(prot_bytes, flags):
    import kvdata
    kd = kvdata.make_kv(3000, 11 + prot_bytes, prot_bytes, *flags)
    g = _kv_dev(kd)
    prot = engine.kv_protect_batch(g["base"], g["ko"], g["ks"], g["vo"], g["vs"], g["ops"],
                                   g["seqs"], g["cfs"])
    assert (host(prot).view(np.uint64) == kd["prot"]).all()
    comp, ok, bad = engine.kv_verify_batch(g["base"], g["ko"], g["ks"], g["vo"], g["vs"],
                                           prot_bytes, g["co"], g["ops"], g["seqs"], g["cfs"])
    assert int(host(bad)[0]) == 0 and host(ok).all()
    # corrupt key, value and stored checksum bytes of chosen entries
    b2 = kd["base"].copy()
    rng = np.random.default_rng(prot_bytes)
    victims = sorted(set(rng.integers(0, 3000, 30).tolist()))
    hit = set()
    for j, i in enumerate(victims):
        spots = [int(kd["co"][i]) + j % prot_bytes]
        if kd["ks"][i]:
            spots.append(int(kd["ko"][i]) + (j * 31) % int(kd["ks"][i]))
        if kd["vs"][i]:
            spots.append(int(kd["vo"][i]) + (j * 7919) % int(kd["vs"][i]))
        b2[spots[j % len(spots)]] ^= 1 << (j % 8)
        hit.add(i)
    comp, ok, bad = engine.kv_verify_batch(d(b2), g["ko"], g["ks"], g["vo"], g["vs"], prot_bytes,
                                           g["co"], g["ops"], g["seqs"], g["cfs"])
    failed = set(np.nonzero(host(ok) == 0)[0].tolist())
    # a flipped bit in the 1-byte truncation can collide only if the hash byte
    # happens to match; with distinct single-bit flips every victim must fail
    assert failed == hit and int(host(bad)[0]) == len(hit)


def test_kv_out_of_range_and_bad_args():
    base = d(np.zeros(100, np.uint8))
    o = d(np.array([0, 90, 10], np.int64))
    s = d(np.array([10, 20, 5], np.int32))
    c = d(np.array([50, 50, 99], np.int64))
    comp, ok, bad = engine.kv_verify_batch(base, o, s, o, s, 4, c)
    okh = host(ok)
    assert okh[1] == 0 and okh[2] == 0 and int(host(bad)[0]) >= 2
    from forst_amd import ForstError
    with pytest.raises(ForstError):
        engine.kv_verify_batch(base, o, s, o, s, 3, c)


@pytest.mark.parametrize("prot_bytes,flags", [(8, (True, True, False)), (1, (False, False, False)),
                                              (4, (True, True, True)), (2, (True, False, True))])
def test_kv_full_size_roundtrip(prot_bytes, flags):
    """1 M memtable-shaped entries (16-64 B keys, 0-1000 B values, the bench's
    a15 batch), at the four (protection_bytes, op/seq/cf) shapes the reference
    uses: write side computes, EVERY entry's protection is compared with the
    oracle, the read side verifies, 50 injected flips are detected exactly."""
    with_ops, with_seq, with_cf = flags
    n = 1 << 20
    rng = np.random.default_rng(99)
    ks = rng.integers(16, 65, n).astype(np.int64)
    vs = rng.integers(0, 1001, n).astype(np.int64)
    ko = np.zeros(n, np.int64)
    ko[1:] = np.cumsum(ks[:-1] + vs[:-1] + prot_bytes)
    vo = ko + ks
    co = vo + vs
    total = int(co[-1]) + prot_bytes
    alloc = (total + 255) // 256 * 256
    base = torch.empty(alloc, dtype=torch.uint8, device=DEV)
    engine.fill_stream(base, 0, 0xF0E57000A15 + prot_bytes)
    dko, dks, dvo, dvs = d(ko), d(ks.astype(np.int32)), d(vo), d(vs.astype(np.int32))
    hops = rng.integers(0, 26, n).astype(np.uint8) if with_ops else None
    hseq = rng.integers(0, 2**62, n).astype(np.uint64) if with_seq else None
    hcf = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if with_cf else None
    ops = None if hops is None else d(hops)
    seqs = None if hseq is None else d(hseq.view(np.int64))
    cfs = None if hcf is None else d(hcf.view(np.int32))
    prot = engine.kv_protect_batch(base, dko, dks, dvo, dvs, ops, seqs, cfs)
    hb = host(base)
    want = O.kv_protect_batch(hb, ko.view(np.uint64), ks, vo.view(np.uint64), vs, hops, hseq, hcf)
    got = host(prot).view(np.uint64)
    bad_i = np.nonzero(got != want)[0]
    assert len(bad_i) == 0, f"{len(bad_i)} of {n} entries differ, first {bad_i[:8].tolist()}"
    # Encode(prot_bytes): the low LE bytes at co
    pb = prot.view(torch.uint8).view(n, 8)[:, :prot_bytes]
    idx = d(co)[:, None] + torch.arange(prot_bytes, device=DEV)[None, :]
    base[idx.reshape(-1)] = pb.reshape(-1)
    comp, ok, bad = engine.kv_verify_batch(base, dko, dks, dvo, dvs, prot_bytes, d(co), ops, seqs,
                                           cfs)
    assert int(host(bad)[0]) == 0
    assert (host(comp).view(np.uint64) == want).all()
    victims = rng.choice(n, 50, replace=False)
    base[d(ko[victims] + 3)] ^= 0x20
    _, ok, bad = engine.kv_verify_batch(base, dko, dks, dvo, dvs, prot_bytes, d(co), ops, seqs, cfs)
    # a 1-byte truncation lets a flip pass with probability 1/256 (kv_checksum.h:117-133);
    # every detected entry must be a victim, and with 8 bytes all must be
    failed = set(np.nonzero(host(ok) == 0)[0].tolist())
    assert failed <= set(victims.tolist()) and int(host(bad)[0]) == len(failed)
    if prot_bytes >= 4:
        assert failed == set(victims.tolist())


# ---- C5: WAL images built on the device -----------------------------------

@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_batch_matches_oracle_framing(recyclable):
    """make_wal_batch (layout on the host, bytes + CRCs on the GPU) produces
    byte-for-byte the image the oracle's log::Writer restatement frames from
    the same payloads; the reader-side kernel accepts every record."""
    lens = workload.log_uniform_lengths(3000, 32, 32768, 0xF0E5700005)
    lens[:5] = [0, 32761, 32762, 70000, 1]
    w = workload.make_wal_batch(0, 0xF0E5700005, recyclable=recyclable, log_number=0x1234,
                                lengths=lens)
    img = host(w.log)
    hs = 11 if recyclable else 7
    payload = np.concatenate([img[int(o) + hs:int(o) + hs + int(n)]
                              for o, n in zip(w.rec_offsets, w.rec_lengths)])
    buf, oo, ol = O.wal_frame(payload, lens, recyclable=recyclable, log_number=0x1234)
    assert (oo == w.rec_offsets).all()
    assert len(buf) == len(img) and (buf == img).all()
    status, nrec, fail, bad = engine.wal_verify_batch(w.log, log_number=0x1234)
    assert int(host(bad)[0]) == 0 and (host(status) == 0).all()
    assert int(host(nrec).astype(np.int64).sum()) == len(w.rec_offsets)


def test_full_size_c5_properties():
    """C5 at full size (10 M records, ~44 GiB log): every physical record
    verifies, record counts per log block match the writer's layout, 16 sampled
    log blocks agree with the oracle reader, and 48 injected payload flips are
    reported exactly at their blocks and record offsets."""
    n = 10_000_000
    w = workload.make_wal_batch(n, workload.SEEDS["C5"])
    status, nrec, fail, bad = engine.wal_verify_batch(w.log)
    assert int(host(bad)[0]) == 0 and int(host(status).max()) == 0
    per_block = np.bincount((w.rec_offsets // 32768).astype(np.int64),
                            minlength=w.n_log_blocks)
    assert (host(nrec).astype(np.int64) == per_block).all()
    rng = np.random.default_rng(12)
    # every log block against the oracle's per-block reader check
    logh = host(w.log[:w.total])
    ost, onr, ofo = O.wal_verify_blocks(logh, 0, nthreads=NT)
    assert np.array_equal(host(status), ost) and np.array_equal(host(nrec), onr)
    assert np.array_equal(host(fail), ofo)
    cand = np.nonzero(w.rec_lengths > 0)[0]
    victims = rng.choice(cand, 400, replace=False)
    blocks = w.rec_offsets[victims] // 32768
    _, first = np.unique(blocks, return_index=True)
    victims = np.sort(victims[first][:48])
    pos = w.rec_offsets[victims].astype(np.int64) + 7 + \
        rng.integers(0, w.rec_lengths[victims].astype(np.int64))
    w.log[torch.from_numpy(pos).to(DEV)] ^= 0x01
    status, nrec, fail, bad = engine.wal_verify_batch(w.log)
    st = host(status)
    assert int(host(bad)[0]) == len(victims)
    vb = (w.rec_offsets[victims] // 32768).astype(np.int64)
    assert set(np.nonzero(st)[0].tolist()) == set(vb.tolist()) and (st[vb] == 1).all()
    assert (host(fail)[vb].astype(np.int64) == (w.rec_offsets[victims] % 32768)).all()
    logh[pos] ^= 0x01
    ost, onr, ofo = O.wal_verify_blocks(logh, 0, nthreads=NT)
    assert np.array_equal(st, ost) and np.array_equal(host(nrec), onr)
    assert np.array_equal(host(fail), ofo)


# ---- a3: Crc32cCombine and whole-buffer CRC32C ----------------------------

def test_crc32c_buffer_vs_oracle():
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, 5 * 65536 + 1234, dtype=np.uint8)
    dbuf = d(buf)
    for n in (0, 1, 3, 64, 65535, 65536, 65537, 3 * 65536 + 17, len(buf)):
        for init in (0, 0x12345678):
            got = int(host(engine.crc32c_buffer(dbuf[:n], init))[0])
            assert got == O.crc32c_extend(init, buf[:n].tobytes()), (n, init)


def test_crc32c_buffer_large():
    """1 GiB + 3 bytes in one call (16385 chunks through the block kernel)"""
    n = (1 << 30) + 3
    dev = torch.empty(n + 253, dtype=torch.uint8, device=DEV)
    engine.fill_stream(dev, 0, 0xC0FFEE)
    want = O.crc32c_extend(0xFFFF0000, host(dev[:n]).tobytes())
    assert int(host(engine.crc32c_buffer(dev[:n], 0xFFFF0000))[0]) == want


def test_crc32c_combine_batch_vs_oracle():
    rng = np.random.default_rng(78)
    n = 5000
    c1 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    c2 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ln = rng.integers(0, 2**40, n, dtype=np.uint64)
    ln[:6] = [0, 1, 3, 4, 65536, (1 << 63) + 5]
    got = host(engine.crc32c_combine_batch(d(c1.view(np.int32)), d(c2.view(np.int32)),
                                           d(ln.view(np.int64)))).view(np.uint32)
    want = np.array([O.crc32c_combine(int(a), int(b), int(c)) for a, b, c in zip(c1, c2, ln)],
                    np.uint32)
    assert (got == want).all()


# ---- a14: XXH3 of logical WAL records -------------------------------------

@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_record_xxh3(recyclable):
    rng = np.random.default_rng(21)
    lens = workload.log_uniform_lengths(3000, 1, 100000, 0xF0E5700005)
    lens[:5] = [0, 32761, 32762, 65536 * 3, 1]
    payload = rng.integers(0, 256, int(lens.astype(np.int64).sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=recyclable, log_number=77)
    h, first = engine.wal_record_xxh3_batch(d(buf), d(poffs.astype(np.int64)))
    h = host(h).view(np.uint64)
    assert len(h) == len(lens)
    starts = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    want = np.array([O.xxh3_64(payload[starts[j]:starts[j + 1]].tobytes())
                     for j in range(len(lens))], np.uint64)
    assert (h == want).all()


@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_record_xxh3_fragment_edges(recyclable):
    """every boundary placement of tests/walcases.py, 20 rounds (~4800
    records): the in-place fragment-aware kernel and the gathered fallback"""
    import walcases as W
    buf, po, payload, lens, targets = W.frag_edge_log(recyclable, seed=40 + recyclable, repeat=20)
    h, first = engine.wal_record_xxh3_batch(d(buf), d(po.astype(np.int64)))
    assert (host(h).view(np.uint64) == W.expected_hashes(payload, lens)).all()


@pytest.mark.parametrize("recyclable", [False, True])
def test_full_size_c5_writer_crc(recyclable):
    """C5 at full size, the writer's CRC of EVERY physical record (11.4 M,
    log_writer.cc:228-263), both entry points (header offsets; the writer's
    payload lengths), not written in place, against the CRCs the oracle's
    framing stored in the headers: no result store is skipped (the verify
    path pre-fills its results with the stored CRCs, so only a pass that stores
    every CRC shows a record the kernels never reached)"""
    w = workload.make_wal_batch(10_000_000, workload.SEEDS["C5"], recyclable=recyclable,
                                log_number=77)
    o = torch.from_numpy(w.rec_offsets.view(np.int64)).to(DEV)
    stored = (w.log[(o[:, None] + torch.arange(4, device=DEV)[None, :]).reshape(-1)]
              .reshape(-1, 4).to(torch.int64))
    stored = host(stored[:, 0] | (stored[:, 1] << 8) | (stored[:, 2] << 16) | (stored[:, 3] << 24))
    lens = w.rec_lengths
    for kw in ({}, {"payload_lengths": d(lens.astype(np.int32)), "recyclable": recyclable}):
        out = torch.full((len(w.rec_offsets),), 0x5A5A5A5A, dtype=torch.int32, device=DEV)
        got = host(engine.wal_record_crc_batch(w.log, o, write_in_place=False, out=out,
                                               **kw)).view(np.uint32)
        bad = np.nonzero(got.astype(np.int64) != stored)[0]
        assert len(bad) == 0, (len(bad), bad[:8].tolist(), lens[bad[:8]].tolist(),
                               (got[bad[:8]] == 0x5A5A5A5A).tolist())


@pytest.mark.parametrize("recyclable", [False, True])
def test_full_size_c5_record_xxh3(recyclable):
    """10 M logical records of C5 (legacy 7-byte and recyclable 11-byte
    headers): count, first fragments against the writer's layout, and EVERY
    record's hash against the threaded oracle XXH3 over its fragments
    gathered from a host copy of the log (db/log_reader.cc:95-165)"""
    hs = 11 if recyclable else 7
    w = workload.make_wal_batch(10_000_000, workload.SEEDS["C5"], recyclable=recyclable,
                                log_number=0x5EED if recyclable else 0)
    h, first = engine.wal_record_xxh3_batch(w.log, torch.from_numpy(
        w.rec_offsets.view(np.int64)).to(DEV))
    assert h.numel() == w.n_records
    rt = w.rec_types
    starts = np.nonzero((rt == 1) | (rt == 2) | (rt == 5) | (rt == 6))[0]
    assert len(starts) == w.n_records
    assert (host(first) == starts).all()
    logh = host(w.log[:w.total])
    want = O.wal_record_xxh3_batch(logh, w.rec_offsets, w.rec_lengths, starts, hs=hs, nthreads=NT)
    del logh
    assert np.array_equal(host(h).view(np.uint64), want)


def test_c4_full_volume_sharded_on_one_gpu():
    """C4 at its stated volume (BASELINE configs[3]): 64 GiB of 16 KiB kCRC32c
    blocks (4 M descriptors, bench.py describe("C4", 8)), split into the 8
    byte-balanced shards shard.rank_slice gives the ranks of an 8-GPU node
    (db/compaction/compaction_job.cc:1123 -> block_based_table_reader.cc:2491:
    independent blocks, no exchange).  On one MI355X (288 GB) each shard is
    verified in turn exactly as its rank would -- its own view of the buffer
    starting at the shard's first byte, offsets relative to it -- and:
    the shards are the equal contiguous eighths;
    the 8 results concatenated equal one unsplit 4 M-descriptor call; every
    block of every shard matches the threaded oracle on the shard's host copy
    (8 GiB at a time); a
    flip on each side of every shard boundary is reported once, by the
    shard that owns the block, and by the unsplit call."""
    from forst_amd import shard
    world = 8
    n = (1 << 19) * world
    seed = workload.SEEDS["C4"]
    sizes_all = workload.block_sizes(n, 16384, seed)
    b = workload.make_sst_batch(n, 16384, seed, ctype=CT.kCRC32c)
    assert b.total == n * (16384 + 5) and b.total >= 64 << 30
    comp_all, st_all, ok_all, bad_all = engine.block_verify_batch(CT.kCRC32c, b.base, b.offsets,
                                                                  b.sizes)
    assert int(host(bad_all)[0]) == 0
    offs = host(b.offsets)
    slices = [shard.rank_slice(sizes_all, r, world) for r in range(world)]
    assert [s[0] for s in slices] == [r * (n // world) for r in range(world)]  # equal sizes
    assert slices[-1][1] == n and all(slices[r][1] == slices[r + 1][0] for r in range(world - 1))
    rng = np.random.default_rng(44)

    def run_shards(check=False):
        comps, oks, bads = [], [], []
        for lo, hi, start in slices:
            end = int(offs[hi - 1]) + 16384 + 5
            assert start == int(offs[lo])
            # the rank's own buffer: the shard's bytes from its first block on
            # (bench.py run_config: make_sst_batch(..., stream_start=start))
            own = torch.empty((end - start + 255) // 256 * 256, dtype=torch.uint8, device=DEV)
            own[:end - start].copy_(b.base[start:end])
            c, _, ok, bad = engine.block_verify_batch(CT.kCRC32c, own[:end - start],
                                                      b.offsets[lo:hi] - start, b.sizes[lo:hi])
            comps.append(host(c))
            oks.append(host(ok))
            bads.append(int(host(bad)[0]))
            if check:  # every block of the shard against the threaded oracle
                hs_ = host(own[:end - start])
                oc, ook, obad = O.block_verify_batch(
                    int(CT.kCRC32c), hs_, (offs[lo:hi] - start).astype(np.uint64),
                    sizes_all[lo:hi].astype(np.uint32), nthreads=NT)
                del hs_
                assert obad == 0 and np.array_equal(comps[-1], oc), (lo, hi)
            del own
        return np.concatenate(comps), np.concatenate(oks), bads

    comp, ok, bads = run_shards(check=True)
    assert bads == [0] * world and ok.all()
    # a rank generating its shard on its own (bench.py run_config) has those bytes
    lo, hi, start = slices[5]
    rb = workload.make_sst_batch(hi - lo, None, seed, ctype=CT.kCRC32c, sizes=sizes_all[lo:hi],
                                 stream_start=start)
    assert torch.equal(rb.base, b.base[start:start + rb.total])
    del rb
    assert (comp == host(comp_all)).all()
    # a flip in the last block of every shard and the first block of the next
    victims = sorted({s[1] - 1 for s in slices[:-1]} | {s[0] for s in slices[1:]})
    assert len(victims) == 2 * (world - 1)
    pos = offs[victims].astype(np.int64) + np.array([7, 16383] * (world - 1), np.int64)
    b.base[torch.from_numpy(pos).to(DEV)] ^= 0x40
    comp, ok, bads = run_shards()
    assert bads == [1] + [2] * (world - 2) + [1]
    assert np.nonzero(ok == 0)[0].tolist() == victims
    _, _, ok_all, bad_all = engine.block_verify_batch(CT.kCRC32c, b.base, b.offsets, b.sizes)
    assert int(host(bad_all)[0]) == len(victims)
    assert np.nonzero(host(ok_all) == 0)[0].tolist() == victims


def test_wal_block_range_shards_tile_the_log():
    """bench.py's C5 at N GPUs: make_wal_batch(block_range=...) builds a
    rank's contiguous log blocks of one log; the 3 shards concatenated are the
    whole log byte for byte, their records are the log's records, and each
    shard's per-block verify equals the whole log's (log_writer.cc:86-102:
    records never straddle a block)"""
    lengths = workload.log_uniform_lengths(60000, 32, 32768, workload.SEEDS["C5"])
    full = workload.make_wal_batch(0, workload.SEEDS["C5"], lengths=lengths)
    st, nr, fo, bad = engine.wal_verify_batch(full.log)
    assert int(host(bad)[0]) == 0
    nb = full.n_log_blocks
    parts, recs = [], 0
    for r in range(3):
        b0, b1 = nb * r // 3, nb * (r + 1) // 3
        w = workload.make_wal_batch(0, workload.SEEDS["C5"], lengths=lengths, block_range=(b0, b1))
        parts.append(host(w.log))
        s2, n2, f2, bad2 = engine.wal_verify_batch(w.log)
        assert int(host(bad2)[0]) == 0
        assert np.array_equal(host(s2), host(st)[b0:b1]) and np.array_equal(host(n2), host(nr)[b0:b1])
        assert np.array_equal(host(f2), host(fo)[b0:b1])
        assert np.array_equal(w.rec_offsets + np.uint64(b0 * 32768),
                              full.rec_offsets[(full.rec_offsets >= b0 * 32768) &
                                               (full.rec_offsets < b1 * 32768)])
        recs += w.n_records
    assert np.array_equal(np.concatenate(parts), host(full.log))
    assert recs == full.n_records


def test_bench_wal_sharded_runs_at_world_one():
    """bench.py's N-GPU C5 extra (run_wal_sharded) end to end at world 1
    (the driver runs it at N = 2..8): its shard covers the whole log and
    every block verifies"""
    import bench
    r = bench.run_wal_sharded(2, 1, 0, 1, n_per_gpu=200_000)
    assert r["GiBps"] > 0 and 0 < r["roofline_frac_per_gpu"] < 1
