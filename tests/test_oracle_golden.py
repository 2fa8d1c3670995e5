"""Pin the CPU oracle (oracle/oracle.c) before trusting it.

* against the reference's own known-answer tests (table_test.cc:2312-2398,
  crc32c_test.cc:26-110, hash_test.cc:162-232 where covered), and
* against vectors produced by the real reference code (tests/golden/gen_golden.py).
"""
import struct

import numpy as np
import pytest

from oracle import oracle as O


def _le_hex(v):
    return struct.pack("<I", v).hex().upper()


def test_table_test_schema_kats(kats):
    k = kats["table_test"]
    for t_str, expected in k["expected_hex"].items():
        t = int(t_str)
        got = []
        for name, ct in k["cases"]:
            data = k["inputs"][name].encode()
            if ct is not None:
                data = data[:-1] + bytes([ct])
            v = O.compute_builtin_checksum(t, data)
            if len(data) >= 1:
                # format.h:300-306 consistency rule
                assert v == O.compute_builtin_checksum_with_last_byte(t, data[:-1], data[-1])
            got.append(_le_hex(v))
        assert got == expected, f"type {t}"


def test_crc32c_rfc3720(kats):
    for case in kats["crc32c_test"]["rfc3720"]:
        assert O.crc32c_value(bytes.fromhex(case["hex"])) == case["crc"], case["desc"]


def test_crc32c_folly_table(kats):
    from gen_golden import fnv_buffer

    k = kats["crc32c_test"]
    buf = np.frombuffer(fnv_buffer(k["buffer_size"]), dtype=np.uint8)
    for off, n, inv in k["folly"]:
        seg = buf[off:off + n]
        want = (~inv) & 0xFFFFFFFF
        assert O.crc32c_value(seg) == want, (off, n)
        assert O.crc32c_extend(0, seg, fast=True) == want, (off, n)
        # stitching (crc32c_test.cc:100-109)
        half = n // 2
        part = O.crc32c_value(seg[:half])
        assert O.crc32c_extend(part, seg[half:]) == want


def test_crc32c_mask_extend_combine():
    assert O.crc32c_extend(O.crc32c_value(b"hello "), b"world") == O.crc32c_value(b"hello world")
    c = O.crc32c_value(b"foo")
    assert O.unmask(O.mask(c)) == c and O.mask(c) != c
    assert O.unmask(O.unmask(O.mask(O.mask(c)))) == c
    a, b = O.crc32c_value(b"hello "), O.crc32c_value(b"world")
    assert O.crc32c_combine(a, b, 5) == O.crc32c_value(b"hello world")
    assert O.crc32c_combine(b, a, 6) != O.crc32c_value(b"hello world")
    rng = np.random.default_rng(5)
    s1 = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    c1 = O.crc32c_value(s1)
    for n in list(range(0, 300)) + [4095, 4096, 65537]:
        s2 = rng.integers(0, 256, n, dtype=np.uint8)
        assert O.crc32c_combine(c1, O.crc32c_value(s2), n) == O.crc32c_extend(c1, s2)


def test_oracle_vs_reference_vectors(ref_vectors):
    v, blob = ref_vectors
    arr = np.frombuffer(blob, dtype=np.uint8)
    for rec in v["vectors"]:
        off, n = rec["off"], rec["n"]
        d = arr[off:off + n]
        assert O.crc32c_value(d) == rec["crc32c"], n
        assert O.crc32c_extend(0, d, fast=True) == rec["crc32c"], n
        assert O.xxh3_64(d) == rec["xxh3"], n
        assert O.xxh32(d) == rec["xxh32"], n
        assert O.xxh64(d) == rec["xxh64"], n
        for t in range(5):
            assert O.compute_builtin_checksum(t, d) == rec["builtin"][t], (t, n)
            assert O.compute_builtin_checksum(t, arr[off:off + n + 1]) == rec["builtin_plus1"][t]
            assert O.compute_builtin_checksum_with_last_byte(t, d, int(arr[off + n])) == \
                rec["with_last"][t], (t, n)


def test_context_modifier(ref_vectors):
    v, _ = ref_vectors
    for base, off, want in v["modifiers"]:
        assert O.checksum_modifier_for_context(base, off) == want


def test_wal_record_crc(ref_vectors):
    v, _ = ref_vectors
    for w in v["wal"]:
        payload = bytes.fromhex(w["payload_hex"])
        assert O.wal_record_crc(w["type"], w["log_number"], payload) == w["masked_crc"]


def test_zero_inputs_never_zero():
    # table_test.cc:2400-2435 (lengths < 20000; only XXH3 len 0 is exempt)
    zeros = np.zeros(20000, dtype=np.uint8)
    for t in (1, 2, 3, 4):
        for n in list(range(0, 300)) + list(range(4000, 4200)) + [16385, 19999]:
            v = O.compute_builtin_checksum(t, zeros[:n])
            if t == 4 and n == 0:
                continue
            assert v != 0, (t, n)


def test_batch_helpers_match_scalar():
    rng = np.random.default_rng(9)
    sizes = rng.integers(0, 5000, 200).astype(np.uint32)
    offs = np.zeros(200, dtype=np.uint64)
    offs[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5)
    total = int(offs[-1]) + int(sizes[-1]) + 5
    base = rng.integers(0, 256, total, dtype=np.uint8)
    for t in (1, 2, 3, 4):
        out = O.block_checksum_batch(t, base, offs, sizes, nthreads=3)
        for i in range(0, 200, 7):
            o, n = int(offs[i]), int(sizes[i])
            assert out[i] == O.compute_builtin_checksum(t, base[o:o + n + 1])
        # write trailers, verify all ok, corrupt a few
        for i in range(200):
            o, n = int(offs[i]), int(sizes[i])
            base[o + n + 1:o + n + 5] = np.frombuffer(struct.pack("<I", int(out[i])), np.uint8)
        comp, ok, bad = O.block_verify_batch(t, base, offs, sizes, nthreads=4)
        assert bad == 0 and ok.all()
        assert (comp == out).all()
        o = int(offs[17])
        base[o] ^= 0x40
        comp, ok, bad = O.block_verify_batch(t, base, offs, sizes, nthreads=2)
        assert bad == (1 if sizes[17] > 0 or t in (2, 3) else bad) and not ok[17]
        base[o] ^= 0x40


@pytest.mark.parametrize("recyclable", [False, True])
def test_wal_frame_and_verify(recyclable):
    rng = np.random.default_rng(3)
    lens = np.exp(rng.uniform(np.log(32), np.log(32768), 300)).astype(np.uint32)
    lens[:5] = [0, 1, 32761, 32762, 100000]
    payload = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    buf, poffs, plens = O.wal_frame(payload, lens, recyclable=recyclable, log_number=77)
    n, bad = O.wal_verify(buf, nthreads=3)
    assert bad == 0 and n == len(poffs)
    hs = 11 if recyclable else 7
    # every physical record: CRC restated as log_test.cc FixChecksum does
    for o, l in zip(poffs[:50], plens[:50]):
        o = int(o)
        crc = O.mask(O.crc32c_value(buf[o + 6:o + hs + int(l)]))
        assert struct.unpack("<I", buf[o:o + 4].tobytes())[0] == crc
    # corrupt one payload byte -> exactly that block reports one bad record
    o = int(poffs[10]) + hs
    buf[o] ^= 1
    n2, bad2 = O.wal_verify(buf, nthreads=1)
    assert bad2 == 1


def test_stream_matches_oracle_fill():
    import stream

    for start, n in ((0, 100), (5, 77), (1 << 20, 4099)):
        a = stream.stream(0x1234, start, n)
        b = O.fill_stream(start, n, 0x1234)
        assert (a == b).all()


# ---- a15: Hash64 (XXPH3 0.7.2 preview) and per-KV protection ---------------

def test_hash64_kats(kats):
    # util/hash_test.cc:162-232 Hash64(s, n, 0)
    for hexs, want in kats["hash_test"]:
        assert O.hash64(bytes.fromhex(hexs), 0) == want, hexs


def test_hash64_reference_vectors(ref_vectors):
    # every length class (0-16, 17-128, 129-240, long with/without a last
    # stripe, multiples of 1024) for seed 0 and seed kSeedV, by the reference
    v, blob = ref_vectors
    arr = np.frombuffer(blob, dtype=np.uint8)
    for r in v["vectors"]:
        d = arr[r["off"]:r["off"] + r["n"]]
        assert O.hash64(d, 0) == r["hash64_s0"], r["n"]
        assert O.hash64(d, O.KV_SEED_V) == r["hash64_s1"], r["n"]


def test_kv_field_hashes_reference(ref_vectors):
    # NPHash64 of op type / sequence / column family with their seeds
    # (db/kv_checksum.h:84-88, :296-460), values from the reference's Hash64
    kv = ref_vectors[0]["kv_fields"]
    for op, want in kv["op"]:
        assert O.hash64(bytes([op]), O.KV_SEED_O) == want
    for seq, want in kv["seq"]:
        assert O.hash64(seq.to_bytes(8, "little"), O.KV_SEED_S) == want
    for cf, want in kv["cf"]:
        assert O.hash64(cf.to_bytes(4, "little"), O.KV_SEED_C) == want


def test_kv_protect_composition(ref_vectors):
    # ProtectKVO(k, v, op).ProtectS(seq).ProtectC(cf) == XOR of the field
    # hashes (kv_checksum.h:296-307, :420-460); XOR is an involution, so
    # Strip == Protect (kv_checksum.h:391-470)
    v, blob = ref_vectors
    arr = np.frombuffer(blob, dtype=np.uint8)
    kv = v["kv_fields"]
    for t, r in enumerate(v["vectors"][:120]):
        key = arr[r["off"]:r["off"] + min(r["n"], 40)]
        val = arr[r["off"]:r["off"] + r["n"]]
        op, hop = kv["op"][t % len(kv["op"])]
        seq, hseq = kv["seq"][t % len(kv["seq"])]
        cf, hcf = kv["cf"][t % len(kv["cf"])]
        hk = O.hash64(key, 0)
        assert O.kv_protect(key, val) == hk ^ r["hash64_s1"]
        assert O.kv_protect(key, val, op) == hk ^ r["hash64_s1"] ^ hop
        assert O.kv_protect(key, val, op, seq=seq) == hk ^ r["hash64_s1"] ^ hop ^ hseq
        assert O.kv_protect(key, val, op, seq=seq, cf=cf) == hk ^ r["hash64_s1"] ^ hop ^ hseq ^ hcf


# ---- a15 call sites: the oracle against the reference's own call-site code --
def test_oracle_memtable_entries_vs_reference(kv_sites):
    """MemTable::Add entries and MemTable::VerifyEntryChecksum statuses
    (db/memtable.cc:273-307, :696-732) on intact, corrupted and crafted entries"""
    import kvsites

    meta, arrays = kv_sites
    cases = kvsites.memtable_cases(meta, arrays)
    assert len(cases) == 9
    for name, base, offs, pb, want in cases:
        comp, st = O.memtable_verify_batch(base, len(base), offs, pb)
        got = [O.MEM_STATUS[int(s)] for s in st]
        assert got == want, name
        assert (comp[st == 0] != 0).all()


def test_oracle_write_batch_vs_reference(kv_sites):
    """WriteBatch::Iterate statuses and ProtectionInfoUpdater values
    (db/write_batch.cc:361-716, :3016-3080) on every fixture rep"""
    import kvsites

    base, offs, lens, reps = kvsites.write_batch_case(*kv_sites)
    assert len(reps) > 280
    for (name, status, prot), o, n in zip(reps, offs, lens):
        code, got = O.write_batch_protect(base[int(o):int(o) + int(n)].tobytes())
        assert O.WB_STATUS[code] == status, name
        assert [int(x) for x in prot] == got, name
