#!/usr/bin/env python3
"""tests/golden/gen_golden.py -- TEST INFRASTRUCTURE ONLY: makes the fixtures.

Two kinds of fixture, both pure data (inputs + expected outputs):

1. Known-answer vectors transcribed from the reference's own tests
   (`kat_reference_tests.json`):
     * table/table_test.cc:2312-2398  ComputeBuiltinChecksum schema KATs
     * util/crc32c_test.cc:26-110      RFC3720 B.4 + folly 3-way table over the
                                       FNV-filled buffer (generator :173-212)
     * util/hash_test.cc:162-232       Hash64 (XXPH3) small-value schema
   These need nothing but this script.

2. Random vectors computed by the REAL reference (`ref_vectors.json`;
   inputs regenerated from a splitmix64 stream by tests/golden/stream.py): the
   reference's checksum sources (util/crc32c.cc, util/xxhash.cc, util/hash.cc,
   util/coding.cc, table/format.cc) plus tests/golden/ref_shim.cc are
   compiled where they lie under /root/reference into a temporary directory
   OUTSIDE the repository, called through ctypes, and deleted.  Only the
   resulting numbers are committed.  Python `xxhash` (libxxhash 0.8.2) is used
   as an independent cross-check of every XXH3/XXH32/XXH64 value.

Re-run:  python tests/golden/gen_golden.py   (needs /root/reference + g++)
"""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import stream  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("FORST_REFERENCE", "/root/reference")

# --------------------------------------------------------------------------
# 1. KATs transcribed from the reference tests
# --------------------------------------------------------------------------

# table/table_test.cc:2326-2393; values are the little-endian trailer bytes.
TABLE_TEST_KAT = {
    "inputs": {
        "empty": "",
        "b0": "x",
        "b1": "This is a short block!x",
        "b2": "This is a long block!" * 100 + "x",
    },
    # (input, last byte) order of the EXPECT_EQ lines; last byte replaces the
    # trailing 'x': kNoCompression=0, kSnappyCompression=1, kZSTD=7
    "cases": [["empty", None]] + [[b, ct] for b in ("b0", "b1", "b2") for ct in (0, 1, 7)],
    "expected_hex": {
        "0": ["00000000"] * 10,
        "1": ["D8EA82A2", "D28F2549", "052B2843", "46F8F711", "583F0355", "2F9B0A57",
              "ECE7DA1D", "943EF0AB", "43A2EDB1", "00E53D63"],
        "2": ["055DCC02", "3EB065CF", "31F79238", "320D2E00", "4A2E5FB0", "0BD9F652",
              "B4107E50", "20F4D4BA", "8F1A1F99", "A191A338"],
        "3": ["99E9D851", "682705DB", "30E7211B", "B7BB58E8", "B74655EF", "B6C8BBBE",
              "AED9E3B4", "0D4999FE", "F5932423", "6B31BAB1"],
        "4": ["00000000", "C294D338", "1B174353", "2D0E20C8", "B37FB5E6", "6AFC258D",
              "5CE54616", "FA2D482E", "23AED845", "15B7BBDE"],
    },
}

# util/crc32c_test.cc:67-88 (RFC3720 B.4) and :30-61 (folly table, ~crc).
CRC32C_TEST_KAT = {
    "rfc3720": [
        {"desc": "32 x 0x00", "hex": "00" * 32, "crc": 0x8A9136AA},
        {"desc": "32 x 0xff", "hex": "ff" * 32, "crc": 0x62A8AB43},
        {"desc": "0..31", "hex": bytes(range(32)).hex(), "crc": 0x46DD794E},
        {"desc": "31..0", "hex": bytes(range(31, -1, -1)).hex(), "crc": 0x113FDB5C},
        {"desc": "iSCSI PDU", "hex": (
            "01c00000000000000000000000000000"
            "14000000000004000000001400000018"
            "28000000000000000200000000000000"), "crc": 0xD9963A56},
    ],
    "buffer_size": 512 * 1024 * 8,
    # (offset, length, ~crc32c) -- test compares Value(...) == ~expected
    "folly": [
        [0, 0, 0xFFFFFFFF],
        [8, 1, 1543413366], [8, 2, 523493126], [8, 3, 1560427360],
        [8, 4, 3422504776], [8, 5, 447841138], [8, 6, 3910050499],
        [8, 7, 3346241981],
        [9, 1, 3855826643], [10, 2, 560880875], [11, 3, 1479707779],
        [12, 4, 2237687071], [13, 5, 4063855784], [14, 6, 2553454047],
        [15, 7, 1349220140],
        [8, 8, 627613930], [8, 9, 2105929409], [8, 10, 2447068514],
        [8, 11, 863807079], [8, 12, 292050879], [8, 13, 1411837737],
        [8, 14, 2614515001], [8, 15, 3579076296], [8, 16, 2897079161],
        [8, 17, 675168386],
        [0, 512 * 1024 * 8, 2096790750],
        [1, 512 * 1024 * 8 // 2, 3854797577],
    ],
}

# util/hash_test.cc:165-232 Hash64(s, n, 0)
HASH64_KAT = [
    ["", 5999572062939766020], ["08", 583283813901344696],
    ["17", 16175549975585474943], ["9a", 16322991629225003903],
    ["1c", 13269285487706833447], ["4d76", 6859542833406258115],
    ["52d5", 4919611532550636959], ["91f7", 14199427467559720719],
    ["d627", 12292689282614532691], ["30460b", 11404699285340020889],
    ["56dcd6", 12404347133785524237], ["d45233", 15853805298481534034],
    ["6ab5f4", 16863488758399383382], ["6753811c", 9010661983527562386],
    ["69b8c088", 6611781377647041447], ["1e84af2d", 15290969111616346501],
    ["46dc54be", 7063754590279313623], ["d07a6eea56", 6384167718754869899],
    ["8683d5a4d8", 16874407254108011067], ["b746bb77ce", 16809880630149135206],
    ["6ca8bce599", 1249038833153141148], ["5c5ee1a07381", 17358142495308219330],
    ["085d731ce52e", 4237646583134806322], ["42fbf252b410", 4373664924115234051],
    ["73e1ff569cce", 12012981210634596029], ["5cbe9775549a52", 5716522398211028826],
    ["16823949882b36", 15604531309862565013], ["5977f0a724f478", 8601330687345614172],
    ["d3a57c0ec00207", 8088079329364056942], ["311b98759622d39a", 9844314944338447628],
    ["38d6f72820b48ae9", 10973293517982163143], ["bb185df41203f799", 9986007080564743219],
    ["80d43b3bae22a278", 1729303145008254458], ["1ab5d0feabc361b299", 13253403748084181481],
    ["8e4ac318202f06e63c", 7768754303876232188], ["b6c0dd053fc4864cef", 12439346786701492],
    ["9a5f780daf50e11f55", 10841838338450144690],
    ["226f391ff8dd4f521794", 12883919702069153152],
    ["32892a75483a4a0269dd", 12692903507676842188],
    ["06925cf4880e7e68383e", 6540985900674032620],
    ["bd2c6338bfe978b7bf15", 10551812464348219044],
]


def fnv_buffer(size):
    """util/crc32c_test.cc:173-212: word 0 = 0; word i = fnv64 of the 8 bytes
    of word i-1 (as signed chars), little-endian."""
    M = (1 << 64) - 1
    out = bytearray(size)
    prev = bytes(8)
    for i in range(1, size // 8):
        h = 14695981039346656037
        for c in prev:
            h = (h + (h << 1) + (h << 4) + (h << 5) + (h << 7) + (h << 8) + (h << 40)) & M
            sc = c - 256 if c >= 128 else c
            h = (h ^ (sc & M)) & M
        prev = h.to_bytes(8, "little")
        out[8 * i:8 * i + 8] = prev
    return bytes(out)


# --------------------------------------------------------------------------
# 2. Vectors from the compiled reference (built outside the repo)
# --------------------------------------------------------------------------
REF_SRCS = ["util/crc32c.cc", "util/xxhash.cc", "util/hash.cc", "util/coding.cc",
            "table/format.cc"]


def build_reference(tmpdir):
    out = os.path.join(tmpdir, "libforst_ref.so")
    cmd = (["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-march=native",
            "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections",
            "-Wl,--no-undefined", "-DROCKSDB_PLATFORM_POSIX", "-DOS_LINUX", "-DNDEBUG", "-DNPERF_CONTEXT",
            "-fvisibility=hidden", "-fvisibility-inlines-hidden",
            "-w", f"-I{REF}", f"-I{REF}/include", "-o", out]
           + [os.path.join(REF, s) for s in REF_SRCS]
           + [os.path.join(HERE, "ref_shim.cc"), "-lpthread"])
    subprocess.check_call(cmd)
    L = ctypes.CDLL(out)
    u32, u64, sz, vp, i = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t,
                           ctypes.c_void_p, ctypes.c_int)
    sigs = {
        "ref_crc32c_extend": (u32, [u32, vp, sz]),
        "ref_crc32c_value": (u32, [vp, sz]),
        "ref_crc32c_combine": (u32, [u32, u32, sz]),
        "ref_crc32c_mask": (u32, [u32]),
        "ref_xxh3_64": (u64, [vp, sz]),
        "ref_xxh32": (u32, [vp, sz, u32]),
        "ref_xxh64": (u64, [vp, sz, u64]),
        "ref_hash64": (u64, [vp, sz, u64]),
        "ref_compute_builtin_checksum": (u32, [i, vp, sz]),
        "ref_compute_builtin_checksum_with_last_byte": (u32, [i, vp, sz, ctypes.c_char]),
        "ref_checksum_modifier_for_context": (u32, [u32, u64]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def edge_lengths():
    ls = set(range(0, 80))
    for b in (128, 240, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536):
        for d in (-65, -64, -63, -17, -16, -9, -8, -5, -4, -3, -2, -1, 0, 1, 2, 3, 4, 5,
                  7, 8, 9, 15, 16, 17, 63, 64, 65):
            if 0 <= b + d <= 70000:
                ls.add(b + d)
    return sorted(ls)


def make_ref_vectors(L):
    rng = np.random.default_rng(0xF0E57000)
    lengths = edge_lengths()
    lengths += [int(x) for x in rng.integers(0, 70000, 64)]
    total = sum(l + 5 + 2 for l in lengths) + 64
    raw = stream.golden_blob(total)
    base = ctypes.c_char_p(raw)
    bp = ctypes.cast(base, ctypes.c_void_p).value
    import xxhash

    vecs = []
    off = 0
    for k, n in enumerate(lengths):
        # unaligned starts on purpose: advance by n+5 like an SST (table.h trailer)
        p = bp + off
        d = raw[off:off + n]
        rec = {"off": off, "n": n,
               "crc32c": L.ref_crc32c_value(p, n),
               "xxh3": L.ref_xxh3_64(p, n),
               "xxh32": L.ref_xxh32(p, n, 0),
               "xxh64": L.ref_xxh64(p, n, 0),
               "hash64_s0": L.ref_hash64(p, n, 0),
               "hash64_s1": L.ref_hash64(p, n, 0xD28AAD72F49BD50B),
               "builtin": [L.ref_compute_builtin_checksum(t, p, n) for t in range(5)],
               "builtin_plus1": [L.ref_compute_builtin_checksum(t, p, n + 1) for t in range(5)],
               "with_last": [L.ref_compute_builtin_checksum_with_last_byte(
                   t, p, n, bytes([raw[off + n]])) for t in range(5)]}
        assert rec["xxh3"] == xxhash.xxh3_64_intdigest(d)
        assert rec["xxh32"] == xxhash.xxh32_intdigest(d)
        assert rec["xxh64"] == xxhash.xxh64_intdigest(d)
        vecs.append(rec)
        off += n + 5
        off += k % 3  # vary alignment further
    # context modifiers (table/format.h:119)
    mods = []
    for base_ctx in (0, 1, 0x12345678, 0xFFFFFFFF, 0x9E3779B1):
        for o in (0, 1, 4096, 0xFFFFFFFF, 0x100000000, 0x123456789ABC, (1 << 64) - 1):
            mods.append([base_ctx, o, L.ref_checksum_modifier_for_context(base_ctx, o)])
    # WAL record CRC: log_test.cc:231-238 FixChecksum restates it as
    # Mask(Value(header[6] .. payload)); compute with the reference crc32c.
    wal = []
    for rtype in (1, 2, 3, 4, 5, 6, 7, 8):
        for n in (0, 1, 7, 100, 32761):
            payload = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            recyc = rtype >= 5
            lognum = 0xC0FFEE if recyc else 0
            hdr_tail = bytes([rtype]) + (lognum.to_bytes(4, "little") if recyc else b"")
            buf = hdr_tail + payload
            crc = L.ref_crc32c_mask(L.ref_crc32c_value(ctypes.c_char_p(buf), len(buf)))
            wal.append({"type": rtype, "log_number": lognum, "payload_hex": payload.hex(),
                        "masked_crc": crc})
    # per-KV protection fields (db/kv_checksum.h:84-88, :296-460): NPHash64 of
    # the op type (1 byte), sequence number (8 bytes LE) and column family id
    # (4 bytes LE) with their seeds, by the reference's Hash64 (util/hash.cc:81)
    kv = {"op": [], "seq": [], "cf": []}
    for op in range(0, 32):
        b = bytes([op])
        kv["op"].append([op, L.ref_hash64(ctypes.c_char_p(b), 1, 0xA5155AE5E937AA16)])
    for seq in [0, 1, 2, 255, 256, 0x123456789A, (1 << 56) - 1, (1 << 64) - 1] + \
            [int(x) for x in rng.integers(0, 2**63, 24)]:
        b = seq.to_bytes(8, "little")
        kv["seq"].append([seq, L.ref_hash64(ctypes.c_char_p(b), 8, 0x77A00858DDD37F21)])
    for cf in [0, 1, 2, 7, 0xFFFFFFFF] + [int(x) for x in rng.integers(0, 2**32, 11)]:
        b = cf.to_bytes(4, "little")
        kv["cf"].append([cf, L.ref_hash64(ctypes.c_char_p(b), 4, 0x4A2AB5CBD26F542C)])
    return raw, {"blob_bytes": total,
                 "lengths_note": "vectors[i] covers stream.golden_blob(blob_bytes)[off:off+n]",
                 "vectors": vecs, "modifiers": mods, "wal": wal, "kv_fields": kv}


def main():
    with open(os.path.join(HERE, "kat_reference_tests.json"), "w") as f:
        json.dump({"table_test": TABLE_TEST_KAT, "crc32c_test": CRC32C_TEST_KAT,
                   "hash_test": HASH64_KAT}, f, indent=1)
    if not os.path.isdir(REF):
        print("reference tree absent; only KAT fixture written")
        return
    tmp = tempfile.mkdtemp(prefix="forst_ref_")
    try:
        L = build_reference(tmp)
        raw, vec = make_ref_vectors(L)
        # check the FNV buffer + folly table with the reference itself
        buf = fnv_buffer(CRC32C_TEST_KAT["buffer_size"])
        for off, n, inv in CRC32C_TEST_KAT["folly"]:
            v = L.ref_crc32c_value(ctypes.c_char_p(buf[off:off + n] or b"\0"), n)
            assert v == (~inv & 0xFFFFFFFF), (off, n)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    with open(os.path.join(HERE, "ref_vectors.json"), "w") as f:
        json.dump(vec, f)
    print(f"wrote {len(vec['vectors'])} vectors, {len(raw)} input bytes")


if __name__ == "__main__":
    sys.exit(main())
