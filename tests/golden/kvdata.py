"""tests/golden/kvdata.py -- TEST INFRASTRUCTURE ONLY: memtable-shaped per-KV
protection batches (db/memtable.cc:273-307 layout: key, value, then the
protection_bytes checksum right after the value), checksums written with the
oracle (the parity checker)."""
import numpy as np

from oracle import oracle as O

EDGE = [0, 1, 2, 3, 4, 5, 8, 9, 16, 17, 32, 33, 64, 65, 96, 97, 128, 129, 239, 240, 241,
        255, 256, 1023, 1024, 1025, 1087, 1088, 2048, 2049, 3000, 4096, 5000]


def make_kv(n, seed, prot_bytes=8, with_ops=True, with_seq=True, with_cf=False):
    rng = np.random.default_rng(seed)
    ks = rng.integers(0, 300, n).astype(np.uint32)
    vs = rng.integers(0, 5000, n).astype(np.uint32)
    ks[:len(EDGE)] = [e % 300 for e in EDGE]
    vs[:len(EDGE)] = EDGE
    vs[len(EDGE):2 * len(EDGE)] = EDGE[::-1]
    ks[len(EDGE):2 * len(EDGE)] = np.minimum(np.array(EDGE[::-1]), 2000)
    gaps = rng.integers(0, 8, n)
    ko = np.zeros(n, np.uint64)
    vo = np.zeros(n, np.uint64)
    co = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        ko[i] = pos
        pos += int(ks[i]) + 1  # + a varint-ish separator byte
        vo[i] = pos
        pos += int(vs[i])
        co[i] = pos
        pos += prot_bytes
    base = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    ops = rng.integers(0, 26, n).astype(np.uint8) if with_ops else None
    seqs = rng.integers(0, 2**63, n, dtype=np.uint64) if with_seq else None
    cfs = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if with_cf else None
    prot = O.kv_protect_batch(base, ko, ks, vo, vs, ops, seqs, cfs)
    for i in range(n):  # ProtectionInfo::Encode (kv_checksum.h:97-115): low bytes, LE
        base[int(co[i]):int(co[i]) + prot_bytes] = np.frombuffer(
            int(prot[i]).to_bytes(8, "little")[:prot_bytes], np.uint8)
    return dict(base=base, ko=ko, ks=ks, vo=vo, vs=vs, co=co, ops=ops, seqs=seqs, cfs=cfs,
                prot=prot, prot_bytes=prot_bytes)
