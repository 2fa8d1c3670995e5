"""tests/kvsites.py -- TEST INFRASTRUCTURE: the a15 call-site cases of
tests/golden/kv_sites.{json,npz} (reference-made, gen_kv_golden.py) laid out
as the engine's batch calls take them: memtable entry buffers with their
corrupted copies, and the WriteBatch reps back to back."""
import numpy as np


def memtable_cases(meta, arrays):
    """-> [(name, base u8, entry offsets u64, prot_bytes, expected status texts)]
    intact buffers, one per protection size, then each buffer with ALL its
    corruptions applied at once (they hit distinct entries), then the crafted
    headers as one buffer"""
    out = []
    for c in meta["memtable"]["cases"]:
        base = arrays[c["tag"] + "_base"]
        offs = arrays[c["tag"] + "_offs"]
        out.append((c["tag"], base, offs, c["prot_bytes"], ["OK"] * c["n"]))
        b2 = base.copy()
        want = ["OK"] * c["n"]
        for x in c["corrupt"]:
            b2[x["at"]] ^= x["xor"]
            want[x["entry"]] = x["status"]
        out.append((c["tag"] + "_corrupt", b2, offs, c["prot_bytes"], want))
    parts, offs, want, pos = [], [], [], 0
    for x in meta["memtable"]["crafted"]:
        raw = bytes.fromhex(x["hex"])
        parts.append(raw)
        offs.append(pos)
        want.append(x["status"])
        pos += len(raw)
    out.append(("crafted", np.frombuffer(b"".join(parts) + bytes(64), np.uint8).copy(),
                np.array(offs, np.uint64), 8, want))
    return out


def write_batch_case(meta, arrays):
    """-> (base u8, rep offsets u64, rep sizes u32, [(name, status text, prot u64[])])"""
    reps = [(b["name"], b["status"], arrays[f"wb_prot_{i}"]) for i, b in enumerate(meta["writebatch"])]
    return arrays["wb_base"], arrays["wb_offs"], arrays["wb_lens"], reps


def _varint(b, p):
    r = sh = 0
    while True:
        x = int(b[p])
        p += 1
        r |= (x & 127) << sh
        if not x & 128:
            return r, p
        sh += 7


def mem_checksum_pos(base, off):
    """position of a well-formed memtable entry's checksum bytes"""
    ikl, kp = _varint(base, off)
    vl, vp = _varint(base, kp + ikl)
    return vp + vl


def block_case(meta, arrays):
    """-> (base u8, offsets u64, sizes u32, kinds u8, cases): every block of the
    fixture (reference-written SSTs' blocks + crafted damaged ones)"""
    cases = meta["blocks"]
    return (arrays["blk_base"], arrays["blk_offs"],
            np.array([c["size"] for c in cases], np.uint32),
            np.array([c["kind"] for c in cases], np.uint8), cases)
