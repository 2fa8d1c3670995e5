"""tests/emu/emu.py -- TEST INFRASTRUCTURE ONLY.

Builds the kernel sources against the SIMT emulator (build_emu.sh) and calls
the same C ABI on host (numpy) buffers, so kernel logic can be checked against
the oracle on a CPU.  Never used by the product.
"""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_libs = {}
_defines = ""  # extra -D options of the build lib() returns (variant())


class variant:
    """with emu.variant("-DFOO=1"): ... -- the calls inside go through a build
    of the kernel sources with those build knobs (built once, cached)"""

    def __init__(self, defines):
        self.defines = defines

    def __enter__(self):
        global _defines
        self.prev, _defines = _defines, self.defines
        return self

    def __exit__(self, *exc):
        global _defines
        _defines = self.prev


def lib():
    L = _libs.get(_defines)
    if L is None:
        tag = abs(hash(_defines)) if _defines else 0
        out = os.path.join(tempfile.gettempdir(), f"libforst_emu_{os.getpid()}_{tag}.so")
        env = dict(os.environ)
        if _defines:
            env["EMU_DEFINES"] = (env.get("EMU_DEFINES", "") + " " + _defines).strip()
        subprocess.check_call([os.path.join(HERE, "build_emu.sh"), out],
                              stdout=subprocess.DEVNULL, env=env)
        L = ctypes.CDLL(out)
        vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        sigs = {
            "forst_last_error": (ctypes.c_char_p, []),
            "forst_block_checksum_batch": (i, [i, vp, u64, vp, vp, vp, vp, vp, u64, vp]),
            "forst_block_trailer_batch": (i, [i, vp, u64, vp, vp, vp, vp, vp, u64, vp]),
            "forst_block_verify_batch": (i, [i, vp, u64, vp, vp, vp, vp, vp, vp, vp, u64, vp]),
                "forst_crc32c_batch": (i, [vp, u64, vp, vp, vp, vp, u64, vp]),
            "forst_crc32c_buffer": (i, [vp, u64, u32, vp, vp]),
            "forst_wal_record_xxh3_batch": (i, [vp, u64, vp, u64, vp, vp, vp, vp]),
            "forst_crc32c_combine": (u32, [u32, u32, u64]),
            "forst_xxh3_64_batch": (i, [vp, u64, vp, vp, vp, u64, vp]),
            "forst_wal_verify_batch": (i, [vp, u64, u64, u64, u32, vp, vp, vp, vp, vp]),
            "forst_wal_record_crc_batch": (i, [vp, u64, vp, u64, i, vp, vp]),
            "forst_wal_record_crc_lengths": (i, [vp, u64, vp, vp, u64, i, i, vp, vp]),
            "forst_hash64_batch": (i, [vp, u64, vp, vp, vp, u64, vp, u64, vp]),
            "forst_kv_protect_batch": (i, [vp, u64, vp, vp, vp, vp, vp, vp, vp, vp, u64, vp]),
            "forst_kv_verify_batch": (i, [vp, u64, vp, vp, vp, vp, vp, vp, vp, u32, vp, vp, vp,
                                          vp, u64, vp]),
            "forst_memtable_verify_batch": (i, [vp, u64, vp, u64, u32, vp, vp, vp, vp]),
            "forst_memtable_protect_batch": (i, [vp, u64, vp, u64, u32, i, vp, vp, vp]),
            "forst_write_batch_protect_batch": (i, [vp, u64, vp, vp, u64, vp, vp, u64, vp, vp,
                                                    vp, vp]),
            "forst_block_kv_checksum_batch": (i, [vp, u64, vp, vp, vp, u64, u32, vp, vp, vp, u64,
                                                  vp, vp, vp]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _libs[_defines] = L
    return L


def _p(a):
    return None if a is None else a.ctypes.data


def _chk(rc):
    if rc != 0:
        raise RuntimeError(lib().forst_last_error().decode())


def _aligned(base):
    """copy into a 16-byte aligned buffer (the C ABI wants 4-byte alignment)"""
    raw = np.zeros(base.nbytes + 64, dtype=np.uint8)
    off = (-raw.ctypes.data) % 16
    a = raw[off:off + base.nbytes]
    a[:] = base
    return a


def block_checksum(ctype, base, offs, sizes, last=None, mods=None):
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    sizes = np.ascontiguousarray(sizes, np.uint32)
    out = np.zeros(len(offs), np.uint32)
    _chk(lib().forst_block_checksum_batch(int(ctype), _p(base), base.nbytes, _p(offs), _p(sizes),
                                          _p(last), _p(mods), _p(out), len(offs), None))
    return out


def block_trailer(ctype, base, offs, sizes, last, mods=None):
    b = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    sizes = np.ascontiguousarray(sizes, np.uint32)
    out = np.zeros(len(offs), np.uint32)
    _chk(lib().forst_block_trailer_batch(int(ctype), _p(b), b.nbytes, _p(offs), _p(sizes),
                                         _p(last), _p(mods), _p(out), len(offs), None))
    return b.copy(), out


def block_verify(ctype, base, offs, sizes, mods=None):
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    sizes = np.ascontiguousarray(sizes, np.uint32)
    n = len(offs)
    comp = np.zeros(n, np.uint32)
    st = np.zeros(n, np.uint32)
    ok = np.zeros(n, np.uint8)
    bad = np.zeros(1, np.uint64)
    _chk(lib().forst_block_verify_batch(int(ctype), _p(base), base.nbytes, _p(offs), _p(sizes),
                                        _p(mods), _p(comp), _p(st), _p(ok), _p(bad), n, None))
    return comp, st, ok, int(bad[0])


def crc32c(base, offs, lens, init=None):
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    out = np.zeros(len(offs), np.uint32)
    _chk(lib().forst_crc32c_batch(_p(base), base.nbytes, _p(offs), _p(lens), _p(init), _p(out),
                                  len(offs), None))
    return out


def xxh3(base, offs, lens):
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    out = np.zeros(len(offs), np.uint64)
    _chk(lib().forst_xxh3_64_batch(_p(base), base.nbytes, _p(offs), _p(lens), _p(out),
                                   len(offs), None))
    return out


def wal_verify(log, log_number=0):
    log = _aligned(log)
    nb = (log.nbytes + 32767) // 32768
    st = np.zeros(nb, np.uint8)
    nrec = np.zeros(nb, np.uint32)
    fail = np.zeros(nb, np.uint32)
    bad = np.zeros(1, np.uint64)
    _chk(lib().forst_wal_verify_batch(_p(log), log.nbytes, 0, nb, log_number, _p(st), _p(nrec),
                                      _p(fail), _p(bad), None))
    return st, nrec, fail, int(bad[0])


def crc32c_buffer(base, init=0):
    base = _aligned(base)
    out = np.zeros(1, np.uint32)
    _chk(lib().forst_crc32c_buffer(_p(base), base.nbytes, init, _p(out), None))
    return int(out[0])


def wal_record_xxh3(log, header_offsets):
    log = _aligned(log)
    offs = np.ascontiguousarray(header_offsets, dtype=np.uint64)
    h = np.zeros(max(1, len(offs)), np.uint64)
    first = np.zeros(max(1, len(offs)), np.uint64)
    nl = ctypes.c_uint64()
    _chk(lib().forst_wal_record_xxh3_batch(_p(log), log.nbytes, _p(offs), len(offs), _p(h),
                                           _p(first), ctypes.byref(nl), None))
    return h[:nl.value], first[:nl.value]


def wal_record_crc(log, header_offsets, write_in_place=True):
    log = _aligned(log)
    offs = np.ascontiguousarray(header_offsets, dtype=np.uint64)
    out = np.zeros(len(offs), np.uint32)
    _chk(lib().forst_wal_record_crc_batch(_p(log), log.nbytes, _p(offs), len(offs),
                                          int(write_in_place), _p(out), None))
    return out, log


def wal_record_crc_lengths(log, header_offsets, payload_lengths, recyclable=False,
                           write_in_place=True, with_out=True):
    log = _aligned(log)
    offs = np.ascontiguousarray(header_offsets, dtype=np.uint64)
    lens = np.ascontiguousarray(payload_lengths, dtype=np.uint32)
    out = np.zeros(len(offs), np.uint32)
    _chk(lib().forst_wal_record_crc_lengths(_p(log), log.nbytes, _p(offs), _p(lens), len(offs),
                                            int(recyclable), int(write_in_place),
                                            _p(out) if with_out else None, None))
    return out, log


def hash64(base, offs, lens, seeds=None, seed=0):
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    sd = None if seeds is None else np.ascontiguousarray(seeds, np.uint64)
    out = np.zeros(len(offs), np.uint64)
    _chk(lib().forst_hash64_batch(_p(base), base.nbytes, _p(offs), _p(lens), _p(sd), seed,
                                  _p(out), len(offs), None))
    return out


def _kv_arrays(ko, ks, vo, vs, ops, seqs, cfs):
    return ([np.ascontiguousarray(ko, np.uint64), np.ascontiguousarray(ks, np.uint32),
             np.ascontiguousarray(vo, np.uint64), np.ascontiguousarray(vs, np.uint32)],
            [None if ops is None else np.ascontiguousarray(ops, np.uint8),
             None if seqs is None else np.ascontiguousarray(seqs, np.uint64),
             None if cfs is None else np.ascontiguousarray(cfs, np.uint32)])


def kv_protect(base, ko, ks, vo, vs, ops=None, seqs=None, cfs=None, misalign=0):
    base = _aligned(base) if not misalign else _aligned(
        np.concatenate([np.zeros(misalign, np.uint8), base]))[misalign:]
    arrs, opt = _kv_arrays(ko, ks, vo, vs, ops, seqs, cfs)
    out = np.zeros(len(arrs[0]), np.uint64)
    _chk(lib().forst_kv_protect_batch(_p(base), base.nbytes, *[_p(a) for a in arrs],
                                      *[_p(a) for a in opt], _p(out), len(out), None))
    return out


def kv_verify(base, ko, ks, vo, vs, prot_bytes, chk, ops=None, seqs=None, cfs=None):
    base = _aligned(base)
    arrs, opt = _kv_arrays(ko, ks, vo, vs, ops, seqs, cfs)
    n = len(arrs[0])
    chk = np.ascontiguousarray(chk, np.uint64)
    comp = np.zeros(n, np.uint64)
    ok = np.zeros(n, np.uint8)
    bad = np.zeros(1, np.uint64)
    _chk(lib().forst_kv_verify_batch(_p(base), base.nbytes, *[_p(a) for a in arrs],
                                     *[_p(a) for a in opt], prot_bytes, _p(chk), _p(comp),
                                     _p(ok), _p(bad), n, None))
    return comp, ok, int(bad[0])


def memtable_verify(base, offs, prot_bytes):
    """-> (computed, status, mismatches)"""
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    comp = np.zeros(len(offs), np.uint64)
    st = np.zeros(len(offs), np.uint8)
    bad = np.zeros(1, np.uint64)
    _chk(lib().forst_memtable_verify_batch(_p(base), base.nbytes, _p(offs), len(offs), prot_bytes,
                                           _p(comp), _p(st), _p(bad), None))
    return comp, st, int(bad[0])


def memtable_protect(base, offs, prot_bytes):
    """-> (buffer with the checksums written in place, values, status)"""
    b = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    out = np.zeros(len(offs), np.uint64)
    st = np.zeros(len(offs), np.uint8)
    _chk(lib().forst_memtable_protect_batch(_p(b), b.nbytes, _p(offs), len(offs), prot_bytes, 1,
                                            _p(out), _p(st), None))
    return b.copy(), out, st


def write_batch_protect(base, offs, lens):
    """-> (prot, first_entry, status, n_protected)"""
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    n = len(offs)
    first = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.uint8)
    nprot = np.zeros(n, np.uint32)
    total = ctypes.c_uint64()
    lib().forst_write_batch_protect_batch(_p(base), base.nbytes, _p(offs), _p(lens), n,
                                          _p(first), None, 0, None, None, ctypes.byref(total),
                                          None)
    prot = np.zeros(max(1, total.value), np.uint64)
    _chk(lib().forst_write_batch_protect_batch(_p(base), base.nbytes, _p(offs), _p(lens), n,
                                               _p(first), _p(prot), total.value, _p(st),
                                               _p(nprot), ctypes.byref(total), None))
    return prot[:total.value], first, st, nprot


def block_kv_checksum(base, offs, sizes, kinds, pb):
    """-> (kv_checksums u8, prot u64, first_key, status)"""
    base = _aligned(base)
    offs = np.ascontiguousarray(offs, np.uint64)
    sizes = np.ascontiguousarray(sizes, np.uint32)
    kinds = np.ascontiguousarray(kinds, np.uint8)
    n = len(offs)
    first = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.uint8)
    total = ctypes.c_uint64()
    lib().forst_block_kv_checksum_batch(_p(base), base.nbytes, _p(offs), _p(sizes), _p(kinds), n,
                                        pb, _p(first), None, None, 0, None, ctypes.byref(total),
                                        None)
    m = total.value
    enc = np.zeros(max(1, m) * pb, np.uint8)
    prot = np.zeros(max(1, m), np.uint64)
    _chk(lib().forst_block_kv_checksum_batch(_p(base), base.nbytes, _p(offs), _p(sizes),
                                             _p(kinds), n, pb, _p(first), _p(enc), _p(prot), m,
                                             _p(st), ctypes.byref(total), None))
    return enc[:m * pb], prot[:m], first, st


def wal_recover(log, log_number=0, mode=2, cap=None):
    """forst_wal_recover_batch on the SIMT emulator: (records, reports, result)
    with records = (offset, length, hash, n_fragments) arrays, reports =
    (offset, bytes, reason, type) arrays"""
    from forst_amd.engine import WalRecords, WalReports, WalRecoverResult, _recover_sig
    L = lib()
    _recover_sig(L)
    log = _aligned(log)
    cap = cap or max(64, log.nbytes // 7 + 2)
    ro, rl, rh = (np.zeros(cap, np.uint64) for _ in range(3))
    rn = np.zeros(cap, np.uint32)
    po, pb = np.zeros(cap, np.uint64), np.zeros(cap, np.uint64)
    pr, pt = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    res = WalRecoverResult()
    rc = L.forst_wal_recover_batch(_p(log), log.nbytes, log_number, mode,
                                   WalRecords(_p(ro), _p(rl), _p(rh), _p(rn)), cap,
                                   WalReports(_p(po), _p(pb), _p(pr), _p(pt)), cap,
                                   ctypes.byref(res), None)
    _chk(rc)
    n, m = res.n_records, res.n_reports
    return (ro[:n], rl[:n], rh[:n], rn[:n]), (po[:m], pb[:m], pr[:m], pt[:m]), res
