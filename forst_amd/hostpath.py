"""Host-memory batches over the GPUs of one process (forst_amd/csrc/host_batch.cc).

ForSt runs in one process (DB::VerifyChecksum, db/db_impl/db_impl.cc:6254)
and its blocks start in host memory -- the table builder's buffer, a
FilePrefetchBuffer or an mmap'd SST file (env/io_posix.cc:958).  These calls
take numpy (host) arrays and a device list: the engine cuts the blocks into
byte-balanced contiguous ranges, one host thread + HIP stream + pinned staging
per device, and returns the per-block results in host arrays.
"""
import ctypes
import mmap
import os

import numpy as np

from ._lib import ForstError, lib


def _check(rc):
    if rc != 0:
        raise ForstError(f"forst host call failed ({rc}): "
                         f"{lib().forst_host_last_error().decode(errors='replace')}")


def _arr(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _ptr(a):
    return None if a is None else a.ctypes.data


def _base_ptr(base):
    if isinstance(base, np.ndarray):
        return base.ctypes.data, base.nbytes
    if isinstance(base, MappedFile):
        return base.address, base.size
    raise TypeError("base must be a numpy uint8 array or a MappedFile")


def partition_bytes(sizes, parts):
    """forst_partition_bytes: cuts[0..parts] of byte-balanced contiguous parts"""
    s = _arr(sizes, np.uint32)
    cuts = np.zeros(parts + 1, np.uint64)
    _check(lib().forst_partition_bytes(_ptr(s), len(s), parts, _ptr(cuts)))
    return cuts


def block_verify_host(ctype, base, offsets, sizes, modifiers=None, devices=(0,)):
    """VerifyBlockChecksum per block of a host batch on the given devices.
    Returns (computed, stored, ok, mismatches)."""
    offs = _arr(offsets, np.uint64)
    sz = _arr(sizes, np.uint32)
    mods = None if modifiers is None else _arr(modifiers, np.uint32)
    n = len(offs)
    comp = np.zeros(n, np.uint32)
    st = np.zeros(n, np.uint32)
    ok = np.zeros(n, np.uint8)
    bad = ctypes.c_uint64()
    dev = _arr(devices, np.int32)
    bp, blen = _base_ptr(base)
    _check(lib().forst_block_verify_host(int(ctype), bp, blen, _ptr(offs), _ptr(sz), _ptr(mods),
                                         _ptr(comp), _ptr(st), _ptr(ok), ctypes.byref(bad), n,
                                         _ptr(dev), len(dev)))
    return comp, st, ok, bad.value


def block_checksum_host(ctype, base, offsets, sizes, last_bytes=None, modifiers=None,
                        devices=(0,)):
    """ComputeBuiltinChecksumWithLastByte + modifier per block of a host batch."""
    offs = _arr(offsets, np.uint64)
    sz = _arr(sizes, np.uint32)
    lb = None if last_bytes is None else _arr(last_bytes, np.uint8)
    mods = None if modifiers is None else _arr(modifiers, np.uint32)
    out = np.zeros(len(offs), np.uint32)
    dev = _arr(devices, np.int32)
    bp, blen = _base_ptr(base)
    _check(lib().forst_block_checksum_host(int(ctype), bp, blen, _ptr(offs), _ptr(sz), _ptr(lb),
                                           _ptr(mods), _ptr(out), len(offs), _ptr(dev),
                                           len(dev)))
    return out


def wal_verify_host(log, log_number=0, devices=(0,)):
    """forst_wal_verify_batch over a log in host memory (numpy uint8 array or a
    MappedFile), its log blocks split over `devices`: per 32 KiB log block
    (status, verified records, failing offset) and the failing-block count
    (db/log_reader.cc:450-531)."""
    bp, blen = _base_ptr(log)
    nb = (blen + 32767) // 32768
    st = np.zeros(nb, np.uint8)
    nr = np.zeros(nb, np.uint32)
    fo = np.zeros(nb, np.uint32)
    bad = ctypes.c_uint64()
    dev = _arr(devices, np.int32)
    _check(lib().forst_wal_verify_host(bp, blen, log_number, _ptr(st), _ptr(nr), _ptr(fo),
                                       ctypes.byref(bad), _ptr(dev), len(dev)))
    return st, nr, fo, bad.value


class MappedFile:
    """A read-only mmap of a file (as PosixMmapReadableFile, env/io_posix.cc:958),
    optionally hipHostRegister'd so the host-memory calls read it by DMA."""

    def __init__(self, path, register=True):
        self.size = os.path.getsize(path)
        self._fd = os.open(path, os.O_RDONLY)
        self._mm = mmap.mmap(self._fd, self.size, prot=mmap.PROT_READ,
                             flags=mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0))
        self._view = np.frombuffer(self._mm, dtype=np.uint8)  # no copy
        self.address = self._view.ctypes.data
        self.registered = False
        self.register_error = None
        if register:
            rc = lib().forst_host_register(self.address, self.size)
            if rc == 0:
                self.registered = True
            else:
                self.register_error = lib().forst_host_last_error().decode(errors="replace")

    def view(self):
        return self._view

    def close(self):
        if self.registered:
            lib().forst_host_unregister(self.address)
            self.registered = False
        self._view = None
        self._mm.close()
        os.close(self._fd)


def context_stats():
    """(contexts, device bytes, pinned bytes) held by the host path's
    per-device context pool (forst_host_context_stats)"""
    c, d, p = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().forst_host_context_stats(ctypes.byref(c), ctypes.byref(d), ctypes.byref(p)))
    return c.value, d.value, p.value


def context_trim():
    """give the buffers of every idle context back to the driver
    (forst_host_context_trim); returns the bytes released"""
    r = ctypes.c_uint64()
    _check(lib().forst_host_context_trim(ctypes.byref(r)))
    return r.value


def aux_stream_stats():
    """(live, idle): the WAL calls' second streams in the per-device pool
    (forst_aux_stream_stats); forst_host_context_trim destroys the idle ones"""
    live, idle = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().forst_aux_stream_stats(ctypes.byref(live), ctypes.byref(idle)))
    return live.value, idle.value
