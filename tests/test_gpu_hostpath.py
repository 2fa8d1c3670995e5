"""In-process multi-device host-memory path (forst_amd/csrc/host_batch.cc):
blocks in host memory -- pageable, pinned, or an mmap'd file registered with
hipHostRegister (PosixMmapReadableFile, env/io_posix.cc:958) -- cut into
byte-balanced per-device ranges, one host thread + HIP stream + pinned staging
per device.  Every result must be bit-identical to the single-device
device-resident call; a device listed twice runs two threads and streams on
one GPU, so the partition and join are exercised on a one-GPU box."""
import numpy as np
import pytest
import torch

from forst_amd import engine, hostpath, workload
from forst_amd.engine import ChecksumType as CT

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)


def batch(n, spec, ctype, seed):
    b = workload.make_sst_batch(n, spec, seed, ctype=ctype)
    return b, b.base.cpu().numpy(), b.offsets.cpu().numpy(), b.sizes.cpu().numpy()


@pytest.mark.parametrize("ctype,spec,devices", [
    (CT.kCRC32c, 4096, (0,)), (CT.kXXH3, (4096, 16384, 65536), (0, 0)),
    (CT.kCRC32c, ("dev", 16384), (0, 0, 0)), (CT.kxxHash64, ("logu", 32, 32768), (0, 0)),
])
def test_verify_host_matches_device_call(ctype, spec, devices):
    b, hb, offs, sizes = batch(30000, spec, ctype, 0xF0E57000AB)
    rng = np.random.default_rng(3)
    victims = np.unique(rng.integers(0, b.n, 25))
    hb = hb.copy()
    hb[offs[victims] + sizes[victims] // 2] ^= 0x04  # payload flips
    dev = torch.from_numpy(hb).cuda()
    comp, st, ok, bad = engine.block_verify_batch(ctype, dev, b.offsets, b.sizes)
    hcomp, hst, hok, hbad = hostpath.block_verify_host(ctype, hb, offs, sizes, devices=devices)
    assert (hcomp == comp.cpu().numpy()).all()
    assert (hst == st.cpu().numpy()).all()
    assert (hok == ok.cpu().numpy()).all()
    assert hbad == int(bad.item()) == len(victims)
    assert set(np.nonzero(hok == 0)[0].tolist()) == set(victims.tolist())


def test_checksum_host_matches_device_call_pinned_and_pageable():
    b, hb, offs, sizes = batch(20000, (4096, 16384), CT.kXXH3, 0xF0E57000AC)
    rng = np.random.default_rng(4)
    last = rng.integers(0, 8, b.n).astype(np.uint8)
    mods = rng.integers(0, 2**32, b.n, dtype=np.uint64).astype(np.uint32)
    want = engine.block_checksum_batch(
        CT.kXXH3, b.base, b.offsets, b.sizes, last_bytes=torch.from_numpy(last).cuda(),
        modifiers=torch.from_numpy(mods.view(np.int32)).cuda()).cpu().numpy()
    got = hostpath.block_checksum_host(CT.kXXH3, hb, offs, sizes, last, mods, devices=(0, 0))
    assert (got == want).all()
    pinned = torch.from_numpy(hb).pin_memory().numpy()  # DMA straight from the pages
    got2 = hostpath.block_checksum_host(CT.kXXH3, pinned, offs, sizes, last, mods, devices=(0,))
    assert (got2 == want).all()


def test_mmap_registered_file(tmp_path):
    """an SST-shaped file mmap'd read-only and registered (or staged when the
    driver refuses to pin the mapping): same verify results as the device
    call"""
    b, hb, offs, sizes = batch(8000, 16384, CT.kCRC32c, 0xF0E57000AD)
    p = tmp_path / "000123.sst"
    hb.tofile(p)
    m = hostpath.MappedFile(str(p), register=True)
    try:
        comp, st, ok, bad = engine.block_verify_batch(CT.kCRC32c, b.base, b.offsets, b.sizes)
        hcomp, _, hok, hbad = hostpath.block_verify_host(CT.kCRC32c, m, offs, sizes,
                                                         devices=(0, 0))
        assert hbad == 0 and hok.all()
        assert (hcomp == comp.cpu().numpy()).all()
        print("registered:", m.registered, m.register_error)
    finally:
        m.close()


def test_host_args_rejected():
    from forst_amd import ForstError
    hb = np.zeros(100, np.uint8)
    with pytest.raises(ForstError):  # block past the buffer
        hostpath.block_verify_host(CT.kCRC32c, hb, [90], [10])
    with pytest.raises(ForstError):
        hostpath.block_verify_host(9, hb, [0], [10])
    with pytest.raises(ForstError):
        hostpath.block_verify_host(CT.kCRC32c, hb, [0], [10], devices=())


def test_back_to_back_calls_reuse_the_context():
    """1000 forst_block_verify_host calls in a row: after the first, the
    context pool holds the same contexts and bytes, and free device memory
    does not move (no per-call hipMalloc / hipHostMalloc / stream)"""
    b, hb, offs, sizes = batch(2000, (4096, 16384), CT.kCRC32c, 0xF0E57000AE)
    want = hostpath.block_verify_host(CT.kCRC32c, hb, offs, sizes, devices=(0,))
    torch.cuda.synchronize()
    s0 = hostpath.context_stats()
    free0 = torch.cuda.mem_get_info()[0]
    for k in range(1000):
        got = hostpath.block_verify_host(CT.kCRC32c, hb, offs, sizes, devices=(0,))
        if k % 250 == 0:
            assert (got[0] == want[0]).all() and got[3] == 0
    assert hostpath.context_stats() == s0, (s0, hostpath.context_stats())
    assert torch.cuda.mem_get_info()[0] == free0
    assert s0[0] >= 1 and s0[1] > 0 and s0[2] > 0
    # trim: idle contexts give their buffers back; the next call grows them again
    assert hostpath.context_trim() == s0[1] + s0[2]
    assert hostpath.context_stats() == (s0[0], 0, 0)
    got = hostpath.block_verify_host(CT.kCRC32c, hb, offs, sizes, devices=(0,))
    assert (got[0] == want[0]).all() and got[3] == 0
    assert hostpath.context_stats()[1] > 0


def test_out_of_order_descriptors_and_partial_registration():
    """descriptors that do not ascend (a window spans its blocks' minimum
    offset) and a pinned buffer of which only the first part is pinned (the
    batch is staged instead of DMA'd from unpinned pages)"""
    b, hb, offs, sizes = batch(6000, 4096, CT.kXXH3, 0xF0E57000AF)
    perm = np.random.default_rng(8).permutation(b.n)
    comp, _, ok, bad = hostpath.block_verify_host(CT.kXXH3, hb, offs[perm], sizes[perm],
                                                  devices=(0,))
    assert bad == 0 and ok.all()
    want = engine.block_verify_batch(CT.kXXH3, b.base, b.offsets, b.sizes)[0].cpu().numpy()
    assert (comp == want[perm]).all()
    import ctypes
    import mmap
    from forst_amd._lib import lib
    mm = mmap.mmap(-1, (len(hb) + 4095) // 4096 * 4096)
    buf = np.frombuffer(mm, np.uint8)
    buf[:len(hb)] = hb
    ptr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
    half = (len(buf) // 2) // 4096 * 4096
    assert lib().forst_host_register(ptr, half) == 0  # only the first half pinned
    try:
        comp2, _, ok2, bad2 = hostpath.block_verify_host(CT.kXXH3, buf[:len(hb)], offs, sizes,
                                                         devices=(0,))
        assert bad2 == 0 and (comp2 == want).all()
        # a second registration over the tail, unregistered pages between the
        # two: the first and last bytes are both pinned, the batch is still
        # staged (one registration must cover the whole range)
        tail = (len(buf) - half) // 2 // 4096 * 4096
        t0 = len(buf) - tail
        assert lib().forst_host_register(ptr + t0, tail) == 0
        try:
            comp3, _, ok3, bad3 = hostpath.block_verify_host(CT.kXXH3, buf[:len(hb)], offs,
                                                             sizes, devices=(0,))
            assert bad3 == 0 and (comp3 == want).all()
        finally:
            lib().forst_host_unregister(ptr + t0)
    finally:
        lib().forst_host_unregister(ptr)
        del buf
        mm.close()


def test_aux_streams_bounded_by_calls_in_flight():
    """64 short-lived host threads, 8 at a time, each on its own torch stream,
    through forst_wal_record_xxh3_batch and forst_wal_recover_batch (their
    side branches run on a second stream, db_impl_open.cc:1206-1245 calls
    from whichever thread recovers): the second streams come from the
    per-device pool, so no more exist than calls were in flight at once,
    results are unchanged, and forst_host_context_trim destroys the idle ones
    and leaves the caller's current device as it was"""
    import threading
    PIT = 2  # WALRecoveryMode::kPointInTimeRecovery (options.h:1192)
    w = workload.make_wal_batch(20000, workload.SEEDS["C5"])
    offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
    want = engine.wal_record_xxh3_batch(w.log, offs)[0].cpu()
    rec0, _, res0 = engine.wal_recover_batch(w.log, 0, PIT)
    want_rec = rec0["hash"][:res0.n_records].cpu()
    torch.cuda.synchronize()
    live0, _ = hostpath.aux_stream_stats()
    errs = []

    def work(k):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                if k % 2:
                    h, _ = engine.wal_record_xxh3_batch(w.log, offs)
                    ok = torch.equal(h.cpu(), want)
                else:
                    rec, _, res = engine.wal_recover_batch(w.log, 0, PIT)
                    ok = torch.equal(rec["hash"][:res.n_records].cpu(), want_rec)
            if not ok:
                errs.append(f"thread {k}: wrong result")
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(f"thread {k}: {e!r}")

    for wave in range(8):
        ts = [threading.Thread(target=work, args=(8 * wave + i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errs, errs[:3]
    live, idle = hostpath.aux_stream_stats()
    assert live <= max(live0, 8) and idle == live, (live0, live, idle)
    dev = torch.cuda.current_device()
    hostpath.context_trim()
    assert hostpath.aux_stream_stats() == (0, 0)
    assert torch.cuda.current_device() == dev
    # the next call creates one again and gives it back
    assert torch.equal(engine.wal_record_xxh3_batch(w.log, offs)[0].cpu(), want)
    assert hostpath.aux_stream_stats() == (1, 1)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_trim_keeps_the_callers_device():
    """a context on device 1, trimmed from a thread whose current device is 0:
    the thread's device stays 0 (forst_host_context_trim restores it)"""
    b, hb, offs, sizes = batch(500, 4096, CT.kCRC32c, 0xF0E57000B1)
    hostpath.block_verify_host(CT.kCRC32c, hb, offs, sizes, devices=(1,))
    torch.cuda.set_device(0)
    hostpath.context_trim()
    assert torch.cuda.current_device() == 0


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0)])
def test_wal_verify_host_matches_device_call(devices):
    """a WAL log in host memory (pageable, then a registered mmap of the log
    file) verified over a device list -- one context per entry, equal
    contiguous log-block ranges, 64 MiB windows -- gives per block exactly the
    device-resident forst_wal_verify_batch's status / records / offset, with
    flips in every range detected (db/log_reader.cc:450-531)"""
    import tempfile

    w = workload.make_wal_batch(60000, workload.SEEDS["C5"] + 1)  # ~260 MiB: several windows
    rng = np.random.default_rng(31)
    cand = np.nonzero(w.rec_lengths > 0)[0]
    victims = rng.choice(cand, 9, replace=False)
    pos = w.rec_offsets[victims].astype(np.int64) + 7 + \
        rng.integers(0, w.rec_lengths[victims].astype(np.int64))
    w.log[torch.from_numpy(pos).cuda()] ^= 0x04
    st, nr, fo, bad = engine.wal_verify_batch(w.log)
    want = (st.cpu().numpy(), nr.cpu().numpy(), fo.cpu().numpy(), int(bad.item()))
    assert want[3] == len(set((w.rec_offsets[victims] // 32768).tolist()))
    logh = w.log.cpu().numpy()
    got = hostpath.wal_verify_host(logh, 0, devices)
    for g, x in zip(got[:3], want[:3]):
        assert np.array_equal(g, x)
    assert got[3] == want[3]
    d = tempfile.mkdtemp()
    path = d + "/000007.log"
    logh.tofile(path)
    m = hostpath.MappedFile(path, register=True)
    try:
        got = hostpath.wal_verify_host(m, 0, devices)
        for g, x in zip(got[:3], want[:3]):
            assert np.array_equal(g, x)
        assert got[3] == want[3]
    finally:
        m.close()
        import os
        os.unlink(path)
        os.rmdir(d)
