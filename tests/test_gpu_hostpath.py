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
