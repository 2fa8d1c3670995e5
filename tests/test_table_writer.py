"""Write-side batching (§8f-3): the deferred-trailer table writer
(forst_amd/csrc/table_writer.cc) re-writes whole SST files from their blocks --
data, filter, index / partitions, properties, metaindex, in builder order --
with every trailer computed in GPU batches and the footer from
forst_sst_footer_build, and the bytes must equal the file written block by
block with the CPU oracle's trailers (tests/sstgen.py, the restatement of
WriteMaybeCompressedBlock + FooterBuilder::Build whose checksums are pinned to
the reference vectors).  fv 0-6 x all five ChecksumTypes x index types, tiny
windows (many GPU launches, both windows alternating) and the default window,
block_align padding, and a 20 000-block fv6 stream against the oracle.

The file layout is pinned: tests/sstgen.py writes the reference-encoded files
of tests/golden/sst byte for byte (tests/test_sst_pinned.py, which also
rewrites those files through this writer)."""
import struct

import numpy as np
import pytest

import sstgen
from oracle import oracle as O

CASES = [(0, 1, 0, 1), (1, 2, 0, 1), (2, 3, 0, 1), (3, 4, 1, 1), (4, 1, 0, 4), (5, 4, 3, 1),
         (5, 1, 2, 1), (6, 1, 0, 1), (6, 4, 2, 4), (6, 2, 3, 1), (6, 3, 0, 1), (6, 0, 0, 1)]


def make(fv, ct, it, ri, seed=3):
    w = sstgen.SstWriter(fv=fv, ctype=ct, index_type=it, base_context=0x5EED1234 + seed,
                         restart_interval=ri, seed=seed)
    return w, w.build()


@pytest.mark.parametrize("fv,ct,it,ri", [c for c in CASES if c[0] < 6])
def test_footer_build_without_gpu(fv, ct, it, ri):
    """format_version < 6 footers carry no checksum: built on the host only"""
    from forst_amd import table_writer as tw
    w, f = make(fv, ct, it, ri)
    mi = [(o, n) for k, o, n in w.blocks if k == "metaindex"][0]
    ix = [(o, n) for k, o, n in w.blocks if k == "index"][0]
    got = tw.footer_build(fv, 1 if fv == 0 else ct, w.footer_offset, 0, mi, ix)
    assert got == f[w.footer_offset:]


def test_footer_build_rejects_bad_args():
    from forst_amd import ForstError
    from forst_amd import table_writer as tw
    with pytest.raises(ForstError):
        tw.footer_build(7, 1, 0, 0, (0, 0))
    with pytest.raises(ForstError):
        tw.footer_build(0, 4, 0, 0, (0, 0))  # fv 0 implies kCRC32c


def rewrite(w, f, window_bytes, start=0):
    from forst_amd import table_writer as tw
    fv, ct = w.fv, (1 if w.fv == 0 else w.ctype)
    tr = tw.TrailerWriter(ct, w.bcc, start_offset=start, window_bytes=window_bytes)
    handles = []
    for kind, off, n in sorted(w.blocks, key=lambda b: b[1]):
        h = tr.add(f[off:off + n], f[off + n], is_data_block=(kind == "data"))
        assert h == (off, n)  # the handle is final before the trailer exists
        handles.append((kind, h))
    mi = [h for k, h in handles if k == "metaindex"][0]
    ix = [h for k, h in handles if k == "index"][0]
    tr.footer(fv, mi, ix)
    return tr.close(), tr


@pytest.mark.gpu
@pytest.mark.parametrize("window", [4096, 0])
@pytest.mark.parametrize("fv,ct,it,ri", CASES)
def test_rewrite_sst_byte_identical(fv, ct, it, ri, window):
    w, f = make(fv, ct, it, ri)
    out, tr = rewrite(w, f, window)
    assert out == f
    if window:
        assert tr.chunks > 3  # several GPU windows, written in file order


@pytest.mark.gpu
def test_block_align_padding_and_large_stream():
    """20 000 blocks of 0-20 KiB, fv6 kXXH3 with a base context, data blocks
    padded to 4 KiB (block_align, builder.cc:1385-1395): every trailer equals
    the oracle's, pads are zero, handles are the padded offsets."""
    from forst_amd import table_writer as tw
    rng = np.random.default_rng(8)
    n = 20000
    sizes = rng.integers(0, 20000, n)
    sizes[:5] = [0, 1, 4091, 4092, 65536]
    types = rng.integers(0, 8, n).astype(np.uint8)
    data = rng.integers(0, 256, int(sizes.sum()), np.uint8)
    starts = np.concatenate([[0], np.cumsum(sizes)])
    bcc = 0x9E3779B1
    tr = tw.TrailerWriter(4, bcc, start_offset=0, block_align=4096, window_bytes=1 << 20)
    want = bytearray()
    for i in range(n):
        blk = data[starts[i]:starts[i + 1]].tobytes()
        off = len(want)
        assert tr.add(blk, int(types[i]), is_data_block=(i % 7 != 0)) == (off, len(blk))
        c = O.compute_builtin_checksum_with_last_byte(4, blk, int(types[i]))
        c = (c + O.checksum_modifier_for_context(bcc, off)) & 0xFFFFFFFF
        want += blk + bytes([int(types[i])]) + struct.pack("<I", c)
        if i % 7 != 0:
            want += bytes((4096 - ((len(blk) + 5) & 4095)) & 4095)
    assert tr.offset == len(want)
    assert tr.close() == bytes(want)
