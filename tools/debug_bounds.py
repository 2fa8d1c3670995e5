#!/usr/bin/env python3
"""tools/debug_bounds.py -- run the CRC block kernels from the bounds-checked
diagnostics build (lib/libforst_checksum_dbg.so) on the golden vectors and on
SST-shaped batches; report any out-of-bounds access the kernels attempted
(recorded and skipped instead of faulting) and any result mismatch."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import stream  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, "forst_amd", "lib", "libforst_checksum_dbg.so"))
vp, u64, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
L.forst_block_verify_batch.argtypes = [i, vp, u64, vp, vp, vp, vp, vp, vp, vp, u64, vp]
L.forst_block_trailer_batch.argtypes = [i, vp, u64, vp, vp, vp, vp, vp, u64, vp]
L.forst_crc32c_batch.argtypes = [vp, u64, vp, vp, vp, vp, u64, vp]
L.forst_debug_fetch.argtypes = [vp]


def fetch():
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 4)()
    assert L.forst_debug_fetch(out) == 0
    return list(out)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run_verify(tag, base, offs, sizes, want=None):
    n = len(offs)
    b, o, s = dev(base), dev(offs.astype(np.int64)), dev(sizes.astype(np.int32))
    comp = torch.zeros(n, dtype=torch.int32, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    rc = L.forst_block_verify_batch(1, b.data_ptr(), b.numel(), o.data_ptr(), s.data_ptr(), None,
                                    comp.data_ptr(), None, ok.data_ptr(), bad.data_ptr(), n, None)
    rec = fetch()
    res = {"tag": tag, "rc": rc, "oob_record": rec, "mismatches": int(bad.item())}
    if want is not None:
        c = comp.cpu().numpy().view(np.uint32)
        res["computed_wrong"] = int((c != want).sum())
    print(json.dumps(res), flush=True)
    return res


def main():
    with open(os.path.join(ROOT, "tests", "golden", "ref_vectors.json")) as f:
        v = json.load(f)
    blob = np.frombuffer(stream.golden_blob(v["blob_bytes"]), dtype=np.uint8).copy()
    offs = np.array([r["off"] for r in v["vectors"]], dtype=np.uint64)
    lens = np.array([r["n"] for r in v["vectors"]], dtype=np.uint32)
    want = np.array([r["builtin_plus1"][1] for r in v["vectors"]], dtype=np.uint32)
    run_verify("golden", blob, offs, lens, want)
    for spec in (4096, 16384):
        n = 20000
        sizes = np.full(n, spec, dtype=np.uint32)
        o = np.zeros(n, dtype=np.uint64)
        o[1:] = np.cumsum(sizes[:-1].astype(np.uint64) + 5)
        total = int(o[-1]) + spec + 5
        base = stream.stream(0xF0E5700002, 0, total)
        b = dev(base)
        do, ds = dev(o.astype(np.int64)), dev(sizes.astype(np.int32))
        types = torch.zeros(n, dtype=torch.uint8, device="cuda")
        rc = L.forst_block_trailer_batch(1, b.data_ptr(), b.numel(), do.data_ptr(), ds.data_ptr(),
                                         types.data_ptr(), None, None, n, None)
        print(json.dumps({"tag": f"trailer{spec}", "rc": rc, "oob_record": fetch()}), flush=True)
        run_verify(f"verify{spec}", b.cpu().numpy(), o, sizes)


if __name__ == "__main__":
    main()
