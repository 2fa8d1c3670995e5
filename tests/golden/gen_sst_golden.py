#!/usr/bin/env python3
"""tests/golden/gen_sst_golden.py -- TEST INFRASTRUCTURE ONLY: SST fixtures
written with the REFERENCE's own table-writer code.

The reference's BlockBuilder, BlockHandle / IndexValue encoders,
PropertyBlockBuilder, MetaIndexBuilder, FooterBuilder, and the block trailer
(ComputeBuiltinChecksumWithLastByte + ChecksumModifierForContext) are compiled
from the sources where they lie under /root/reference (the files in
REF_SRCS, plus the veneers tests/golden/ref_shim.cc and ref_sst_shim.cc;
hidden visibility and --gc-sections link only what the veneers reach) into a
temporary directory OUTSIDE the repository, called through ctypes, and
deleted.  The block ORDER and the key/value content come from
tests/sstgen.SstWriter, run with a codec that routes every encoding to the
reference (RefCodec below); the resulting files are committed as
tests/golden/sst/*.sst (+ manifest.json), and every FooterBuilder::Build
output for format_version 0-6 x the 5 checksum types as ref_footers.json.
tests/test_sst_pinned.py then checks that sstgen's own restated encodings
write the same bytes, and the GPU verify / writer paths run on these files.

Second family (round 3): whole files from the reference's own
SstFileWriter -> BlockBasedTableBuilder (tests/golden/ref_sstwriter_shim.cc,
linked against the reference archive of tests/golden/refbuild.py), so block
ORDER, filter blocks and partitions, index partitions, range-deletion and
compression-dictionary blocks, and zlib-compressed data AND index blocks
(enable_index_compression, include/rocksdb/table.h:526) are all the
reference's: tests/golden/sst/builder_*.sst + builder_manifest.json.  For
each file, single-byte corruptions of chosen blocks (located with
tests/sstwalk.py) are run through the reference's SstFileReader::
VerifyChecksum, and its Status text is recorded ("{file}" stands for the path).

Re-run:  python tests/golden/gen_sst_golden.py [--builder]   (needs /root/reference + g++)
"""
import ctypes
import json
import os
import shutil
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path.insert(0, TESTS)
sys.path.insert(0, os.path.dirname(TESTS))
import sstgen  # noqa: E402

REF = os.environ.get("FORST_REFERENCE", "/root/reference")
REF_SRCS = [
    "util/crc32c.cc", "util/xxhash.cc", "util/hash.cc", "util/coding.cc", "util/status.cc",
    "util/slice.cc", "util/comparator.cc", "util/string_util.cc", "table/format.cc",
    "table/meta_blocks.cc", "table/block_based/block_builder.cc",
    "table/block_based/data_block_hash_index.cc", "table/block_based/data_block_footer.cc",
    # the table magic numbers FooterBuilder writes are defined here
    "table/block_based/block_based_table_builder.cc", "table/plain/plain_table_builder.cc",
    "db/dbformat.cc", "options/customizable.cc", "options/configurable.cc",
    "options/options_helper.cc",
]
OUT_DIR = os.path.join(HERE, "sst")

# (format_version, checksum type, index type, external, restart interval,
#  base context checksum, data blocks, seed); index types: 0 binary search,
# 2 two-level (partitioned), 3 binary search with first key
CONFIGS = [
    (0, 1, 0, False, 1, 0, 8, 101),
    (2, 2, 0, False, 1, 0, 8, 102),
    (3, 3, 2, False, 1, 0, 10, 103),
    (4, 1, 3, False, 1, 0, 8, 104),
    (5, 4, 0, True, 4, 0, 8, 105),
    (5, 1, 2, False, 16, 0, 12, 106),
    (6, 4, 3, False, 1, 0x5EED0001, 8, 107),
    (6, 1, 2, True, 4, 0x5EED0002, 10, 108),
    (6, 0, 0, False, 1, 0x5EED0003, 6, 109),
    (6, 3, 0, False, 1, 0x5EED0004, 6, 110),
]


def build_reference(tmpdir):
    out = os.path.join(tmpdir, "libforst_ref_sst.so")
    cmd = (["g++", "-std=c++17", "-O1", "-fPIC", "-shared",
            "-ffunction-sections", "-fdata-sections", "-Wl,--gc-sections",
            "-DROCKSDB_PLATFORM_POSIX", "-DOS_LINUX", "-DNDEBUG", "-DNPERF_CONTEXT",
            "-fvisibility=hidden", "-fvisibility-inlines-hidden",
            "-w", f"-I{REF}", f"-I{REF}/include", "-o", out]
           + [os.path.join(REF, s) for s in REF_SRCS]
           + [os.path.join(HERE, "ref_shim.cc"), os.path.join(HERE, "ref_sst_shim.cc"),
              "-lpthread"])
    subprocess.check_call(cmd)
    und = subprocess.run(["nm", "-D", "--undefined-only", out], capture_output=True,
                         text=True).stdout
    assert "forstdb" not in und and "rocksdb" not in und, und  # nothing stood in for
    L = ctypes.CDLL(out)
    u32, u64, vp, i = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
    pu64 = ctypes.POINTER(u64)
    sigs = {
        "ref_compute_builtin_checksum_with_last_byte": (u32, [i, vp, ctypes.c_size_t,
                                                              ctypes.c_char]),
        "ref_checksum_modifier_for_context": (u32, [u32, u64]),
        "ref_footer_build": (i, [u64, u32, u64, i, u64, u64, u64, u64, u32, vp, u64, pu64]),
        "ref_block_build": (i, [i, i, i, vp, u32, vp, u64, pu64]),
        "ref_handle_encode": (i, [u64, u64, vp, u64, pu64]),
        "ref_index_value_encode": (i, [u64, u64, vp, u32, i, i, u64, u64, vp, u64, pu64]),
        "ref_properties_build": (i, [vp, u32, vp, u64, pu64]),
        "ref_metaindex_build": (i, [vp, u32, vp, u64, pu64]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def _call(fn, *args, cap=1 << 22):
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_uint64()
    rc = fn(*args, out, cap, ctypes.byref(n))
    assert rc == 0, rc
    return out.raw[:n.value]


class RefCodec:
    """sstgen's codec interface, every encoding by the reference"""

    def __init__(self, L):
        self.L = L

    def block(self, restart_interval, delta_keys, value_delta, entries):
        buf = bytearray()
        for key, value, delta in entries:
            buf += struct.pack("<III", len(key), len(value),
                               0xFFFFFFFF if delta is None else len(delta))
            buf += key + value + (delta or b"")
        return _call(self.L.ref_block_build, restart_interval, int(delta_keys), int(value_delta),
                     bytes(buf), len(entries))

    def handle(self, off, n):
        return _call(self.L.ref_handle_encode, off, n)

    def index_value(self, off, n, first_key, have_first_key, prev):
        return _call(self.L.ref_index_value_encode, off, n, first_key, len(first_key),
                     int(have_first_key), int(prev is not None),
                     prev[0] if prev else 0, prev[1] if prev else 0)

    def properties(self, props):
        buf = bytearray()
        for k, kind, v in props:
            val = struct.pack("<Q", v) if kind == "u64" else v
            buf += struct.pack("<IBI", len(k), 0 if kind == "u64" else 1,
                               8 if kind == "u64" else len(v)) + k + val
        return _call(self.L.ref_properties_build, bytes(buf), len(props))

    def metaindex(self, entries):
        buf = bytearray()
        for k, (off, n) in entries:
            buf += struct.pack("<IQQ", len(k), off, n) + k
        return _call(self.L.ref_metaindex_build, bytes(buf), len(entries))

    def trailer(self, ctype, contents, ctype_byte, bcc, off):
        c = self.L.ref_compute_builtin_checksum_with_last_byte(ctype, contents, len(contents),
                                                               bytes([ctype_byte]))
        c = (c + self.L.ref_checksum_modifier_for_context(bcc, off)) & 0xFFFFFFFF
        return bytes([ctype_byte]) + struct.pack("<I", c)

    def footer(self, fv, ctype, footer_offset, mi, ix, bcc):
        return _call(self.L.ref_footer_build, sstgen.MAGIC, fv, footer_offset, ctype,
                     mi[0], mi[1], ix[0], ix[1], bcc)


# SstFileWriter configurations: (format_version, checksum, index type, filter
# (0 none, 1 full bloom, 2 partitioned), compression (0 none, 2 zlib), index
# compression, block_size, restart interval, keys, value length, range
# deletions, compression dictionary bytes, seed)
BUILDER_CONFIGS = [
    (5, 1, 0, 1, 2, 1, 1024, 16, 700, 60, 0, 0, 201),
    (6, 4, 2, 2, 2, 1, 1024, 16, 1100, 60, 2, 0, 202),
    (6, 1, 3, 1, 2, 1, 2048, 4, 800, 80, 0, 4096, 203),
    (5, 4, 0, 0, 0, 0, 4096, 16, 500, 100, 1, 0, 204),
    (4, 3, 2, 1, 2, 1, 1024, 16, 700, 60, 0, 0, 205),
    (3, 2, 0, 1, 2, 0, 1024, 16, 500, 60, 0, 0, 206),
    (6, 0, 0, 1, 2, 1, 1024, 16, 400, 60, 0, 0, 207),
    (2, 1, 2, 2, 2, 1, 512, 1, 900, 40, 1, 0, 208),
    (5, 1, 2, 2, 2, 1, 512, 16, 1400, 40, 0, 0, 209),
    (1, 1, 0, 1, 2, 1, 1024, 16, 600, 60, 0, 0, 210),  # compress_format_version 1
    (0, 1, 2, 0, 2, 1, 1024, 16, 600, 60, 0, 0, 211),
]
FLIP_KINDS = ("data", "index", "index_partition", "metaindex", "properties", "filter",
              "filter_index", "filter_partition", "rangedel", "dict")


def gen_builder_files(tmp):
    import sstwalk
    so = os.path.join(tmp, "libref_sstw.so")
    sys.path.insert(0, HERE)
    import refbuild
    refbuild.link_veneer([os.path.join(HERE, "ref_sstwriter_shim.cc")], so)
    L = ctypes.CDLL(so)
    L.ref_sst_write.restype = ctypes.c_int
    L.ref_sst_verify.restype = ctypes.c_int
    err = ctypes.create_string_buffer(1024)
    files = []
    for i, (fv, ct, it, flt, comp, icomp, bs, ri, nk, vl, rd, db, seed) in enumerate(BUILDER_CONFIGS):
        name = f"builder_fv{fv}_ct{ct}_ix{it}_f{flt}_c{comp}.sst"
        path = os.path.join(tmp, name)
        rc = L.ref_sst_write(path.encode(), fv, ct, it, flt, comp, icomp, bs, ri, nk, vl,
                             ctypes.c_ulonglong(seed), rd, db, err, 1024)
        assert rc == 0, err.value
        data = open(path, "rb").read()
        blocks, f = sstwalk.walk(data)
        assert sstwalk.tiles(blocks, f), name
        rc = L.ref_sst_verify(path.encode(), err, 1024)
        assert rc == 0, err.value
        flips = []
        for kind in FLIP_KINDS:
            ks = [b for b in blocks if b[0] == kind]
            for b in (ks[:1] + ks[len(ks) // 2:len(ks) // 2 + 1] if kind == "data" else ks[:1]):
                _, o, n, _ = b
                at = o + n // 2
                bad = bytearray(data)
                bad[at] ^= 0x20
                cpath = os.path.join(tmp, "corrupt_" + name)
                open(cpath, "wb").write(bad)
                L.ref_sst_verify(cpath.encode(), err, 1024)
                flips.append({"kind": kind, "block": [o, n], "offset": at,
                              "status": err.value.decode().replace(cpath, "{file}")})
        if f["fv"] >= 6:  # the footer checksum field
            bad = bytearray(data)
            bad[f["footer_offset"] + 6] ^= 0x01
            cpath = os.path.join(tmp, "corrupt_" + name)
            open(cpath, "wb").write(bad)
            L.ref_sst_verify(cpath.encode(), err, 1024)
            flips.append({"kind": "footer", "block": [f["footer_offset"], 53],
                          "offset": f["footer_offset"] + 6,
                          "status": err.value.decode().replace(cpath, "{file}")})
        with open(os.path.join(OUT_DIR, name), "wb") as fh:
            fh.write(data)
        files.append({"file": name, "format_version": fv, "checksum": ct, "index_type": it,
                      "filter": flt, "compression": comp, "index_compression": icomp,
                      "block_size": bs, "restart_interval": ri, "keys": nk, "value_len": vl,
                      "range_dels": rd, "dict_bytes": db, "seed": seed, "size": len(data),
                      "blocks": [[k, o, n, t] for k, o, n, t in blocks],
                      "footer_offset": f["footer_offset"], "flips": flips})
        print(name, len(data), len(blocks), [x["status"][:60] for x in flips][:3])
    with open(os.path.join(OUT_DIR, "builder_manifest.json"), "w") as fh:
        json.dump({"generator": "tests/golden/gen_sst_golden.py (SstFileWriter, "
                                "table/sst_file_writer.cc; SstFileReader::VerifyChecksum)",
                   "files": files}, fh, indent=0)


def main():
    tmp = tempfile.mkdtemp(prefix="forst_ref_sst_")
    if "--builder" in sys.argv:
        try:
            gen_builder_files(tmp)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    try:
        L = build_reference(tmp)
        codec = RefCodec(L)
        os.makedirs(OUT_DIR, exist_ok=True)
        manifest = []
        for fv, ct, it, ext, ri, bcc, nd, seed in CONFIGS:
            w = sstgen.SstWriter(fv=fv, ctype=ct, index_type=it, base_context=bcc,
                                 restart_interval=ri, seed=seed, codec=codec)
            f = w.build(n_data=nd, external=ext)
            name = f"ref_fv{fv}_ct{ct}_ix{it}{'_ext' if ext else ''}.sst"
            with open(os.path.join(OUT_DIR, name), "wb") as fh:
                fh.write(f)
            manifest.append({"file": name, "format_version": fv, "checksum": ct,
                             "index_type": it, "external": ext, "restart_interval": ri,
                             "base_context_checksum": bcc, "n_data": nd, "seed": seed,
                             "size": len(f), "footer_offset": w.footer_offset,
                             "blocks": [[k, o, n] for k, o, n in w.blocks]})
        with open(os.path.join(OUT_DIR, "manifest.json"), "w") as fh:
            json.dump({"generator": "tests/golden/gen_sst_golden.py",
                       "reference_sources": REF_SRCS, "files": manifest}, fh, indent=1)
        footers = []
        for fv in range(7):
            for ct in range(5):
                for off, mi, ix, bcc in ((4096, (3000, 96), (2000, 1000), 0x01020304),
                                         (123456789, (123000000, 4321), (9, 122999990), 0xFFFFFFFF),
                                         (1 << 40, ((1 << 40) - 70, 65), (0, 0), 0)):
                    b = codec.footer(fv, ct, off, mi, ix, bcc if fv >= 6 else 0)
                    footers.append({"format_version": fv, "checksum": ct, "footer_offset": off,
                                    "metaindex": list(mi), "index": list(ix),
                                    "base_context_checksum": bcc if fv >= 6 else 0,
                                    "hex": b.hex()})
        with open(os.path.join(HERE, "ref_footers.json"), "w") as fh:
            json.dump({"generator": "tests/golden/gen_sst_golden.py (FooterBuilder::Build, "
                                    "table/format.cc:231)", "footers": footers}, fh, indent=0)
        print(f"{len(manifest)} SST files, {len(footers)} footers")
        gen_builder_files(tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
