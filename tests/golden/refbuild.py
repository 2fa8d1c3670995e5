#!/usr/bin/env python3
"""tests/golden/refbuild.py -- TEST INFRASTRUCTURE ONLY: compile the
REFERENCE's own library sources (the LIB_SOURCES list of /root/reference/src.mk)
with g++ into a throwaway directory OUTSIDE the repository, archive them, and
link a fixture veneer against that archive.

Why an archive: the reference objects we need (log::Reader, SstFileWriter /
BlockBasedTableBuilder) reach the Env / FileSystem / options layer, a link
closure of a few hundred files.  A static archive lets the linker pull exactly
the members the veneer reaches; `-z defs` proves that nothing is left
undefined, so no reference symbol is ever stood in for.

This does not run the reference's build system (no make / cmake): it reads the
source list from src.mk and drives g++ on the files where they lie.  Excluded:
  * env/flink/*, utilities/flink/* -- need jni.h, absent from the image.
util/build_version.cc is a generated source: it is produced from the
reference's own template util/build_version.cc.in by the substitution the
reference Makefile prescribes (Makefile:830 gen_build_version), with no git
metadata and no plugins (ROCKSDB_PLUGIN_BUILTINS / _EXTERNS empty, as in a
build without ROCKSDB_PLUGINS).  Nothing is hand-written in its place.
Compression: only zlib has headers in the image, so -DZLIB (kZlibCompression);
snappy / lz4 / zstd / bzip2 are compiled out exactly as a reference build
without those libraries would be.

Objects are cached under $FORST_REFOBJ (default /tmp/forst_refobj), keyed by
flags, so the generators can be re-run cheaply.  Nothing produced here is
committed; the generators commit only data (inputs and expected outputs).
"""
import hashlib
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REF = os.environ.get("FORST_REFERENCE", "/root/reference")
CACHE = os.environ.get("FORST_REFOBJ", "/tmp/forst_refobj")
DEFS = ["-DROCKSDB_PLATFORM_POSIX", "-DROCKSDB_LIB_IO_POSIX", "-DOS_LINUX", "-DZLIB",
        "-DNDEBUG", "-DROCKSDB_SUPPORT_THREAD_LOCAL"]
CXXFLAGS = ["-std=c++17", "-O1", "-fPIC", "-ffunction-sections", "-fdata-sections", "-w",
            "-march=native"] + DEFS
EXCLUDE = re.compile(r"^(env/flink/|utilities/flink/)")


def lib_sources():
    text = open(os.path.join(REF, "src.mk")).read()
    m = re.search(r"^LIB_SOURCES =(.*?)\n\n", text, re.S | re.M)
    srcs = [s for s in m.group(1).replace("\\", " ").split() if s.endswith(".cc")]
    return [s for s in srcs if not EXCLUDE.match(s)]


def _gen_build_version(out):
    """util/build_version.cc from build_version.cc.in, Makefile:830's recipe"""
    t = open(os.path.join(REF, "util/build_version.cc.in")).read()
    for k, v in (("@GIT_SHA@", "unknown"), ("@GIT_TAG@", ""), ("@GIT_MOD@", "0"),
                 ("@BUILD_DATE@", "unknown"), ("@GIT_DATE@", "unknown"),
                 ("@ROCKSDB_PLUGIN_BUILTINS@", ""), ("@ROCKSDB_PLUGIN_EXTERNS@", "")):
        t = t.replace(k, v)
    path = os.path.join(out, "build_version.cc")
    with open(path, "w") as f:
        f.write(t)
    return path


def _key():
    h = hashlib.sha1(" ".join(CXXFLAGS).encode()).hexdigest()[:10]
    return os.path.join(CACHE, h)


def build_archive(jobs=None):
    """compile every LIB_SOURCE once (cached) -> path of libref.a"""
    out = _key()
    os.makedirs(out, exist_ok=True)
    lib = os.path.join(out, "libref.a")
    srcs = lib_sources()
    objs = [os.path.join(out, s.replace("/", "__")[:-3] + ".o") for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if not os.path.exists(o)]

    gen = _gen_build_version(out)

    def cc(so):
        s, o = so
        tmp = o + ".tmp"
        src = gen if s == "util/build_version.cc" else os.path.join(REF, s)
        r = subprocess.run(["g++"] + CXXFLAGS + [f"-I{REF}", f"-I{REF}/include", f"-I{REF}/util",
                            "-c", src, "-o", tmp], capture_output=True, text=True)
        if r.returncode != 0:
            return s, r.stderr[-2000:]
        os.replace(tmp, o)
        return s, None

    if todo:
        print(f"refbuild: compiling {len(todo)} of {len(srcs)} reference sources into {out}",
              file=sys.stderr, flush=True)
        with ThreadPoolExecutor(jobs or min(8, os.cpu_count() or 4)) as ex:
            errs = [(s, e) for s, e in ex.map(cc, todo) if e]
        if errs:
            raise RuntimeError("reference compile failed: " + "; ".join(f"{s}: {e}" for s, e in errs[:3]))
        if os.path.exists(lib):
            os.remove(lib)
    if not os.path.exists(lib):
        subprocess.check_call(["ar", "rcs", lib + ".tmp"] + objs)
        os.replace(lib + ".tmp", lib)
    return lib


def link_veneer(veneers, out, extra_objs=()):
    """link veneer sources + the archive members they reach into a shared lib"""
    lib = build_archive()
    cmd = (["g++"] + CXXFLAGS + ["-shared", "-fvisibility=hidden", "-fvisibility-inlines-hidden",
                                 f"-I{REF}", f"-I{REF}/include", "-o", out]
           + list(veneers) + list(extra_objs)
           + ["-Wl,--gc-sections", "-Wl,-z,defs", lib, "-lz", "-lpthread", "-ldl"])
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    print(build_archive())
