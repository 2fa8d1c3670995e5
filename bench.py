#!/usr/bin/env python3
"""bench.py -- device-resident block-checksum throughput on MI355X.

Metric (BASELINE.json): device-resident GiB/s checksummed (CRC32C/XXH3).
Default workload = configs[1] ("C2"): 1 M x 4 KiB SST blocks per GPU,
kCRC32c, compute (write side: trailer pass, ComputeBuiltinChecksumWithLastByte
+ trailer, block_based_table_builder.cc:1340) + verify (read side,
VerifyBlockChecksum, reader_common.cc:26).  One step = both passes over the
rank's blocks; checksummed bytes per pass = sum(size + 1).

Multi-GPU: `--gpus N` runs one process per GPU.  Launched
without a torch.distributed environment, bench.py starts
`torch.distributed.run --nproc-per-node N` itself (as a child process, before
any GPU call) and exits with its code.  The N ranks share ONE described batch
of N x n blocks (weak scaling: n blocks of work per GPU) and each takes its
byte-balanced contiguous slice (forst_amd.shard.rank_slice) -- the bytes of a
block are the same whichever rank hashes it.  No collective touches the data
path: barrier + synchronize bracket the timed steps, the elapsed time is the
max over ranks and value = all ranks' checksummed bytes / that time.
`--dry-run` runs the same sharding on the CPU (gloo, no GPU call) and checks
that the ranks cover every block exactly once.

Also reported: per-kernel roofline (HIP events on the launch stream, and the
kernel-trace average of the committed rocprofv3 profile of the same config),
HBM traffic from the committed PMC summary, the CPU baseline (oracle = our
restatement, timed on this host), the north-star point (1 M x 16 KiB, CRC32C
and XXH3), C3/C4, the legacy kxxHash / kxxHash64 types, the WAL config C5,
per-KV protection (a15) and the PCIe-inclusive end-to-end rates (DESIGN.md
§6).  At N = 1 with extras, bench.py runs the headline config and each extra
in a child process of its own (this process never touches the GPU) and prints
the merged line: each measurement starts from a fresh device allocation
state.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from forst_amd import shard  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
GIB = float(1 << 30)
METRIC = "device-resident GiB/s checksummed (CRC32C/XXH3), 4–64 KiB blocks, 1/2/4/8 GPU"

CONFIGS = {
    # name: (blocks per GPU, size spec, checksum, description)
    "C2": (1 << 20, 4096, 1, "1 M x 4 KiB kCRC32c compute+verify"),
    "C3": (1 << 20, (4096, 16384, 65536), 4, "1 M mixed 4/16/64 KiB kXXH3 compute+verify"),
    "C4": (1 << 19, 16384, 1, "compaction-shaped 8 GiB/GPU of 16 KiB kCRC32c compute+verify"),
    "NS16": (1 << 20, 16384, 1, "north-star 1 M x 16 KiB kCRC32c compute+verify"),
    "NS16X": (1 << 20, 16384, 4, "north-star 1 M x 16 KiB kXXH3 compute+verify"),
    "C3S": (1 << 20, ("sorted", (4096, 16384, 65536)), 4,
            "C3's blocks sorted by size (64 KiB, then 16 KiB, then 4 KiB) kXXH3 compute+verify"),
    # the two legacy selector types (format.cc:573-576, 603-622) at the
    # north-star shape
    "NS16H32": (1 << 20, 16384, 2, "1 M x 16 KiB kxxHash (XXH32) compute+verify"),
    "NS16H64": (1 << 20, 16384, 3, "1 M x 16 KiB kxxHash64 (XXH64) compute+verify"),
}
SEEDS = {"C2": 0xF0E5700002, "C3": 0xF0E5700003, "C4": 0xF0E5700004,
         "NS16": 0xF0E5700002, "NS16X": 0xF0E5700002, "C3S": 0xF0E5700003,
         "NS16H32": 0xF0E5700002, "NS16H64": 0xF0E5700002}


def algorithmic_bytes(kind, payload_bytes, n):
    """per-launch algorithmic HBM bytes:
    trailer: read n + type byte (1) + descriptor (12); write trailer (5)
    verify : read n+5 + descriptor (12); write computed (4) + ok (1)"""
    if kind == "trailer":
        return payload_bytes + n * (1 + 12 + 5)
    return payload_bytes + n * (5 + 12 + 4 + 1)


def describe(name, world):
    """the global batch of a config at world size N: N x n blocks (weak
    scaling), one splitmix64 byte stream; returns (sizes, ctype, desc, seed)"""
    from forst_amd import workload

    n, spec, ctype, desc = CONFIGS[name]
    seed = SEEDS[name]
    return workload.block_sizes(n * world, spec, seed), ctype, desc, seed


def run_config(name, steps, warmup, rank, world):
    from forst_amd import engine, workload

    sizes_all, ctype, desc, seed = describe(name, world)
    lo, hi, start = shard.rank_slice(sizes_all, rank, world)
    b = workload.make_sst_batch(hi - lo, None, seed, ctype=ctype, sizes=sizes_all[lo:hi],
                                stream_start=start)
    n = b.n
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    comp = torch.empty(n, dtype=torch.uint32, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step(ev=None):
        if ev:
            ev[0].record()
        engine.block_trailer_batch(ctype, b.base, b.offsets, b.sizes, b.types)
        if ev:
            ev[1].record()
        engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes, computed=comp,
                                  stored=None, ok=ok, mismatches=bad)
        if ev:
            ev[2].record()

    names = {}
    for _ in range(max(1, warmup)):
        engine.block_trailer_batch(ctype, b.base, b.offsets, b.sizes, b.types)
        names["trailer"] = engine.last_kernel()
        engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes, computed=comp,
                                  stored=None, ok=ok, mismatches=bad)
        names["verify"] = engine.last_kernel()
    torch.cuda.synchronize()
    bad.zero_()
    # HIP events on the launch stream (torch's current stream, which the
    # engine wrappers launch on)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    shard.barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(evs[k])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    shard.barrier(world)
    elapsed = shard.max_over_ranks(t1 - t0, world)
    mism = shard.sum_over_ranks(int(bad.item()), world)
    assert mism == 0, f"{mism} blocks failed verification in the timed region"
    blocks_total = shard.sum_over_ranks(n, world)
    assert blocks_total == len(sizes_all), "ranks must cover the described batch"
    t_tr = np.mean([e[0].elapsed_time(e[1]) for e in evs]) / 1e3
    t_vf = np.mean([e[1].elapsed_time(e[2]) for e in evs]) / 1e3
    bytes_all = int(sizes_all.astype(np.int64).sum()) + len(sizes_all)  # checksummed, all ranks
    res = {
        "name": name, "desc": desc, "n": n, "n_total": len(sizes_all), "ctype": ctype,
        "elapsed": elapsed, "steps": steps, "shard": [lo, hi],
        "gibs_total": 2 * bytes_all * steps / elapsed / GIB,
        "ms_per_step": elapsed / steps * 1e3,
        "kernels": {
            "trailer": {"name": names["trailer"], "avg_s": t_tr,
                        "alg_bytes": algorithmic_bytes("trailer", b.payload_bytes, n),
                        "gibs_checksummed": b.checksummed_bytes / t_tr / GIB},
            "verify": {"name": names["verify"], "avg_s": t_vf,
                       "alg_bytes": algorithmic_bytes("verify", b.payload_bytes, n),
                       "gibs_checksummed": b.checksummed_bytes / t_vf / GIB},
        },
        "batch": b,
    }
    for k in res["kernels"].values():
        k["achieved_gbs"] = k["alg_bytes"] / k["avg_s"] / 1e9
        k["frac"] = k["achieved_gbs"] / HBM_PEAK_GBS
    return res


def run_wal(steps, warmup, n_records=10_000_000):
    """C5 WAL replay: 10 M logical records log-uniform in
    [32, 32768] B framed by log::Writer's rules; writer-side record CRC pass
    (log_writer.cc EmitPhysicalRecord) + reader-side verify of every physical
    record CRC (log_reader.cc ReadPhysicalRecord).  Algorithmic bytes:
    verify  = whole log read + per log block status/nrec/fail_off (9 B);
    writer  = headers+payloads read + offset (8) + CRC written twice (in place
              and out, 4+4) per physical record;
    record XXH3 (a14) = payload bytes read + 8 B header offset + 8 B hash."""
    from forst_amd import engine, workload

    w = workload.make_wal_batch(n_records, workload.SEEDS["C5"])
    offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
    lens = torch.from_numpy(w.rec_lengths.astype(np.int32)).cuda()
    crc = torch.empty(len(w.rec_offsets), dtype=torch.uint32, device="cuda")
    nb = w.n_log_blocks
    st = torch.empty(nb, dtype=torch.uint8, device="cuda")
    nrec = torch.empty(nb, dtype=torch.uint32, device="cuda")
    fail = torch.empty(nb, dtype=torch.uint32, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    L = engine.lib()
    s0 = engine._stream(None)

    def verify():
        engine.check(L.forst_wal_verify_batch(w.log.data_ptr(), w.total, 0, nb, 0,
                                              st.data_ptr(), nrec.data_ptr(), fail.data_ptr(),
                                              bad.data_ptr(), s0))

    def write():  # the writer's own lengths (forst_wal_record_crc_lengths)
        engine.wal_record_crc_batch(w.log, offs, write_in_place=True, out=crc,
                                    payload_lengths=lens)

    for _ in range(max(1, warmup)):
        write()
        verify()
    torch.cuda.synchronize()
    bad.zero_()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in evs:
        e[0].record()
        write()
        e[1].record()
        verify()
        e[2].record()
    torch.cuda.synchronize()
    assert int(bad.item()) == 0, "WAL blocks failed verification in the timed region"
    assert int(nrec.sum().item()) == len(w.rec_offsets)
    # a14: XXH3 of every logical record; includes its stream synchronisations.
    # One untimed call first: the engine's scratch pool grows to this call's
    # sizes once (stream-ordered pool, release threshold = keep)
    engine.wal_record_xxh3_batch(w.log, offs)
    torch.cuda.synchronize()
    hs = []
    for _ in range(max(3, steps // 2)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hh, _ = engine.wal_record_xxh3_batch(w.log, offs)
        torch.cuda.synchronize()
        hs.append(time.perf_counter() - t0)
    assert hh.numel() == w.n_records
    t_h = float(np.median(hs))
    # f2: the fused recovery pass (walk + CRC + fragment state machine +
    # record XXH3, forst_wal_recover_batch), PIT recovery mode
    engine.wal_recover_batch(w.log, 0, engine.kPointInTimeRecovery,
                             record_capacity=w.n_records + 1024)  # untimed: pool growth
    torch.cuda.synchronize()
    rs = []
    for _ in range(max(3, steps // 2)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rec, rep, res = engine.wal_recover_batch(w.log, 0, engine.kPointInTimeRecovery,
                                                 record_capacity=w.n_records + 1024)
        torch.cuda.synchronize()
        rs.append(time.perf_counter() - t0)
    # (FORST_AB_TIMING_ONLY: timing-only A/B builds that drop result stores)
    assert (res.n_records == w.n_records and res.n_reports == 0) or \
        os.environ.get("FORST_AB_TIMING_ONLY") == "1"
    t_r = float(np.median(rs))
    t_w = np.mean([e[0].elapsed_time(e[1]) for e in evs]) / 1e3
    t_v = np.mean([e[1].elapsed_time(e[2]) for e in evs]) / 1e3
    payload = int(w.rec_lengths.astype(np.int64).sum())
    rec_bytes = payload + 7 * len(w.rec_offsets)
    alg_v = w.total + 9 * nb
    alg_w = rec_bytes + 16 * len(w.rec_offsets)
    alg_h = payload + 16 * len(w.rec_offsets)
    out = {"desc": f"{n_records} records log-uniform 32..32768 B, "
                   f"{w.total / GIB:.1f} GiB log, {len(w.rec_offsets)} physical records",
           "verify_GiBps": round(w.total / t_v / GIB, 1),
           "verify_ms": round(t_v * 1e3, 3),
           "verify_roofline_frac": round(alg_v / t_v / 1e9 / HBM_PEAK_GBS, 4),
           "writer_crc_GiBps": round(rec_bytes / t_w / GIB, 1),
           "writer_crc_ms": round(t_w * 1e3, 3),
           "writer_roofline_frac": round(alg_w / t_w / 1e9 / HBM_PEAK_GBS, 4),
           "record_xxh3_GiBps": round(payload / t_h / GIB, 1),
           "record_xxh3_ms": round(t_h * 1e3, 3),
           "record_xxh3_roofline_frac": round(alg_h / t_h / 1e9 / HBM_PEAK_GBS, 4),
           "recover_ms": round(t_r * 1e3, 3),
           "recover_GiBps": round(w.total / t_r / GIB, 1),
           "recover_desc": "forst_wal_recover_batch: header walk + every physical CRC + "
                           "fragment state machine + XXH3 of every logical record, "
                           "kPointInTimeRecovery, incl. its 5-6 stream synchronisations"}
    del w
    return out


def run_wal_sharded(steps, warmup, rank, world, n_per_gpu=10_000_000):
    """C5 at N GPUs: ONE WAL of N x 10 M records (weak
    scaling) whose 32 KiB log blocks are split into N equal contiguous ranges,
    rank r verifying range r (forst_wal_verify_batch; db/log_reader.cc:450-531
    checks each log block on its own, physical records never straddle one,
    log_writer.cc:86-102).  No collective on the data path: barrier +
    synchronize around the timed steps, max over ranks; value = the whole
    log's bytes / that time."""
    from forst_amd import engine, workload

    lengths = workload.log_uniform_lengths(n_per_gpu * world, 32, 32768, workload.SEEDS["C5"])
    _, _, _, _, _, total = workload.wal_layout(lengths)
    nb = (total + 32767) // 32768
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    w = workload.make_wal_batch(0, workload.SEEDS["C5"], lengths=lengths, block_range=(b0, b1))
    del lengths
    n = b1 - b0
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    nrec = torch.empty(n, dtype=torch.uint32, device="cuda")
    fail = torch.empty(n, dtype=torch.uint32, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    L = engine.lib()
    s0 = engine._stream(None)

    def verify():
        engine.check(L.forst_wal_verify_batch(w.log.data_ptr(), w.total, 0, n, 0, st.data_ptr(),
                                              nrec.data_ptr(), fail.data_ptr(), bad.data_ptr(), s0))

    for _ in range(max(1, warmup)):
        verify()
    torch.cuda.synchronize()
    bad.zero_()
    shard.barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        verify()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    shard.barrier(world)
    elapsed = shard.max_over_ranks(t1 - t0, world)
    assert shard.sum_over_ranks(int(bad.item()), world) == 0, "WAL blocks failed verification"
    assert shard.sum_over_ranks(int(nrec.sum().item()), world) == \
        shard.sum_over_ranks(len(w.rec_offsets), world)
    out = {"desc": f"one WAL of {n_per_gpu * world} records log-uniform 32..32768 B "
                   f"({total / GIB:.1f} GiB), its log blocks in {world} equal contiguous ranges, "
                   "one per GPU, forst_wal_verify_batch",
           "GiBps": round(total * steps / elapsed / GIB, 1),
           "ms_per_step": round(elapsed / steps * 1e3, 3),
           "roofline_frac_per_gpu": round((total + 9 * nb) * steps / elapsed / 1e9 /
                                          HBM_PEAK_GBS / world, 4)}
    del w
    return out


def run_kv(steps, warmup, n=1 << 20):
    """a15 per-KV protection (db/kv_checksum.h:296 ProtectKVO + ProtectS, the
    WriteBatch / memtable shape; MemTable::VerifyEntryChecksum memtable.cc:273
    for the read side) on 1 M memtable-shaped entries: 16-64 B keys, 0-1000 B
    values, 8-byte protection stored after each value (the batch of
    tests/test_gpu_parity.py test_kv_full_size_roundtrip).  Algorithmic bytes:
    protect = key + value bytes + 33 B of descriptors (key/value offset 8+8,
    sizes 4+4, op 1, seq 8) read + 8 B written; verify = the same + 8 B
    checksum offset + 8 B stored protection read + 8 B computed + 1 B ok
    written."""
    from forst_amd import engine

    rng = np.random.default_rng(99)
    ks = rng.integers(16, 65, n).astype(np.int64)
    vs = rng.integers(0, 1001, n).astype(np.int64)
    ko = np.zeros(n, np.int64)
    ko[1:] = np.cumsum(ks[:-1] + vs[:-1] + 8)
    vo = ko + ks
    co = vo + vs
    total = int(co[-1]) + 8
    base = torch.empty((total + 255) // 256 * 256, dtype=torch.uint8, device="cuda")
    engine.fill_stream(base, 0, 0xF0E57000A15)
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    dko, dks, dvo, dvs, dco = dev(ko), dev(ks.astype(np.int32)), dev(vo), dev(vs.astype(np.int32)), dev(co)
    ops = dev(rng.integers(0, 26, n).astype(np.uint8))
    seqs = dev(rng.integers(0, 2**62, n).astype(np.int64))
    prot = torch.empty(n, dtype=torch.uint64, device="cuda")
    comp = torch.empty(n, dtype=torch.uint64, device="cuda")
    okv = torch.empty(n, dtype=torch.uint8, device="cuda")
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    engine.kv_protect_batch(base, dko, dks, dvo, dvs, ops, seqs, out=prot)
    idx = dco[:, None] + torch.arange(8, device="cuda")[None, :]
    base[idx.reshape(-1)] = prot.view(torch.uint8).view(n, 8).reshape(-1)  # Encode(8)
    del idx

    def protect():
        engine.kv_protect_batch(base, dko, dks, dvo, dvs, ops, seqs, out=prot)

    def verify():
        engine.kv_verify_batch(base, dko, dks, dvo, dvs, 8, dco, ops, seqs, computed=comp, ok=okv,
                               mismatches=bad)

    for _ in range(max(1, warmup)):
        protect()
        verify()
    torch.cuda.synchronize()
    bad.zero_()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in evs:
        e[0].record()
        protect()
        e[1].record()
        verify()
        e[2].record()
    torch.cuda.synchronize()
    assert int(bad.item()) == 0, "KV entries failed verification in the timed region"
    t_p = np.mean([e[0].elapsed_time(e[1]) for e in evs]) / 1e3
    t_v = np.mean([e[1].elapsed_time(e[2]) for e in evs]) / 1e3
    kvb = int((ks + vs).sum())
    alg_p = kvb + 41 * n
    alg_v = kvb + 74 * n
    name_v = engine.last_kernel()
    return {"desc": f"{n} entries, keys 16-64 B, values 0-1000 B, ProtectKVO + ProtectS, "
                    f"8-byte protection ({kvb / GIB:.2f} GiB of key+value bytes)",
            "protect_ms": round(t_p * 1e3, 4), "verify_ms": round(t_v * 1e3, 4),
            "protect_Mentries_per_s": round(n / t_p / 1e6, 1),
            "verify_Mentries_per_s": round(n / t_v / 1e6, 1),
            "protect_roofline_frac": round(alg_p / t_p / 1e9 / HBM_PEAK_GBS, 4),
            "verify_roofline_frac": round(alg_v / t_v / 1e9 / HBM_PEAK_GBS, 4),
            "verify_kernel": name_v}


def cpu_info():
    """the host CPU the baseline ran on: model, current clock of the CPUs the
    process may use (/proc/cpuinfo, MHz as the kernel reports it at the time),
    and the affinity list"""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    model, mhz = None, {}
    try:
        cpu = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    cpu = int(v)
                elif k == "model name" and model is None:
                    model = v
                elif k == "cpu MHz" and cpu is not None:
                    mhz[cpu] = float(v)
    except OSError:
        pass
    mine = [mhz[c] for c in aff if c in mhz]

    def ranges(xs):
        out, i = [], 0
        while i < len(xs):
            j = i
            while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
                j += 1
            out.append(f"{xs[i]}-{xs[j]}" if j > i else str(xs[i]))
            i = j + 1
        return ",".join(out)

    return {"cpu_model": model, "affinity": ranges(aff), "affinity_count": len(aff),
            "mhz_median": round(float(np.median(mine)), 0) if mine else None,
            "mhz_min": round(min(mine), 0) if mine else None,
            "mhz_max": round(max(mine), 0) if mine else None}


def cpu_threads():
    """(threads to use, how the count was found): every CPU this process may
    run on (sched_getaffinity), capped by a cgroup CPU quota when one is set;
    os.cpu_count() is reported beside it."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    how = "sched_getaffinity"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            cap = max(1, int(int(q) // int(p)))
            if cap < n:
                n, how = cap, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    return max(1, n or 1), how


def cpu_baseline(b, ctype, budget_s=12.0):
    """Time the oracle (our CPU restatement, compiled -O3 -march=x86-64-v3 with
    SSE4.2 crc32 3-way + AVX2 XXH3) on a bounded sample of the same blocks,
    on every CPU this process may use, and on one thread."""
    from oracle import oracle as O

    nthreads, how = cpu_threads()
    ns = min(b.n, 1 << 18)  # up to 256 K blocks (~1 GiB of 4 KiB blocks)
    offs = b.offsets[:ns].cpu().numpy()
    sizes = b.sizes[:ns].cpu().numpy().astype(np.uint32)
    end = int(offs[-1]) + int(sizes[-1]) + 5
    hb = b.base[:end].cpu().numpy()
    offs = offs.astype(np.uint64)
    types = np.zeros(ns, dtype=np.uint8)
    sample_bytes = int(sizes.astype(np.int64).sum()) + ns

    def one_pass(nt):
        t = time.perf_counter()
        O.block_checksum_batch(ctype, hb, offs, sizes, last_bytes=types, nthreads=nt)
        _, _, bad = O.block_verify_batch(ctype, hb, offs, sizes, nthreads=nt)
        dt = time.perf_counter() - t
        assert bad == 0
        return dt

    res = {}
    for nt in sorted({nthreads, 1}, reverse=True):
        one_pass(nt)  # warm
        best, spent, reps = 1e30, 0.0, 0
        while reps < 5 and spent < budget_s / 2:
            dt = one_pass(nt)
            best, spent, reps = min(best, dt), spent + dt, reps + 1
        res[nt] = 2 * sample_bytes / best / GIB
    # one thread on the first 256 blocks (~1 MiB, cache-resident), repeated:
    # the core's own rate, to tell a slow core from a memory-bound sample
    nc = min(ns, 256)
    cb = int(sizes[:nc].astype(np.int64).sum()) + nc
    best_c = 1e30
    for _ in range(200):
        t = time.perf_counter()
        O.block_verify_batch(ctype, hb, offs[:nc], sizes[:nc], nthreads=1)
        best_c = min(best_c, time.perf_counter() - t)
    return {"value": round(res[nthreads], 3), "unit": "GiB/s", "cores": nthreads, "kind": "port",
            "cores_from": how, "host_os_cpu_count": os.cpu_count(),
            "sample": f"first {ns} blocks of the same batch ({sample_bytes / GIB:.2f} GiB "
                      f"checksummed per pass), compute+verify, best of <=5, "
                      f"oracle/oracle.c -O3 x86-64-v3 (SSE4.2 crc32 3-way, AVX2 XXH3), "
                      f"one std::thread per core over contiguous block ranges",
            "single_thread_GiBps": round(res[1], 3),
            "single_thread_cached_GiBps": round(cb / best_c / GIB, 3),
            "host": cpu_info()}


def end_to_end_pcie(b, ctype, chunk_blocks=1 << 16):
    """Host (pinned) -> HBM -> verify -> host results, double-buffered on two
    streams; returns PCIe-inclusive GiB/s checksummed.  Recorded in DESIGN.md,
    never the headline value."""
    from forst_amd import engine

    n = b.n
    offs = b.offsets.cpu().numpy()
    sizes = b.sizes.cpu().numpy()
    host = b.base.cpu().pin_memory()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    max_bytes = 0
    chunks = []
    for c0 in range(0, n, chunk_blocks):
        c1 = min(n, c0 + chunk_blocks)
        lo = int(offs[c0])
        hi = int(offs[c1 - 1]) + int(sizes[c1 - 1]) + 5
        chunks.append((c0, c1, lo, hi))
        max_bytes = max(max_bytes, hi - lo)
    dbufs = [torch.empty(max_bytes + 256, dtype=torch.uint8, device="cuda") for _ in streams]
    doffs = [torch.empty(chunk_blocks, dtype=torch.int64, device="cuda") for _ in streams]
    oks = torch.empty(n, dtype=torch.uint8).pin_memory()
    dok = [torch.empty(chunk_blocks, dtype=torch.uint8, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, (c0, c1, lo, hi) in enumerate(chunks):
        s = streams[k & 1]
        with torch.cuda.stream(s):
            dbufs[k & 1][:hi - lo].copy_(host[lo:hi], non_blocking=True)
            doffs[k & 1][:c1 - c0].copy_(b.offsets[c0:c1] - lo)
            engine.block_verify_batch(ctype, dbufs[k & 1][:hi - lo], doffs[k & 1][:c1 - c0],
                                      b.sizes[c0:c1], computed=None, stored=None,
                                      ok=dok[k & 1][:c1 - c0], stream=s)
            oks[c0:c1].copy_(dok[k & 1][:c1 - c0], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert bool(oks.all())
    return b.checksummed_bytes / dt / GIB


def host_paths(b, ctype, sample_blocks=1 << 18):
    """Blocks starting in HOST memory through the in-process multi-device entry
    (forst_block_verify_host: per device a host thread + stream + pinned
    staging, 64 MiB windows double-buffered): pageable input (memcpy into
    pinned staging), pinned input (DMA in place), and an SST-shaped file
    mmap'd read-only and hipHostRegister'd (env/io_posix.cc:958).  PCIe-bound;
    recorded in DESIGN.md, never the headline value."""
    import tempfile
    from forst_amd import hostpath

    ns = min(b.n, sample_blocks)
    offs = b.offsets[:ns].cpu().numpy().astype(np.uint64)
    sizes = b.sizes[:ns].cpu().numpy().astype(np.uint32)
    end = int(offs[-1]) + int(sizes[-1]) + 5
    pageable = b.base[:end].cpu().numpy().copy()
    nbytes = int(sizes.astype(np.int64).sum()) + ns
    ndev = torch.cuda.device_count()
    out = {"sample": f"first {ns} blocks ({nbytes / GIB:.2f} GiB checksummed)",
           "devices": list(range(ndev))}

    first = {}

    def rate(base, devices, key=None):
        best = 1e30
        for k in range(3):
            t0 = time.perf_counter()
            _, _, ok, bad = hostpath.block_verify_host(ctype, base, offs, sizes, devices=devices)
            dt = time.perf_counter() - t0
            if k == 0 and key:
                first[key] = round(nbytes / dt / GIB, 2)
            best = min(best, dt)
            assert bad == 0
        return round(nbytes / best / GIB, 2)

    # (the first call of the process also creates the device's host context:
    # worker thread, stream, windows and pinned staging)
    out["pageable_GiBps"] = rate(pageable, list(range(ndev)), "pageable_incl_context_creation")
    out["pageable_2streams_per_gpu_GiBps"] = rate(pageable, [d for d in range(ndev) for _ in (0, 1)])
    t0 = time.perf_counter()
    pinned = torch.from_numpy(pageable).pin_memory()
    out["pin_memory_s"] = round(time.perf_counter() - t0, 4)
    out["pinned_GiBps"] = rate(pinned.numpy(), list(range(ndev)), "pinned")
    del pinned
    d = os.environ.get("TMPDIR", tempfile.gettempdir())
    path = os.path.join(d, f"forst_bench_{os.getpid()}.sst")
    try:
        pageable.tofile(path)
        # a fresh mapping of the file (in the page cache: just written), the
        # way a one-shot VerifyChecksum sees an SST: map, register, verify once
        t0 = time.perf_counter()
        m = hostpath.MappedFile(path, register=False)
        t1 = time.perf_counter()
        from forst_amd._lib import lib
        rc = lib().forst_host_register(m.address, m.size)
        t2 = time.perf_counter()
        m.registered = rc == 0
        out["mmap_registered"] = m.registered
        if not m.registered:
            out["mmap_register_error"] = lib().forst_host_last_error().decode(errors="replace")
        out["mmap_GiBps"] = rate(m, list(range(ndev)), "mmap_registered_verify")
        m.close()
        # the same without registration: staged through pinned memory
        m = hostpath.MappedFile(path, register=False)
        out["mmap_unregistered_GiBps"] = rate(m, list(range(ndev)), "mmap_unregistered")
        m.close()
        out["cold"] = {
            "mmap_populate_s": round(t1 - t0, 4), "register_s": round(t2 - t1, 4),
            "register_GiBps": round(m.size / (t2 - t1) / GIB, 2),
            "first_call_GiBps": first,
            "mmap_register_plus_first_verify_GiBps": round(
                nbytes / ((t2 - t1) + nbytes / first["mmap_registered_verify"] / GIB) / GIB, 2)}
    except OSError as e:  # pragma: no cover
        out["mmap_error"] = str(e)
    finally:
        if os.path.exists(path):
            os.unlink(path)
    return out


def _norm_kernel(name):
    """rocprof / engine kernel names -> one form: 'crc32c_rows_kernel<verify>'"""
    import re
    modes = {"0": "compute", "1": "trailer", "2": "verify", "3": "raw"}
    n = name.replace("forst::(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(forst::")[0].split("(unsigned")[0].strip()
    # xxhash_lane_kernel<MODE, X64> (rocprof) -> xxhash32/64_lane_kernel<mode> (engine)
    n = re.sub(r"^xxhash_lane_kernel<(\d), (true|false)>$",
               lambda m: f"xxhash{64 if m.group(2) == 'true' else 32}_lane_kernel<{m.group(1)}>", n)
    if n.startswith("kv_kernel<"):  # KvMode (engine.h), not the block modes
        kv = {"0": "hash64", "1": "protect", "2": "verify", "3": "mem_verify", "4": "mem_protect"}
        return re.sub(r"<(\d)>", lambda m: "<" + kv[m.group(1)] + ">", n)
    return re.sub(r"<(\d)>", lambda m: "<" + modes[m.group(1)] + ">", n)


def load_profile(kernel_name, config):
    """(kernel-trace average ns, HBM bytes per launch) of the dominant kernel
    from the newest committed rocprofv3 summary of this config
    (profiles/pmc_<tag>_<config>.json, written by profiles/summarize.py from
    a --kernel-trace --stats pass and separate FETCH_SIZE / WRITE_SIZE
    passes), or (None, None)."""
    parts = [_norm_kernel(p) for p in kernel_name.split("+")]
    best = (None, None, None, None)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc_*_{config}.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        rows = {_norm_kernel(r.get("kernel", "")): r for r in d.get("kernels", [])}
        if all(p in rows for p in parts):
            traffic = sum(rows[p].get("hbm_bytes_per_launch") or 0 for p in parts)
            ns = sum(rows[p].get("avg_duration_ns_kernel_trace") or 0 for p in parts)
            # the profiled run's timed steps alone (newer summaries)
            tns = [rows[p].get("avg_duration_ns_timed_steps") for p in parts]
            tns = sum(tns) if all(v is not None for v in tns) else None
            best = (ns or None, traffic or None, os.path.basename(f), tns)
    return best


def spawn_ranks(args):
    """Start one process per GPU under torch.distributed.run (a child process,
    started before any GPU call) and return its exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """the sharding of the described batch, on the CPU (gloo): every block
    exactly once, byte-balanced"""
    sizes_all, ctype, desc, seed = describe(args.config, world)
    lo, hi, start = shard.rank_slice(sizes_all, rank, world)
    got = [None] * world
    if world > 1:
        dist.all_gather_object(got, (lo, hi, start, int(sizes_all[lo:hi].astype(np.int64).sum())))
    else:
        got = [(lo, hi, start, int(sizes_all.astype(np.int64).sum()))]
    if rank == 0:
        cover = np.zeros(len(sizes_all), np.int32)
        for lo_, hi_, _, _ in got:
            cover[lo_:hi_] += 1
        offs = np.concatenate([[0], np.cumsum(sizes_all.astype(np.int64) + 5)])
        print(json.dumps({"dry_run": True, "config": args.config, "n_gpus": world,
                          "blocks_total": len(sizes_all),
                          "every_block_once": bool((cover == 1).all()),
                          "starts_match": all(int(offs[lo_]) == st for lo_, _, st, _ in got),
                          "shards": [{"lo": g[0], "hi": g[1], "bytes": g[3]} for g in got]}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_child(argv, timeout=600):
    """bench.py <argv> in a child process (this process has not touched the
    GPU); returns its last stdout line as JSON"""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    sys.stderr.write(r.stderr[-4000:])
    if r.returncode != 0:
        raise RuntimeError(f"bench.py {' '.join(argv)} failed ({r.returncode})")
    return json.loads(r.stdout.strip().splitlines()[-1])


EXTRA_SST = ("NS16", "NS16X", "C3", "C3S", "C4", "NS16H32", "NS16H64")


def orchestrate(args):
    """N = 1 with extras: the headline config (plus the CPU baseline and the
    host-memory paths) and every extra run in a child process of its own, one
    after the other, so each starts from a fresh device allocation state (in
    one process, a 28 GiB batch allocated after another one measured 3-7 %
    slower: C3 / C3S in BENCH_r04, bench_r05a).  This process never touches
    the GPU; it merges the children's lines into the one JSON line."""
    common = ["--steps", str(args.steps), "--warmup", str(args.warmup)]
    line = run_child(["--config", args.config, "--child"] + common +
                     (["--no-cpu-baseline"] if args.no_cpu_baseline else []))
    extras = line.setdefault("extras", {})
    for nm in EXTRA_SST + ("C5_wal", "a15_kv"):
        try:
            extras[nm] = run_child(["--extra", nm] + common)
        except Exception as e:  # pragma: no cover
            extras[nm + "_error"] = str(e)
    print(json.dumps(line), flush=True)
    return 0


def run_extra(name, steps, warmup):
    """one extra of the N = 1 bench line (a child of orchestrate)"""
    from forst_amd import engine

    engine.init_device()
    if name == "C5_wal":
        return run_wal(max(3, steps // 2), 1)
    if name == "a15_kv":
        return run_kv(steps, warmup)
    r = run_config(name, steps, warmup, 0, 1)
    r.pop("batch")
    kv, kt = r["kernels"]["verify"], r["kernels"]["trailer"]
    ns, _, _, tns = load_profile(kv["name"], name)
    return {
        "desc": r["desc"], "GiBps": round(r["gibs_total"], 1),
        "verify_kernel_GiBps": round(kv["gibs_checksummed"], 1),
        "verify_roofline_frac": round(kv["frac"], 4),
        "verify_roofline_frac_kernel_trace": (
            round(kv["alg_bytes"] / (ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4) if ns else None),
        "verify_roofline_frac_kernel_trace_timed_steps": (
            round(kv["alg_bytes"] / (tns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4) if tns else None),
        "trailer_kernel_GiBps": round(kt["gibs_checksummed"], 1),
        "trailer_roofline_frac": round(kt["frac"], 4),
        "verify_kernel": kv["name"], "trailer_kernel": kt["name"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip north-star, C3/C4, C5 and end-to-end extras")
    ap.add_argument("--dry-run", action="store_true",
                    help="shard the described batch on the CPU (gloo) without a GPU")
    ap.add_argument("--child", action="store_true",
                    help="(orchestrate) the headline config + CPU baseline + host-memory paths")
    ap.add_argument("--extra", default=None,
                    help="(orchestrate) one extra: an SST config, C5_wal or a15_kv")
    args = ap.parse_args()

    if args.extra:
        print(json.dumps(run_extra(args.extra, args.steps, args.warmup)), flush=True)
        return
    if (args.gpus == 1 and "WORLD_SIZE" not in os.environ and not args.dry_run and
            not args.child and not args.no_extras and args.config == "C2"):
        sys.exit(orchestrate(args))

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world, rank, local = shard.setup(cpu_only=args.dry_run)
    if "WORLD_SIZE" in os.environ:
        assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE={world}"
    if world > 1:
        assert dist.get_world_size() == world
    if args.dry_run:
        return dry_run(args, world, rank)
    from forst_amd import engine

    engine.init_device()
    main_res = run_config(args.config, args.steps, args.warmup, rank, world)
    b = main_res.pop("batch")
    extras = {}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(b, main_res["ctype"])
    if world == 1 and (args.child or not args.no_extras):
        try:
            # the first pass pays one-time costs (host pinning, first touch of
            # the staging buffers): best of 3 passes, the first reported too
            e2e = [end_to_end_pcie(b, main_res["ctype"]) for _ in range(3)]
            extras["end_to_end_pcie_GiBps"] = round(max(e2e), 2)
            extras["end_to_end_pcie_first_pass_GiBps"] = round(e2e[0], 2)
        except Exception as e:  # pragma: no cover
            extras["end_to_end_pcie_error"] = str(e)
        try:
            extras["host_memory_verify"] = host_paths(b, main_res["ctype"])
        except Exception as e:  # pragma: no cover
            extras["host_memory_verify_error"] = str(e)
    del b
    torch.cuda.empty_cache()
    if world > 1 and not args.no_extras:
        # (no try: every rank takes part in its barriers; a failure ends the run)
        extras["C5_wal_verify_sharded"] = run_wal_sharded(max(3, args.steps // 2), 1, rank, world)
        torch.cuda.empty_cache()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    kv = main_res["kernels"]["verify"]
    kt = main_res["kernels"]["trailer"]
    dom = kv if kv["avg_s"] >= kt["avg_s"] else kt
    ns, traffic, prof, tns = load_profile(dom["name"], args.config)
    line = {
        "metric": METRIC,
        "value": round(main_res["gibs_total"], 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(main_res["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 payloads, SST-packed unaligned blocks, trailers "
                "written by the write-side kernel)",
        "config": {"workload": f"{args.config}: {main_res['desc']}",
                   "blocks_per_gpu": main_res["n"],
                   "blocks_total": main_res["n_total"],
                   "checksum": {1: "kCRC32c", 2: "kxxHash", 3: "kxxHash64", 4: "kXXH3"}[main_res["ctype"]],
                   "step": "trailer pass (write side) + verify pass (read side)",
                   "parallelism": f"byte-balanced block shards of one batch x{world}, "
                                  "no data-path collective"},
        "roofline": {"bound": "hbm", "kernel": dom["name"],
                     "achieved": round(dom["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(dom["frac"], 4), "traffic": traffic,
                     "alg_bytes_per_launch": dom["alg_bytes"],
                     "avg_ms_hip_events": round(dom["avg_s"] * 1e3, 4),
                     "avg_ms_kernel_trace": round(ns / 1e6, 4) if ns else None,
                     "frac_kernel_trace": (round(dom["alg_bytes"] / (ns * 1e-9) / 1e9
                                                 / HBM_PEAK_GBS, 4) if ns else None),
                     "avg_ms_kernel_trace_timed_steps": round(tns / 1e6, 4) if tns else None,
                     "frac_kernel_trace_timed_steps": (
                         round(dom["alg_bytes"] / (tns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
                         if tns else None),
                     "profile": prof},
        "cpu_baseline": cpu,
        "kernels": {k: {"name": v["name"], "avg_ms": round(v["avg_s"] * 1e3, 4),
                        "alg_bytes": v["alg_bytes"],
                        "achieved_GBps": round(v["achieved_gbs"], 1),
                        "frac": round(v["frac"], 4),
                        "GiBps_checksummed": round(v["gibs_checksummed"], 1)}
                    for k, v in main_res["kernels"].items()},
        "extras": extras,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
