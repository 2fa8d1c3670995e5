#!/usr/bin/env python3
"""bench.py -- device-resident block-checksum throughput on MI355X.

Metric (BASELINE.json): device-resident GiB/s checksummed (CRC32C/XXH3).
Default workload = configs[1] ("C2"): 1 M x 4 KiB SST blocks, kCRC32c,
compute (write side: trailer kernel, ComputeBuiltinChecksumWithLastByte +
trailer, block_based_table_builder.cc:1340) + verify (read side,
VerifyBlockChecksum, reader_common.cc:26).  One step = both passes over the
whole batch; checksummed bytes per pass = sum(size + 1).

Multi-GPU: one process per GPU (torch.distributed.run), each rank owns its
own shard of blocks (weak scaling, no data-path collective: blocks are
independent -- SURVEY.md §8e); barrier + synchronize bracket the timed steps,
the max over ranks is reported and value = all ranks' bytes / that time.

Also reported: per-kernel roofline (HIP events on the launch stream),
the CPU baseline (oracle = our restatement, timed on this host), the
north-star point (1 M x 16 KiB, CRC32C and XXH3) and the PCIe-inclusive
end-to-end rate.
"""
import argparse
import glob
import json
import os
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
    # name: (n_blocks, size spec, checksum, description)
    "C2": (1 << 20, 4096, 1, "1 M x 4 KiB kCRC32c compute+verify"),
    "C3": (1 << 20, (4096, 16384, 65536), 4, "1 M mixed 4/16/64 KiB kXXH3 compute+verify"),
    "C4": (1 << 19, 16384, 1, "compaction-shaped 8 GiB/GPU of 16 KiB kCRC32c compute+verify"),
    "NS16": (1 << 20, 16384, 1, "north-star 1 M x 16 KiB kCRC32c compute+verify"),
    "NS16X": (1 << 20, 16384, 4, "north-star 1 M x 16 KiB kXXH3 compute+verify"),
}


def dist_setup():
    return shard.setup()


def barrier(world):
    shard.barrier(world)


def max_over_ranks(x, world):
    return shard.max_over_ranks(x, world)


def algorithmic_bytes(kind, b):
    """per-launch algorithmic HBM bytes:
    trailer: read n + type byte (1) + descriptor (12); write trailer (5)
    verify : read n+5 + descriptor (12); write computed (4) + ok (1)"""
    if kind == "trailer":
        return b.payload_bytes + b.n * (1 + 12 + 5)
    return b.payload_bytes + b.n * (5 + 12 + 4 + 1)


def run_config(name, steps, warmup, rank, world, seed_base=None):
    from forst_amd import engine, workload

    n, spec, ctype, desc = CONFIGS[name]
    seed = workload.SEEDS.get(name[:2], 0xF0E5700002) + rank * 0x1000
    b = workload.make_sst_batch(n, spec, seed, ctype=ctype)
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
    for w in range(max(1, warmup)):
        engine.block_trailer_batch(ctype, b.base, b.offsets, b.sizes, b.types)
        names["trailer"] = engine.last_kernel()
        engine.block_verify_batch(ctype, b.base, b.offsets, b.sizes, computed=comp,
                                  stored=None, ok=ok, mismatches=bad)
        names["verify"] = engine.last_kernel()
    torch.cuda.synchronize()
    bad.zero_()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(evs[k])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(t1 - t0, world)
    mism = int(bad.item())
    assert mism == 0, f"{mism} blocks failed verification in the timed region"
    t_tr = np.mean([e[0].elapsed_time(e[1]) for e in evs]) / 1e3
    t_vf = np.mean([e[1].elapsed_time(e[2]) for e in evs]) / 1e3
    bytes_per_step = 2 * b.checksummed_bytes
    res = {
        "name": name, "desc": desc, "n": n, "ctype": ctype,
        "elapsed": elapsed, "steps": steps,
        "gibs_total": bytes_per_step * steps * world / elapsed / GIB,
        "ms_per_step": elapsed / steps * 1e3,
        "kernels": {
            "trailer": {"name": names["trailer"],
                        "avg_s": t_tr, "alg_bytes": algorithmic_bytes("trailer", b),
                        "gibs_checksummed": b.checksummed_bytes / t_tr / GIB},
            "verify": {"name": names["verify"],
                       "avg_s": t_vf, "alg_bytes": algorithmic_bytes("verify", b),
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
              and out, 4+4) per physical record."""
    from forst_amd import engine, workload

    w = workload.make_wal_batch(n_records, workload.SEEDS["C5"])
    offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
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

    def write():
        engine.wal_record_crc_batch(w.log, offs, write_in_place=True, out=crc)

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
    # a14: XXH3 of every logical record (gather of multi-fragment records +
    # two raw XXH3 batches); includes its one stream synchronisation
    hs = []
    for _ in range(max(2, steps // 2)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hh, _ = engine.wal_record_xxh3_batch(w.log, offs)
        torch.cuda.synchronize()
        hs.append(time.perf_counter() - t0)
    assert hh.numel() == w.n_records
    t_h = float(np.median(hs))
    t_w = np.mean([e[0].elapsed_time(e[1]) for e in evs]) / 1e3
    t_v = np.mean([e[1].elapsed_time(e[2]) for e in evs]) / 1e3
    rec_bytes = int(w.rec_lengths.astype(np.int64).sum()) + 7 * len(w.rec_offsets)
    alg_v = w.total + 9 * nb
    alg_w = rec_bytes + 16 * len(w.rec_offsets)
    out = {"desc": f"{n_records} records log-uniform 32..32768 B, "
                   f"{w.total / GIB:.1f} GiB log, {len(w.rec_offsets)} physical records",
           "verify_GiBps": round(w.total / t_v / GIB, 1),
           "verify_ms": round(t_v * 1e3, 3),
           "verify_roofline_frac": round(alg_v / t_v / 1e9 / HBM_PEAK_GBS, 4),
           "writer_crc_GiBps": round(rec_bytes / t_w / GIB, 1),
           "writer_crc_ms": round(t_w * 1e3, 3),
           "writer_roofline_frac": round(alg_w / t_w / 1e9 / HBM_PEAK_GBS, 4),
           "record_xxh3_GiBps": round(rec_bytes / t_h / GIB, 1),
           "record_xxh3_ms": round(t_h * 1e3, 3)}
    del w
    return out


def cpu_baseline(b, ctype, budget_s=12.0):
    """Time the oracle (our CPU restatement, compiled -O3 -march=x86-64-v3 with
    SSE4.2 crc32 3-way + AVX2 XXH3) on a bounded sample of the same blocks."""
    from oracle import oracle as O

    nthreads = min(16, os.cpu_count() or 1)
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
    for nt in (nthreads, 1):
        one_pass(nt)  # warm
        best, spent, reps = 1e30, 0.0, 0
        while reps < 5 and spent < budget_s / 2:
            dt = one_pass(nt)
            best, spent, reps = min(best, dt), spent + dt, reps + 1
        res[nt] = 2 * sample_bytes / best / GIB
    return {"value": round(res[nthreads], 3), "unit": "GiB/s", "cores": nthreads, "kind": "port",
            "sample": f"first {ns} blocks of the same batch ({sample_bytes / GIB:.2f} GiB "
                      f"checksummed per pass), compute+verify, best of <=5, "
                      f"oracle/oracle.c -O3 x86-64-v3 (SSE4.2 crc32 3-way, AVX2 XXH3)",
            "single_thread_GiBps": round(res[1], 3)}


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
    rel = (b.offsets - 0)  # device copy reused per chunk
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k, (c0, c1, lo, hi) in enumerate(chunks):
        s = streams[k & 1]
        with torch.cuda.stream(s):
            dbufs[k & 1][:hi - lo].copy_(host[lo:hi], non_blocking=True)
            doffs[k & 1][:c1 - c0].copy_(rel[c0:c1] - lo)
            engine.block_verify_batch(ctype, dbufs[k & 1][:hi - lo], doffs[k & 1][:c1 - c0],
                                      b.sizes[c0:c1], computed=None, stored=None,
                                      ok=dok[k & 1][:c1 - c0], stream=s)
            oks[c0:c1].copy_(dok[k & 1][:c1 - c0], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert bool(oks.all())
    return b.checksummed_bytes / dt / GIB


def load_traffic(kernel_name, config):
    """HBM traffic per launch from the committed rocprofv3 PMC summary
    (profiles/*pmc*.json written by profiles/collect_pmc.py), or None."""
    parts = kernel_name.split("+")  # a pass of several kernels: sum of their traffic
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except Exception:
            continue
        got = {}
        for row in d.get("kernels", []):
            for p in parts:
                if row.get("config") == config and row.get("kernel", "").startswith(p):
                    got[p] = row.get("hbm_bytes_per_launch")
        if len(got) == len(parts) and all(v is not None for v in got.values()):
            best = sum(got.values())
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip north-star and end-to-end extras")
    args = ap.parse_args()

    world, rank, local = dist_setup()
    from forst_amd import engine

    engine.init_device()
    main_res = run_config(args.config, args.steps, args.warmup, rank, world)
    b = main_res.pop("batch")
    extras = {}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(b, main_res["ctype"])
    if world == 1 and not args.no_extras:
        try:
            extras["end_to_end_pcie_GiBps"] = round(end_to_end_pcie(b, main_res["ctype"]), 2)
        except Exception as e:  # pragma: no cover
            extras["end_to_end_pcie_error"] = str(e)
    del b
    torch.cuda.empty_cache()
    if world == 1 and not args.no_extras and args.config == "C2":
        for nm in ("NS16", "NS16X", "C3", "C4"):
            r = run_config(nm, max(3, args.steps // 2), 1, rank, world)
            r.pop("batch")
            torch.cuda.empty_cache()
            extras[nm] = {
                "desc": r["desc"], "GiBps": round(r["gibs_total"], 1),
                "verify_kernel_GiBps": round(r["kernels"]["verify"]["gibs_checksummed"], 1),
                "verify_roofline_frac": round(r["kernels"]["verify"]["frac"], 4),
                "trailer_kernel_GiBps": round(r["kernels"]["trailer"]["gibs_checksummed"], 1),
                "trailer_roofline_frac": round(r["kernels"]["trailer"]["frac"], 4),
                "verify_kernel": r["kernels"]["verify"]["name"],
                "trailer_kernel": r["kernels"]["trailer"]["name"]}
    if world == 1 and not args.no_extras and args.config == "C2":
        extras["C5_wal"] = run_wal(max(3, args.steps // 2), 1)
        torch.cuda.empty_cache()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    kv = main_res["kernels"]["verify"]
    kt = main_res["kernels"]["trailer"]
    dom = kv if kv["avg_s"] >= kt["avg_s"] else kt
    traffic = load_traffic(dom["name"], args.config)
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
                   "checksum": {1: "kCRC32c", 4: "kXXH3"}[main_res["ctype"]],
                   "step": "trailer pass (write side) + verify pass (read side)",
                   "parallelism": f"block shard per GPU x{world}, no collective"},
        "roofline": {"bound": "hbm", "kernel": dom["name"],
                     "achieved": round(dom["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(dom["frac"], 4), "traffic": traffic},
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
