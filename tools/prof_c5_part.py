#!/usr/bin/env python3
"""tools/prof_c5_part.py <part> -- ONE call site of the C5 WAL configuration
(bench.run_wal's log: 10 M records, 44 GiB), 2 untimed + 5 timed calls, for
rocprofv3 passes that summarise that call site alone (profiles/profile.sh
C5A14 / C5REC / C5VER / C5WRI): the same kernel (e.g. xxh3_frag_kernel<3>)
serves a14 and the recovery's remainder with launches of very different
sizes, which one summary over tools/prof_wal.py averages together.
  a14      forst_wal_record_xxh3_batch (log_reader.cc:95-165 record checksum)
  recover  forst_wal_recover_batch, kPointInTimeRecovery
  verify   forst_wal_verify_batch (log_reader.cc:450-531)
  writer   forst_wal_record_crc_lengths (log_writer.cc:228-263)
Prints one JSON line (median ms)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forst_amd import engine, workload  # noqa: E402

part = sys.argv[1] if len(sys.argv) > 1 else "a14"
engine.init_device()
w = workload.make_wal_batch(10_000_000, workload.SEEDS["C5"])
offs = torch.from_numpy(w.rec_offsets.view(np.int64)).cuda()
lens = torch.from_numpy(w.rec_lengths.astype(np.int32)).cuda()
crc = torch.empty(len(w.rec_offsets), dtype=torch.uint32, device="cuda")
if part == "a14":
    def fn():
        engine.wal_record_xxh3_batch(w.log, offs)
elif part == "recover":
    def fn():
        engine.wal_recover_batch(w.log, 0, engine.kPointInTimeRecovery,
                                 record_capacity=w.n_records + 1024)
elif part == "verify":
    def fn():
        engine.wal_verify_batch(w.log)
else:
    def fn():
        engine.wal_record_crc_batch(w.log, offs, write_in_place=True, out=crc,
                                    payload_lengths=lens)
for _ in range(2):
    fn()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(json.dumps({"part": part, "ms": round(float(np.median(ts)) * 1e3, 3),
                  "log_bytes": w.total, "records": w.n_records}), flush=True)
