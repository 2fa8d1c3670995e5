import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np, torch
import test_wal_golden as T
from forst_amd import engine, _lib
if len(sys.argv) > 1: _lib.use_library(sys.argv[1])
engine.init_device()
cases = T.load(); logs = T.build_logs()
for c in cases:
    key = (c["family"], c["name"], c["recyclable"])
    if key not in (("scenarios", "clean", False), ("scenarios", "clean", True)): continue
    log = np.ascontiguousarray(logs[key]); dev = torch.from_numpy(log).cuda()
    wr, wp = T.want(c, 0)
    rec, rep, res = engine.wal_recover_batch(dev, c["log_number"], 0, record_capacity=len(wr) + 8, report_capacity=len(wp) + 8)
    got = list(zip(rec["offset"].cpu().tolist(), rec["length"].cpu().tolist(), [h & (2**64 - 1) for h in rec["hash"].cpu().tolist()]))
    print(key, 'n', len(got), len(wr), 'reports', rep["bytes"].numel(), len(wp))
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, wr)) if g != w]
    print(' mismatches', len(bad))
    for b in bad[:8]: print('  ', b)
    # a14 path on the same log
    offs = torch.tensor([o for o, n, h in wr], dtype=torch.int64).cuda()
