"""debug: the fused kernel's short-record CRC values (dbgshort build) against a
host computation (linear CRC32C of the payload moved to the window end, and
E = the header state moved over 1024 bytes)"""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), 'tests'))
import numpy as np, torch
import test_wal_golden as T
from forst_amd import engine, _lib
_lib.use_library(sys.argv[1])
engine.init_device()
POLY = 0x82F63B78
TAB = []
for i in range(256):
    c = i
    for _ in range(8):
        c = (c >> 1) ^ (POLY if c & 1 else 0)
    TAB.append(c)
def upd(v, data):
    for b in data:
        v = (v >> 8) ^ TAB[(v ^ b) & 0xff]
    return v
cases = T.load(); logs = T.build_logs()
for c in cases:
    key = (c["family"], c["name"], c["recyclable"])
    if key != ("scenarios", "clean", False): continue
    log = np.ascontiguousarray(logs[key]); dev = torch.from_numpy(log).cuda()
    wr, wp = T.want(c, 0)
    rec, rep, res = engine.wal_recover_batch(dev, c["log_number"], 0, record_capacity=len(wr) + 8, report_capacity=len(wp) + 8)
    got = list(zip(rec["offset"].cpu().tolist(), rec["length"].cpu().tolist(), [h & (2**64 - 1) for h in rec["hash"].cpu().tolist()]))
    print('n', len(got), len(wr))
    hs = 7
    k = 0
    for (o, n, h) in got:
        if n > 240 or n == 0: continue
        p0 = o + hs
        payload = bytes(log[p0:p0 + n])
        raw = upd(0, payload + bytes(1024 - n))
        H = upd(0xffffffff, bytes(log[o + 6:o + 7]))
        E = upd(H, bytes(1024))
        gv, gz = h >> 32, h & 0xffffffff
        m = int.from_bytes(bytes(log[o:o + 4]), 'little')
        rot = (m - 0xa282ead8) & 0xffffffff
        stored = ((rot >> 17) | (rot << 15)) & 0xffffffff
        Z = upd((~stored) & 0xffffffff, bytes(1024 - n))
        print(o, n, 'V', hex(gv), 'Z', hex(gz), 'want', hex(Z), 'ok' if (gv == gz == Z) else 'BAD')
        k += 1
        if k > 12: break
