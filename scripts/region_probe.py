"""Where a bench.py service region's time goes (ms_per_step runs 10-15 % above the
grid): per region, the host call, the region (device synchronize on both sides, as bench.py's
W.timed), and block 0's in-kernel loop span (s_memrealtime, hfv_debug_service_clocks) -- with
and without the dispatch timing events; plus the same region shape around one empty launch.
Usage: python scripts/region_probe.py [reps] [K]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
torch.cuda.set_device(0)
ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1))
n = 1 << 20
ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
bufs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
for i, b in enumerate(bufs):
    ctx.gen_records(b, n, bench.SEED_RECORDS, first_index=i * n)
bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
posts = ctx.service_batches([(bufs[k % 8], n, bits[k]) for k in range(K)])
run = ctx.service_run_async_fn(posts)
L = hfv.lib()
L.hfv_debug_service_clocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
clk = (ctypes.c_uint64 * (2 * hfv.SVC_RING + 4))()
x = torch.zeros(1, device="cuda")


def region(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) * 1e6, (t2 - t0) * 1e6


for timing in (False, True):
    ctx.service_set_timing(timing)
    rows = []
    for rep in range(REPS + 1):
        call, reg = region(run)
        grid = ctx.service_stop() * 1e3
        L.hfv_debug_service_clocks(ctx._h, clk)
        t0, r0, t1, r1 = (int(v) for v in clk[hfv.SVC_RING:hfv.SVC_RING + 4])
        span = (r1 - r0) / 100.0
        mhz = (t1 - t0) / ((r1 - r0) / 100.0) if r1 > r0 else 0
        if rep:
            rows.append((call, reg, grid, span, mhz))
    a = np.array(rows)
    med = np.median(a, axis=0)
    print(f"K={K} events={int(timing)}: call {med[0]:6.1f} us  region {med[1]:7.1f} us  grid(events) {med[2]:7.1f} us  "
          f"block0 loop span {med[3]:7.1f} us  region-span {med[1] - med[3]:6.1f} us  mhz {med[4]:6.0f}   "
          f"regions {[round(r, 1) for r in a[:, 1]]}", flush=True)
rows = [region(lambda: x.add_(1)) for _ in range(REPS + 1)][1:]
print(f"one-element torch op: call {np.median([r[0] for r in rows]):.1f} us region {np.median([r[1] for r in rows]):.1f} us")
ctx.close()
