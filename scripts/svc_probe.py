#!/usr/bin/env python3
"""Timeline of the resident verify service: host post and completion times per batch, and
block 0's descriptor-load stamps (hfv_debug_service_clocks, s_memrealtime at 100 MHz)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import scion_hfv as hfv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
ctx = hfv.Ctx(0)
ctx.key_add(0, b"1111111111111111")
recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
ctx.gen_records(recs, n, 0x5C100001)
bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
L = hfv.lib()
L.hfv_debug_service_clocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for rep in range(3):
    ctx.service_start()
    t0 = time.perf_counter()
    tickets, posts = [], []
    for _ in range(K):
        tickets.append(ctx.service_submit(recs, n, bits))
        posts.append(time.perf_counter() - t0)
    done = []
    for t in tickets:
        ctx.service_wait(t, 20000)
        done.append(time.perf_counter() - t0)
    clk = np.zeros(hfv.SVC_RING + 4, dtype=np.uint64)
    L.hfv_debug_service_clocks(ctx._h, clk.ctypes.data)
    grid = ctx.service_stop()
    L.hfv_debug_service_clocks(ctx._h, clk.ctypes.data)   # exit stamps are written at stop
    rc = [int(x) for x in clk[hfv.SVC_RING:hfv.SVC_RING + 4]]
    shader_mhz = (rc[2] - rc[0]) / ((rc[3] - rc[1]) / 100.0) if rc[3] > rc[1] else None
    done_us = np.array(done) * 1e6
    gaps = np.diff(done_us)
    ld = (clk[:K].astype(np.int64) - int(clk[0])) / 100.0
    print(json.dumps({"n": n, "K": K, "grid_ms": round(grid, 4), "shader_mhz": round(shader_mhz, 1) if shader_mhz else None, "host_done_ms": round(done[-1] * 1e3, 3),
                      "post_loop_ms": round(posts[-1] * 1e3, 3), "post_us_mean": round(posts[-1] / K * 1e6, 2),
                      "done_gap_us_median": round(float(np.median(gaps)), 2),
                      "done_gap_us_p10_p90": [round(float(np.percentile(gaps, 10)), 2),
                                              round(float(np.percentile(gaps, 90)), 2)],
                      "first_done_us": round(float(done_us[0]), 2),
                      "load_us_head": [round(float(x), 1) for x in ld[:8]],
                      "done_us_head": [round(float(x), 1) for x in done_us[:8]]}), flush=True)
ctx.close()
