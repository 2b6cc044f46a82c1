"""Host-side cost of a resident-service run as bench.py times it: start call, posting the
batches, stop (waits for the grid), device sync, against the grid's own lifetime
(dispatch events).  Usage: python scripts/svc_overhead.py  (1 GPU)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scion-xdp-br_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import scion_hfv as hfv
import bench
n = 1 << 20
ctx = bench.make_ctx(0, hfv.KEYSEL_ZERO)
stream = torch.cuda.current_stream().cuda_stream
recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
ctx.gen_records(recs, n, bench.SEED_RECORDS, first_index=0, stream=stream)
bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
for _ in range(20): ctx.verify_records(recs, n, bits, stream=stream)
torch.cuda.synchronize()
for _ in range(200): ctx.verify_records(recs, n, bits, stream=stream)
torch.cuda.synchronize()
bits.zero_(); torch.cuda.synchronize()
for _ in range(20): ctx.service_submit(recs, n, bits)
ctx.service_stop()
for rep in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter(); ctx.service_start(); t1 = time.perf_counter()
    for _ in range(200): ctx.service_submit(recs, n, bits)
    t2 = time.perf_counter(); g = ctx.service_stop(); t3 = time.perf_counter()
    torch.cuda.synchronize(); t4 = time.perf_counter()
    print("rep %d: start %.1f submits %.1f stop %.1f sync %.1f total %.1f us; grid %.1f us; wall-grid %.1f" % (rep, (t1-t0)*1e6, (t2-t1)*1e6, (t3-t2)*1e6, (t4-t3)*1e6, (t4-t0)*1e6, g*1e3, (t4-t0)*1e6 - g*1e3), flush=True)
