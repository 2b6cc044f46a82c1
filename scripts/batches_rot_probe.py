#!/usr/bin/env python3
"""Is the batch-list kernel bound by HBM or by the CU at the clocks it runs at?  K = 20 batches
of 2^20 records in one hfv_verify_batches call over R resident buffers (batch k reads buffer
k % R): R = 8 (512 MiB, the bench's rotation: every batch from HBM) against R = 1 and 2 (64 and
128 MiB: resident in the 256 MiB Infinity Cache after the first pass), interleaved; per call the
kernel time and block 0's shader clock; with a settle time (s) the GPU idles before every call,
so each runs at the burst clock.  (diagnostic; python scripts/batches_rot_probe.py [reps] [settle])"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    settle = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    n, K = 1 << 20, 20
    ctx = hfv.Ctx(0)
    ctx.key_add(0, bench.KEY_1111)
    recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(8)]
    for i in range(8):
        ctx.gen_records(recs[i], n, bench.SEED_RECORDS, first_index=i * n)
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    lists = {R: ctx.service_batches([(recs[k % R], n, bits[k]) for k in range(K)]) for R in (8, 2, 1)}
    res = {R: [] for R in lists}
    for _ in range(2):
        for R, bl in lists.items():
            ctx.verify_batches_timed(bl)
    for _ in range(reps):
        for R, bl in lists.items():
            if settle:
                torch.cuda.synchronize()
                time.sleep(settle)
            ms = ctx.verify_batches_timed(bl)
            res[R].append((ms, ctx.batches_shader_mhz()))
    torch.cuda.synchronize()
    for k in range(K):   # the last call was R = 1: every bitmap is buffer 0's truth
        assert torch.equal(bits[k], torch.from_numpy(bench.truth_bitmap(n, 0)).cuda())
    for R, v in res.items():
        ms = [x for x, _ in v]
        mhz = [m for _, m in v if m]
        us = statistics.median(ms) * 1e3 / K
        print(f"R={R}  kernel median {statistics.median(ms) * 1e3:7.1f} us  ({us:6.2f} us per batch, "
              f"{64.125 * n / us / 1e6:6.2f} TB/s)  min {min(ms) * 1e3:7.1f}  shader MHz median "
              f"{statistics.median(mhz) if mhz else 0:6.0f}  cycles per tile per CU "
              f"{us * 1e-6 * statistics.median(mhz) * 1e6 / (n / 64 / 256) if mhz else 0:6.1f}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
