#!/usr/bin/env python3
"""Where a hfv_verify_batches launch's time goes (diagnostic, not used by tests or the bench):
K batches of 2^20 rotated resident records in one call, timed with the dispatch events, and
every block's s_memrealtime at its entry and when its last wave left.  Prints per
launch: kernel ms, block 0's shader clock, the entry spread, the finish spread and the
per-XCD (block % 8) mean finish.
    python scripts/batches_span.py [K] [reps]"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n, R = 1 << 20, 8
    ctx = hfv.Ctx(0)
    ctx.key_add(0, bench.KEY_1111)
    recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(R)]
    for i in range(R):
        ctx.gen_records(recs[i], n, bench.SEED_RECORDS, first_index=i * n)
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    blist = ctx.service_batches([(recs[k % R], n, bits[k]) for k in range(K)])
    grid = min(256, K * n // 64)
    ctx.verify_batches_timed(blist)
    for _ in range(reps):
        ms = ctx.verify_batches_timed(blist)
        mhz = ctx.batches_shader_mhz()
        span = ctx.batches_block_span(grid)
        st = [a for a, _ in span]
        fin = [b for _, b in span]
        xcd = [statistics.mean(fin[x::8]) for x in range(8)]
        print(f"kernel {ms * 1e3:7.1f} us  mhz {mhz:6.0f}  entry spread {max(st) - min(st):5.1f} us  "
              f"finish min/med/max {min(fin):6.1f} {statistics.median(fin):6.1f} {max(fin):6.1f} us  "
              f"per-XCD mean finish {' '.join(f'{x:6.1f}' for x in xcd)}", flush=True)
    torch.cuda.synchronize()
    for k in range(K):
        assert torch.equal(bits[k], torch.from_numpy(bench.truth_bitmap(n, (k % R) * n)).cuda())
    ctx.close()


if __name__ == "__main__":
    main()
