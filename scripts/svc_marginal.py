#!/usr/bin/env python3
"""Fixed and per-batch cost of a resident-service grid: grids of K = 10, 20, 40, 80 batches of
2^20 records (8 resident batches rotated, as in bench.py's headline) timed by their dispatch
events, interleaved; a least-squares line grid(K) = fixed + K * per_batch over each round's
four grids separates the grid's start/fill and drain tail (fixed) from the steady state
(per_batch), with each grid's shader clock.  python scripts/svc_marginal.py [rounds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    torch.cuda.set_device(0)
    ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
    n, R = 1 << 20, 8
    recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(R)]
    for i, r in enumerate(recs):
        ctx.gen_records(r, n, bench.SEED_RECORDS, first_index=i * n)
    Ks = (10, 20, 40, 80)
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(max(Ks))]
    posts = {k: ctx.service_batches([(recs[j % R], n, bits[j]) for j in range(k)]) for k in Ks}
    truth = [torch.from_numpy(bench.truth_bitmap(n, i * n)).cuda() for i in range(R)]
    torch.cuda.synchronize()
    ctx.service_set_timing(True)
    for k in Ks:
        ctx.service_run(posts[k])
    fixed, per = [], []
    for rep in range(rounds):
        row = []
        for k in Ks:
            _, ms = ctx.service_run(posts[k])
            row.append((k, ms * 1e3, ctx.service_shader_mhz()))
        torch.cuda.synchronize()
        for j in range(max(Ks)):
            assert torch.equal(bits[j], truth[j % R]), f"bitmap {j}"
        a, b = np.polyfit([r[0] for r in row], [r[1] for r in row], 1)
        per.append(a)
        fixed.append(b)
        print(f"rep {rep}: " + "  ".join(f"K={k}: {us:7.1f} us {mhz:4.0f} MHz" for k, us, mhz in row) +
              f"  | fit: {b:5.1f} us fixed + {a:6.2f} us per batch", flush=True)
    print(f"median: fixed {np.median(fixed):.1f} us, per batch {np.median(per):.2f} us "
          f"({bench.BYTES_PER_PACKET * n / (np.median(per) * 1e-6) / 1e9 / bench.HBM_PEAK_GBS:.3f} of 8 TB/s)")
    ctx.close()


if __name__ == "__main__":
    main()
