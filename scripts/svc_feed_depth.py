#!/usr/bin/env python3
"""The documented feeder loop (hfv_service_submit per batch, hfv_service_wait on
the ticket DEPTH back; in C through hfv_debug_feed_loop) on a warmed resident grid, for several
depths and run lengths, interleaved: microseconds per 2^20-record batch and the fraction of
8 TB/s, every bitmap checked against the generator truth.
    python scripts/svc_feed_depth.py [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    torch.cuda.set_device(0)
    ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
    n, R = 1 << 20, 8
    recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(R)]
    for i, r in enumerate(recs):
        ctx.gen_records(r, n, bench.SEED_RECORDS, first_index=i * n)
    truth = [torch.from_numpy(bench.truth_bitmap(n, i * n)).cuda() for i in range(R)]
    Ks = (20, 100)
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(max(Ks))]
    warm = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
    posts = {k: ctx.service_batches([(recs[j % R], n, bits[j]) for j in range(k)]) for k in Ks}
    for rep in range(rounds):
        for k in Ks:
            for depth in (1, 2, 4, 8, 16):
                for b in bits:
                    b.zero_()
                torch.cuda.synchronize()
                ctx.service_start()
                ctx.feed_loop(ctx.service_batches([(recs[0], n, warm)]), depth=1)
                el = ctx.feed_loop(posts[k], depth=depth)
                ctx.service_stop()
                torch.cuda.synchronize()
                for j in range(k):
                    assert torch.equal(bits[j], truth[j % R]), f"bitmap {j}"
                us = el / k * 1e6
                print(f"rep {rep} K={k:3d} depth={depth:2d}: {us:6.2f} us per batch "
                      f"({bench.BYTES_PER_PACKET * n / (us * 1e-6) / 1e9 / bench.HBM_PEAK_GBS:.3f} of 8 TB/s)",
                      flush=True)
                time.sleep(0.2)   # idle between runs: each starts near the burst clock
    ctx.close()


if __name__ == "__main__":
    main()
