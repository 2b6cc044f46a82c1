#!/usr/bin/env python3
"""Per-record cost of the resident service against batch size at a fixed total: the same
8 x 2^20 resident records (rotated, HBM) verified as 20 x 2^20, 10 x 2^21 and 5 x 2^22
batches per grid (hfv_service_run), interleaved; prints grid time, ns per 2^20 records and
the shader clock.  Shows what a batch boundary costs the grid.  python scripts/svc_batch_size.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    torch.cuda.set_device(0)
    ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
    n = 1 << 20
    buf = torch.empty((8 * n, 64), dtype=torch.uint8, device="cuda")
    ctx.gen_records(buf, 8 * n, bench.SEED_RECORDS)
    bits = torch.zeros((20 * n) // 64, dtype=torch.int64, device="cuda")
    shapes = {}
    for per in (1, 2, 4):
        k = 20 // per
        posts = []
        for j in range(k):
            first = (j * per) % 8
            posts.append((buf[first * n:], per * n, bits[j * per * n // 64:]))
        shapes[per] = ctx.service_batches(posts)
    torch.cuda.synchronize()
    for per, p in shapes.items():
        ctx.service_run(p)
    for rep in range(4):
        for per, p in shapes.items():
            _, ms = ctx.service_run(p)
            print(f"rep {rep} batches {20 // per:2d} x 2^{20 + per.bit_length() - 1}: grid {ms * 1e3:7.1f} us, "
                  f"{ms * 1e3 / 20:6.2f} us per 2^20 records, {ctx.service_shader_mhz():.0f} MHz", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
