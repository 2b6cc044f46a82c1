#!/usr/bin/env python3
"""Sustained service grids: `reps` grids of K = 200 batches of 2^20 resident records (8 rotated),
event-timed, with each grid's shader clock -- the rate the power limit allows under continuous
verify (bench.py's `sustained` leg, repeated).  HFV_LIB picks the library build, so that
scripts/ab_sustained.sh can interleave builds.  python scripts/svc_sustained.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scion-xdp-br_amd"), ROOT]
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.cuda.set_device(0)
    ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
    n, R, K = 1 << 20, 8, bench.SUSTAINED_STEPS
    recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(R)]
    for i, r in enumerate(recs):
        ctx.gen_records(r, n, bench.SEED_RECORDS, first_index=i * n)
    bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    truth = [torch.from_numpy(bench.truth_bitmap(n, i * n)).cuda() for i in range(R)]
    posts = ctx.service_batches([(recs[j % R], n, bits[j]) for j in range(K)])
    torch.cuda.synchronize()
    ctx.service_set_timing(True)
    ctx.service_run(posts)
    out = []
    for _ in range(reps):
        _, ms = ctx.service_run(posts)
        out.append((ms, ctx.service_shader_mhz()))
    torch.cuda.synchronize()
    for j in range(K):
        assert torch.equal(bits[j], truth[j % R]), f"bitmap {j}"
    lib = os.path.basename(os.environ.get("HFV_LIB", "default"))
    print(lib, " ".join(f"{ms:.4f}ms/{mhz:.0f}MHz/{bench.BYTES_PER_PACKET * n * K / (ms * 1e-3) / 1e9 / 8000:.3f}"
                        for ms, mhz in out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
