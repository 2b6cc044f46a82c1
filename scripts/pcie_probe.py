#!/usr/bin/env python3
"""Host<->device bandwidth of this box (the config-5 ceiling): pinned H2D, D2H and both at once
on two streams, hipMemcpyAsync through torch; plus the NUMA node of the GPU."""
import time

import torch


def bw(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    n = 256 << 20
    h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    h2d = bw(lambda: d1.copy_(h1, non_blocking=True), n)
    d2h = bw(lambda: h2.copy_(d2, non_blocking=True), n)

    def both():
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    bi = bw(both, 2 * n)
    print(f"pinned H2D {h2d:.1f} GB/s  D2H {d2h:.1f} GB/s  both directions at once {bi:.1f} GB/s total", flush=True)
    for sz in (1 << 20, 4 << 20, 16 << 20):
        a = bw(lambda: d1[:sz].copy_(h1[:sz], non_blocking=True), sz, 50)
        b = bw(lambda: h2[:sz].copy_(d2[:sz], non_blocking=True), sz, 50)
        print(f"  {sz >> 20:3d} MiB copies: H2D {a:.1f} GB/s D2H {b:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
