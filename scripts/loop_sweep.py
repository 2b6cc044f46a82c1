#!/usr/bin/env python3
"""Config-5 loop geometry sweep on one GPU: python scripts/loop_sweep.py [total [chunk chunks P C D dma slot]]
One line per (chunk, chunks, producers, consumers): Mpkt/s and each stage's busy fraction."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scion-xdp-br_amd"))
import scion_hfv as hfv  # noqa: E402
from scion_hfv import evaluation as E  # noqa: E402


def main():
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 23
    ctx = hfv.Ctx(0)
    E.setup_ctx(ctx)
    frames = E.frames(1000)
    lens = np.full(1000, E.FRAME_LEN, dtype=np.uint16)
    # dma: 0 zero-copy, 1 DMA both ways, 2 DMA in + the kernel writing its changes into the ring
    one = [tuple(int(x) for x in sys.argv[2:9])] if len(sys.argv) >= 9 else None   # chunk chunks P C D dma slot
    for chunk, chunks, p, c, d, dma, slot in one or [
            (1 << 16, 12, 4, 2, 4, 0, 144), (1 << 16, 12, 4, 2, 3, 1, 144),
            (1 << 16, 12, 4, 2, 2, 2, 144), (1 << 16, 12, 4, 2, 3, 2, 144), (1 << 16, 12, 4, 2, 4, 2, 144),
            (1 << 16, 12, 6, 3, 3, 2, 144), (1 << 16, 12, 8, 4, 4, 2, 144), (1 << 17, 8, 8, 4, 3, 2, 144),
            (1 << 15, 16, 8, 4, 6, 2, 144), (1 << 16, 12, 8, 4, 4, 2, 192)]:
        r = ctx.loop_run(frames, lens, total, rx_ifindex=E.RX_IFINDEX, slot=slot, chunk=chunk, chunks=chunks,
                         producers=p, consumers=c, inflight=d, dma=dma)
        s = r["seconds"]
        print(f"{('zc  ', 'dma ', 'dma2')[dma]} slot {slot} chunk {chunk:7d} x{chunks:2d} P{p:2d} C{c:2d} D{d}  {total / s / 1e6:7.1f} Mpkt/s  router {r['gpu_busy_s'] / s:.2f} "
              f"wait_rx {r['gpu_wait_s'] / s:.2f} prod {r['producer_busy_s'] / p / s:.2f} cons {r['consumer_busy_s'] / c / s:.2f}"
              f"  router_us_per_chunk {r['gpu_busy_s'] / (total / chunk) * 1e6:8.1f}", flush=True)


if __name__ == "__main__":
    main()
