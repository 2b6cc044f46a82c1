#!/usr/bin/env python3
"""Config-4 traffic floor at the memory system's granularity, over bench.py's frame mix:
reads in whole 128-byte L2 lines (gfx950) up to the last header byte the router reads, writes
in 32-byte sectors holding a changed byte (from the oracle router's output), plus the 12 B of
per-frame metadata.  Compare with bench.py's algorithmic bytes (exact bytes) and with PMC
traffic (profiles/traffic.json br:1048576).  CPU only: python scripts/br_traffic_floor.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scion-xdp-br_amd"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402
import orc  # noqa: E402  (test infrastructure: the oracle router gives the changed bytes)
from scion_hfv import topology as TP  # noqa: E402


def main():
    frames, ifis, good, abytes = bench.br_templates()
    n = len(frames)
    slots = np.zeros((n, 2048), dtype=np.uint8)
    for i, f in enumerate(frames):
        slots[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
    before = slots.copy()
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    orc.br_process(slots, lens, np.array(ifis, dtype=np.uint32), TP.br_config("br1"), orc.hop_key(TP.KEYS[1]))
    rows = []
    for i in range(n):
        changed = np.nonzero(slots[i] != before[i])[0]
        sectors = len(set((changed // 32).tolist()))
        hdr = abytes[i] - 12 - 35 - 2   # header bytes read (bench.py: hf_end + rewritten + metadata)
        read_lines = -(-max(hdr, 128) // 128) * 128   # the staged 128-byte window at least
        rows.append((abytes[i], read_lines + 32 * sectors + 12, read_lines, 32 * sectors))
    # bench.br_batch draws template ids uniformly over the flows (half good, half corrupted MACs
    # at 1/16) -- weight every template pair equally, as the batch does
    a = np.array(rows, dtype=float)
    good = np.array(good)
    w = np.where(good, 15 / 16, 1 / 16)
    w = w / w.sum()
    alg, floor, rd, wr = (float((a[:, j] * w).sum()) for j in range(4))
    t = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["br:1048576"]
    pmc = t["hbm_bytes_per_launch"] / 2**20
    print(json.dumps({"algorithmic_bytes_per_frame": round(alg, 1), "granularity_floor_bytes_per_frame": round(floor, 1),
                      "floor_read": round(rd, 1), "floor_write_sectors": round(wr, 1),
                      "pmc_bytes_per_frame": round(pmc, 1), "pmc_over_algorithmic": round(pmc / alg, 3),
                      "pmc_over_floor": round(pmc / floor, 3)}))


if __name__ == "__main__":
    main()
