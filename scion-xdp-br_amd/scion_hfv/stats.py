"""Verdict counters of hfv_br_process and the `watch` view of br-loader
(br/src/stats.cpp:38-144): per-verdict packets and bytes with per-second rates.

The counters are the `stats` buffer of hfv_br_process: u64 [64 ifindex][bytes, packets][11]
in the order of `enum counter` (br/src/bpf/common.h:40-53), i.e. port_stats_map summed over
CPUs.
"""
import sys
import time

import numpy as np

COUNTER_NAMES = ("Undefined", "Forwarded", "Parse error", "Not SCION", "Not implemented", "No interface",
                 "Underlay mismatch", "Router alert", "FIB lookup drop", "FIB lookup pass", "Invalid HF")
N_COUNTERS = len(COUNTER_NAMES)
STATS_IFINDEX = 64


def as_array(stats):
    """Any buffer of 64*2*11 u64 (numpy, bytes, torch CPU tensor) -> uint64 [64, 2, 11] view."""
    a = np.asarray(stats.numpy() if hasattr(stats, "numpy") else stats)
    return a.view(np.uint64).reshape(STATS_IFINDEX, 2, N_COUNTERS)


def port_totals(stats, ifindex):
    """(bytes[11], packets[11]) of one ingress port (getStats, stats.cpp:58-78)."""
    a = as_array(stats)
    return a[ifindex, 0].copy(), a[ifindex, 1].copy()


def rates(cur, prev, dt_s):
    """calcRates (stats.cpp:44-56): per-second byte and packet rates between two snapshots."""
    (b1, p1), (b0, p0) = cur, prev
    return (b1 - b0).astype(np.float64) / dt_s, (p1 - p0).astype(np.float64) / dt_s


def format_stats(totals, rate=None):
    """printStats (stats.cpp:80-112): the table br-loader's `watch` prints each second."""
    b, p = totals
    rb, rp = rate if rate is not None else (np.zeros(N_COUNTERS), np.zeros(N_COUNTERS))
    lines = ["Verdict             Packets    pkts/s         Bytes    Mbit/s"]
    for i, name in enumerate(COUNTER_NAMES):
        lines.append("%-18s%8d%11.0f%14d%10s" % (name, int(p[i]), rp[i], int(b[i]), "%.5g" % (rb[i] * 8e-6)))
    return "\n".join(lines) + "\n"


def watch(read_stats, ifindex, interval=1.0, iterations=None, out=sys.stdout):
    """watchStats (stats.cpp:116-144): print the counters of `ifindex` every `interval`
    seconds.  read_stats() returns the current counter buffer (e.g. a D2H copy of the
    hfv_br_process stats)."""
    t0 = time.monotonic()
    cur = port_totals(read_stats(), ifindex)
    out.write(format_stats(cur))
    k = 0
    while iterations is None or k < iterations:
        time.sleep(interval)
        t1 = time.monotonic()
        prev, cur = cur, port_totals(read_stats(), ifindex)
        out.write(format_stats(cur, rates(cur, prev, t1 - t0)))
        t0 = t1
        k += 1
