#!/usr/bin/env python3
"""Headline benchmark: Mpkt/s of device-resident hop-field AES-CMAC verify on 64 B SCION
records (BASELINE.json metric; config 2 = 2^20 records, single AS key, per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keysel zero|ifid] [--n N] [--rotate R]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One process per GPU.  `--gpus N` with N > 1 and no torch.distributed environment starts the
N rank processes itself (torch.distributed.run as a CHILD process, before this process
touches a GPU) and exits with their status.  A "step" is one batch of the rank's n records
(weak scaling: every rank verifies its own records, no collective on the data path; the
collective backend carries only the timing barrier, max-over-ranks and the per-rank
report).  The rank's records sit in R distinct resident batches (default R = 8: 8 x 64 MiB =
512 MiB, twice the 256 MiB Infinity Cache) and step k verifies batch k % R, so every step
reads its records from HBM, not from the memory-side cache; every step writes its own
verdict bitmap.

By default (--mode batches) the K steps are K batches verified by ONE stream-ordered
hfv_verify_batches call on the rank's stream (one launch per 64 batches: the AES tables are
written into LDS once, the batches' tiles dealt to the CUs as one contiguous range), the launch
and its table fill inside the timed region; --mode service posts the K batches to the resident
service (hfv_service_run_async: a persistent grid fed through a host descriptor ring) and
--mode launch times one hfv_verify_records launch per step (all three are always measured:
`batches`, `service`, `per_launch`).  Rank 0 prints one JSON line.  Besides the contract
fields it carries:
  roofline      -- the headline kernel's algorithmic bytes (64 B read + 1/8 B verdict per
                   record) / its duration from the dispatch's own start/stop events (the
                   launch's, or the service grid's lifetime, over all K batches), against the
                   8 TB/s HBM3E peak and against a streaming read of the same resident batches
                   timed in the same run (`achievable_peak`); `traffic` is the PMC-measured HBM
                   bytes per batch of the same configuration (profiles/traffic.json).
  ceilings      -- LDS lookups and VALU instructions per packet read at run time from the
                   committed PMC summary of this configuration, and the LDS-issue bound at
                   the shader clock the timed kernel ran at (block 0's s_memtime).
  cpu_baseline  -- the reference's own aes.c soft path (oracle/_ref, built from
                   /root/reference) over the same records on this host's cores (median of
                   >= 5 timed passes), verdicts cross-checked against the GPU bitmap; 1-core
                   and AES-NI figures beside it.
  config3       -- the same measurement with 256 ingress-interface keys (KEYSEL_IFID).
  config4       -- the full border-router path (hfv_br_process), see --workload br.
  hbm_resident / mall_resident -- one 2^24-record batch (1 GiB) / one 2^20 batch re-posted
                   (Infinity-Cache resident), for comparison.
  host_e2e      -- rate including H2D/D2H (records in host memory), on every rank, the
                   rank's host threads on its GPU's NUMA node.

    python bench.py --workload br [--n 1048576] [--steps 10]

runs config 4 alone: the full border-router per-packet path (hfv_br_process: parse, AS
ingress/egress, next hop, rewrite, MAC check, counters) as BR 1 of the reference test
topology, over n frames of 64..1500 B in 2 KiB slots (PTF scenario traffic, 1/16 with a
corrupted hop-field MAC).  Frames are rewritten in place, so each timed step gets its own
pristine copy of the batch (K copies resident in HBM, made before the timed region).

    python bench.py --workload br-host [--n 1048576] [--steps 5] [--window 256]

runs config 5's router leg: the same frames start and end in (registered) host memory; per
step one hfv_br_process_host call moves the header windows over PCIe, processes them and
writes the rewritten windows back.

    python bench.py --dry-run --gpus 2

checks the launcher alone: N gloo ranks on the CPU, no GPU work, the line reports n_gpus.
"""
import argparse
import gc
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))

import numpy as np  # noqa: E402

SEED_RECORDS = 0x5C100001
SEED_KEYS = 0x5C100100
KEY_1111 = b"1111111111111111"   # br/test/run_tests:113
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_PACKET = 64 + 1.0 / 8  # algorithmic bytes per verified record
M64 = (1 << 64) - 1
# committed PMC summary of the headline configuration (scripts/pmc_round.sh ... svc rot)
# committed PMC summaries of the headline configurations, by (keysel, path)
PMC_SUMMARY = {("zero", "service"): "profiles/r05/final/pmc_zero_svc/summary.json",
               ("ifid", "service"): "profiles/r05/pmc_ifid_svc/summary.json",
               ("zero", "batches"): "profiles/r06/pmc_zero_bat/summary.json",
               ("ifid", "batches"): "profiles/r06/pmc_ifid_bat/summary.json"}
METRIC = "Mpkt/s device-resident hop-field AES-CMAC verify, 64 B SCION packets"


def splitmix_at(seed, k):
    z = (seed + (k + 1) * 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def key_table_256(seed=SEED_KEYS):
    out = bytearray()
    for k in range(256):
        out += splitmix_at(seed, 2 * k).to_bytes(8, "little") + splitmix_at(seed, 2 * k + 1).to_bytes(8, "little")
    return bytes(out)


def corrupted(n, first_index=0):
    """Generator truth: record i is corrupted iff splitmix draw 4i+2 & 15 == 0."""
    i = np.arange(first_index, first_index + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(SEED_RECORDS) + (np.uint64(4) * i + np.uint64(3)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(15)) == 0


def expected_pass_count(n, first_index):
    return int(n - corrupted(n, first_index).sum())


def popcount(bits_t):
    b = bits_t.cpu().numpy().view(np.uint8)
    return int(np.unpackbits(b).sum())


def truth_bitmap(n, first_index):
    """The exact verdict bitmap of generated records [first_index, first_index + n): record i
    passes iff its MAC was not corrupted, bit i % 64 of word i // 64."""
    ok = ~corrupted(n, first_index)
    padded = np.zeros(((n + 63) // 64) * 64, dtype=bool)
    padded[:n] = ok
    return np.packbits(padded.reshape(-1, 8), axis=1, bitorder="little").reshape(-1).view(np.int64)


# ---- launcher --------------------------------------------------------------------------------

def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """Start args.gpus rank processes (torch.distributed.run, one rank per GPU) as a child
    process and return its exit status.  Nothing in this process has touched a GPU."""
    # torch.distributed.run reads abbreviations of its own options anywhere on the line
    # (`--n` would match --nnodes): pass the record count under its long name
    fwd = [("--records" + a[3:]) if a == "--n" or a.startswith("--n=") else a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + fwd
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


class World:
    """The rank's place in the job and the timing collectives (barrier, max, gather)."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.size = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = args.dry_run
        self.backend = "gloo" if args.dry_run else args.dist_backend
        self.device = self.local if not args.same_device else 0
        # physical GPUs in the job: a --same-device rehearsal puts every rank on GPU 0
        self.n_gpus = 1 if args.same_device else self.size
        if not self.dry:
            torch.cuda.set_device(self.device)
            # host waits on the device spin instead of sleeping (a packet data plane polls; the
            # timed regions' closing synchronize then sees the grid's exit sooner: 76.6 vs 74.9
            # Gpkt/s mean over five interleaved runs, profiles/r02/svc_ab/sync_spin_ab_r02f4.log);
            # HFV_BENCH_SPIN=0 keeps HIP's default
            if os.environ.get("HFV_BENCH_SPIN", "1") != "0":
                import ctypes
                hip = ctypes.CDLL("libamdhip64.so")
                rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))   # hipDeviceScheduleSpin
                if rc != 0:
                    print(f"bench: hipSetDeviceFlags(spin) returned {rc}", file=sys.stderr)
        if self.size > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.device))
            else:
                dist.init_process_group("gloo")
        if self.size != args.gpus and self.rank == 0:
            print(f"bench: --gpus {args.gpus} but the job has {self.size} ranks; reporting {self.size}",
                  file=sys.stderr)

    def sync(self):
        if not self.dry:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.size > 1:
            self.dist.barrier()

    def gather(self, x):
        """Every rank's float x (rank order) on every rank."""
        if self.size == 1:
            return [float(x)]
        dev = "cpu" if self.backend == "gloo" else "cuda"
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=dev)
        out = [self.torch.zeros_like(t) for _ in range(self.size)]
        self.dist.all_gather(out, t)
        return [float(o.item()) for o in out]

    def gather_obj(self, x):
        """Every rank's picklable x (rank order) on every rank."""
        if self.size == 1:
            return [x]
        out = [None] * self.size
        self.dist.all_gather_object(out, x)
        return out

    def timed(self, steps, fn):
        """fn() `steps` times between barrier + device sync on both sides; (max over ranks,
        per-rank list).  Each rank's clock runs from the release of the opening barrier to the
        end of its closing device synchronize; the closing barrier comes after the clock stops
        (with RCCL it is itself a collective launch and synchronize, tens of microseconds that are
        no part of any rank's K steps), and the max over ranks is the job's time."""
        # no garbage-collector pass inside the region (a host pause of its own); no collect()
        # before it either: walking every object leaves the host caches cold, and the region's
        # launch call then took 34-62 us instead of 9-13 (profiles/r03/drv3_gc_collect/)
        gc_on = gc.isenabled()
        gc.disable()
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        self.sync()
        el = time.perf_counter() - t0
        if gc_on:
            gc.enable()
        self.barrier()
        all_el = self.gather(el)
        return max(all_el), all_el

    def close(self):
        if self.size > 1:
            self.dist.destroy_process_group()


# ---- measurement helpers -----------------------------------------------------------------------

def thread_budget(W, ctx):
    """Host threads this rank may use: the CPUs of its GPU's NUMA node (that the process may run
    on) divided among the ranks whose GPU hangs off the same node, capped by OMP_NUM_THREADS (the
    box's per-GPU CPU share).  At N = 8 four ranks share each node of a two-socket host, and
    every rank runs the host legs at once."""
    node = ctx.numa_node()
    cpus = len(ctx.numa_cpus())
    nodes = W.gather(node)
    share = max(1, sum(1 for x in nodes if int(x) == node))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    budget = max(2, cpus // share)
    if omp > 0:
        budget = min(budget, omp)
    return {"budget": budget, "numa_node": node, "node_cpus": cpus, "ranks_on_node": share,
            "omp_num_threads": omp or None}


def apply_thread_budget(args, tb):
    """Size this rank's host pools from its budget: the staging pool of the host path
    (HFV_HOST_THREADS, read when the pool starts) and the config-5 loop's producer / consumer
    threads (the calling thread drives the GPU stage)."""
    b = tb["budget"]
    os.environ.setdefault("HFV_HOST_THREADS", str(max(1, min(8, b))))
    tb["host_threads"] = int(os.environ["HFV_HOST_THREADS"])
    args.loop_threads = max(1, min(args.loop_threads, (b - 1) * 2 // 3))
    args.loop_consumers = max(1, min(args.loop_consumers, b - 1 - args.loop_threads))
    tb["loop_producers"], tb["loop_consumers"] = args.loop_threads, args.loop_consumers
    return tb

def make_ctx(hfv, device, keysel):
    ctx = hfv.Ctx(device)
    if keysel == hfv.KEYSEL_IFID:
        ctx.key_add_batch(0, key_table_256())
    else:
        ctx.key_add(0, KEY_1111)
    ctx.set_keysel(keysel)
    return ctx


def pmc_summary(keysel, path="batches"):
    """The committed PMC summary of the headline configuration for this keysel and path, or None."""
    try:
        return json.load(open(os.path.join(ROOT, PMC_SUMMARY[(keysel, path)])))
    except Exception:
        return None


def pmc_traffic(key):
    """HBM bytes per batch/launch measured by rocprofv3 PMC passes for this exact
    configuration (profiles/traffic.json), or None."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))[key]["hbm_bytes_per_launch"]
    except Exception:
        return None


def settle(args):
    """Idle the GPU before a leg (outside any timed region): the shader clock falls from ~2.0 to
    ~1.5 GHz over a few ms of back-to-back full-chip work (power limit, scripts/svc_batch_size.py)
    and recovers when idle, so each leg starts from the same state instead of inheriting the
    previous leg's heat.  --settle-s 0 turns it off."""
    if args.settle_s > 0:
        time.sleep(args.settle_s)


LOOKUPS_PER_PKT = 145   # T-table lookups per packet (11 + 8 x 16 + 6), each addressed by one v_perm


def ceilings(keysel, n, mhz, cus, path="batches"):
    """Bounds beside HBM, per packet, read from the committed PMC summary of this
    configuration (SQ_INSTS_LDS / SQ_INSTS_VALU are wave-instructions: x 64 lanes / records
    per batch) and the chip's conflict-free ds_read_b32 issue rate (32 lanes per clock per
    CU, MI355X_MICROARCH.md LDS table) at the shader clock the grid ran at."""
    s = pmc_summary(keysel, path)
    out = {"source": PMC_SUMMARY[(keysel, path)] if s else None}
    row = (s or {}).get(str(n))
    if not row:
        return out
    lds = row["SQ_INSTS_LDS"] * 64 / n
    valu = row["SQ_INSTS_VALU"] * 64 / n
    out.update({"lds_instr_per_pkt": round(lds, 1), "valu_instr_per_pkt": round(valu, 1)})
    if mhz:
        out["shader_mhz"] = round(mhz, 1)
        out["lds_issue_bound_mpkts"] = round(cus * 32 * mhz * 1e6 / lds / 1e6, 1)
        # VALU issue: full-rate ops 128 lanes per clock per CU, v_perm (one per table lookup,
        # 145 per packet) half rate (profiles/r01/ubench/valu_rate.log): CU-clocks per packet
        # = (valu + perms) / 128
        out["valu_issue_bound_mpkts"] = round(cus * mhz * 1e6 * 128 / (valu + LOOKUPS_PER_PKT) / 1e6, 1)
    out["hbm_peak_bound_mpkts"] = round(HBM_PEAK_GBS * 1e9 / BYTES_PER_PACKET / 1e6, 1)
    return out


def service_grid(ctx, batches, steps, bitmaps, n, posts=None):
    """One resident-service grid over `steps` batches (batch k % R, bitmap k): hfv_service_run
    posts them and the stop behind them, launches the grid and waits for it; returns the
    grid's lifetime in ms.  posts: the prepared descriptor array (built outside a timed
    region)."""
    if posts is None:
        posts = ctx.service_batches([(batches[k % len(batches)], n, bitmaps[k % len(bitmaps)]) for k in range(steps)])
    return ctx.service_run(posts)[1]


def measure_hf(hfv, W, ctx, keysel_name, n, first, rotate, steps, warmup, stream, bitmap_cap=1024,
               service=True, reps=3):
    """Resident records in `rotate` batches, launch path and service path; returns a dict."""
    torch = W.torch
    R = rotate
    batches = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(R)]
    for i, b in enumerate(batches):
        ctx.gen_records(b, n, SEED_RECORDS, first_index=first + i * n, stream=stream)
    nb = max(R, min(steps, bitmap_cap))
    bitmaps = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(nb)]
    # the exact verdict bitmap of every resident batch (generator truth), on the device
    truth = [torch.from_numpy(truth_bitmap(n, first + i * n)).cuda() for i in range(R)]

    def check(k_steps):
        """Every bitmap the last k_steps steps wrote equals its batch's truth bit for bit (untimed)."""
        torch.cuda.synchronize()
        for k in range(min(k_steps, nb)):
            assert torch.equal(bitmaps[k], truth[k % R]), f"bitmap {k} != the generator truth of batch {k % R}"

    # --- launch path: one hfv_verify_records launch (+ table fill) per batch ---
    for k in range(max(warmup, R)):                 # >= one untimed pass over every batch
        ctx.verify_records(batches[k % R], n, bitmaps[k % nb], stream=stream)
    W.sync()
    check(R)
    step = [0]

    def launch_step():
        k = step[0]
        ctx.verify_records(batches[k % R], n, bitmaps[k % nb], stream=stream)
        step[0] = k + 1

    launch_el, _ = W.timed(steps, launch_step)
    ks = sorted(ctx.verify_records_timed(batches[k % R], n, bitmaps[k % nb], stream=stream)
                for k in range(max(20, min(steps, 200))))
    k_mean, k_med = float(np.mean(ks)), ks[len(ks) // 2]

    out = {"launch_el": launch_el, "k_mean": k_mean, "k_med": k_med, "batches": batches, "bitmaps": bitmaps,
           "svc_el": None, "per_rank_s": None, "grid_ms": None, "mhz": None}

    # --- stream-ordered batch list: the K batches in one hfv_verify_batches call (one launch per
    # 64 batches), table fill and grid ramp paid once; the region's closing synchronize waits ---
    blist = ctx.service_batches([(batches[k % R], n, bitmaps[k % nb]) for k in range(steps)])
    run_b = ctx.verify_batches_fn(blist, stream=stream)
    for b in bitmaps:
        b.zero_()
    run_b()
    W.sync()
    check(steps)
    b_runs = []
    for _ in range(max(1, reps)):
        for b in bitmaps:
            b.zero_()
        W.sync()
        b_runs.append(W.timed(1, run_b))
        check(steps)
    b_runs.sort(key=lambda r: r[0])
    b_ms = []
    for _ in range(max(1, reps)):   # (kernel ms, block 0's shader clock) per event-timed call
        b_ms.append((ctx.verify_batches_timed(blist, stream=stream), ctx.batches_shader_mhz()))
    check(steps)
    b_med = sorted(b_ms)[len(b_ms) // 2]
    # the achievable HBM read rate of these same resident batches in this run: one dense
    # non-temporal streaming read over the K batches (the rotation the steps read), 4 blocks per CU
    sr = sorted(ctx.stream_read_ms([batches[k % R] for k in range(min(steps, 64))], stream=stream)
                for _ in range(max(3, reps)))
    sr_bytes = min(steps, 64) * n * 64
    out["stream_read"] = {"gbs": round(sr_bytes / (sr[len(sr) // 2] * 1e-3) / 1e9, 1),
                          "gbs_best": round(sr_bytes / (sr[0] * 1e-3) / 1e9, 1),
                          "ms_all": [round(x, 4) for x in sr], "bytes": sr_bytes,
                          "kernel": "k_stream_read: 16 B non-temporal loads per lane, 4 x 1024-thread blocks per CU, "
                                    "over the same resident batches (hfv_debug_stream_read)"}
    out.update({"bat_el": b_runs[len(b_runs) // 2][0], "bat_per_rank_s": b_runs[len(b_runs) // 2][1],
                "bat_all_ms": [round(r[0] * 1e3, 4) for r in b_runs], "bat_kernel_ms": b_med[0],
                "bat_mhz": b_med[1], "bat_all_kernel_ms": [round(x[0], 4) for x in b_ms],
                "bat_all_mhz": [round(x[1], 1) if x[1] else None for x in b_ms]})
    if not service:
        out["per_rank_s"] = W.gather(launch_el)
        return out

    # --- resident service: launch, table fill, K batches, drain all inside the timed region ---
    for b in bitmaps:
        b.zero_()
    W.sync()
    # the untimed warm-up grid has the timed grids' shape (K batches), so a kernel trace of the
    # headline command lists only K-batch service grids (their mean is the roofline's grid time)
    service_grid(ctx, batches, max(warmup, R, steps), bitmaps, n)
    check(max(R, steps))
    for b in bitmaps:
        b.zero_()
    W.sync()
    svc = {}
    posts = ctx.service_batches([(batches[k % R], n, bitmaps[k % nb]) for k in range(steps)])
    run_posts = ctx.service_run_async_fn(posts)

    # hfv_service_run_async: the region's closing device synchronize is the only wait (the
    # waiting hfv_service_run, HFV_BENCH_ASYNC=0, spins on the grid's stream first: ~5 % slower,
    # profiles/r02/svc_ab/run_async_ab_r02f2.log)
    run_async = os.environ.get("HFV_BENCH_ASYNC", "1") != "0"

    def service_run():
        t = time.perf_counter()
        if run_async:   # the region's closing device synchronize waits for the grid
            run_posts()
        else:
            svc["grid_ms"] = service_grid(ctx, batches, steps, bitmaps, n, posts)
        svc["call_us"] = (time.perf_counter() - t) * 1e6

    # The K-step timed region is repeated `reps` times (each a fresh grid over the same K
    # batches) and the median region is reported: one timed region of ~0.3 ms is exposed to a
    # single host hiccup (one of three A/B runs measured 0.41 ms for a 0.245 ms grid).
    # `value` comes from regions whose grid carries no dispatch timing events: on MI355X the
    # events add ~12 us to a launch-to-synchronize round trip (24.7 against 12.5 us for the
    # same kernel, scripts/ubench/launch_cost.hip, profiles/r03/launch_cost/), i.e. ~4 % of a
    # K = 20 region.  The grid lifetime the roofline needs is timed with the events in `reps`
    # further regions that are identical otherwise (HFV_BENCH_TIMED_VALUE=1: value from those).
    timed_value = os.environ.get("HFV_BENCH_TIMED_VALUE", "0") != "0"

    def regions(timing):
        ctx.service_set_timing(timing)
        rs = []
        for _ in range(max(1, reps)):
            for b in bitmaps:
                b.zero_()
            W.sync()
            el, per_rank = W.timed(1, service_run)
            if run_async:
                svc["grid_ms"] = ctx.service_stop()   # reaps the exited grid: its lifetime (0 untimed)
            rs.append((el, per_rank, svc["grid_ms"], ctx.service_shader_mhz(), svc["call_us"],
                       ctx.service_weights(), ctx.service_relay()))   # diagnostics
            check(steps)
        return rs

    runs = [] if timed_value else regions(False)
    truns = regions(True)
    ctx.service_set_timing(True)
    if timed_value:
        runs = truns
    runs.sort(key=lambda r: r[0])
    truns_s = sorted(truns, key=lambda r: r[2])
    svc_el, per_rank = runs[len(runs) // 2][:2]
    # the roofline's grid and ITS shader clock (the ceilings are priced at the clock of the grid
    # the roofline times)
    grid_ms, mhz = truns_s[len(truns_s) // 2][2], truns_s[len(truns_s) // 2][3]
    out.update({"svc_el": svc_el, "per_rank_s": per_rank, "grid_ms": grid_ms, "mhz": mhz,
                "svc_all_ms": [round(r[0] * 1e3, 4) for r in runs],
                "svc_all_call_us": [round(r[4], 1) for r in runs],
                "svc_timed_regions_ms": [round(r[0] * 1e3, 4) for r in truns],
                "svc_all_grid_ms": [round(r[2], 4) for r in truns],
                # per event-timed grid: its shader clock and the block weights it left for the
                # next grid (a slow grid at a normal clock with skewed weights is a balance fault)
                "svc_grid_mhz": [round(r[3], 1) if r[3] else None for r in truns],
                "svc_weights": [r[5] for r in truns],
                # per grid (value regions, then event-timed ones): the host link as the relay saw
                # it -- a PCIe round trip probed at grid start, descriptors in the kernel arguments /
                # fetched by the relay, waits of a block for a descriptor (0: no grid ran at the
                # pace of host round trips, the round-3 driver fault)
                "svc_relay": [{"probe_rtt_us": r[6]["probe_rtt_us"], "inline": r[6]["inline"],
                               "relayed": r[6]["relayed"], "block_waits": r[6]["block_waits"]}
                              for r in list(runs if not timed_value else []) + truns if r[6]],
                "svc_value_regions": "timed with dispatch events" if timed_value else "no timing events"})
    return out


SUSTAINED_STEPS = 200   # batches per grid of the sustained leg (~2.3 ms each)
SUSTAINED_GRIDS = 6     # back-to-back grids: the clock the power limit settles at under continuous load
FEED_DEPTH = 8          # batches in flight in INTEGRATION.md section 2's feeder loop (scripts/svc_feed_depth.py)


def service_legs(hfv, W, ctx, m, n, first, rotate, steps):
    """Two more views of the headline's service on the same resident batches (every rank, after
    the headline regions; untimed setup, bitmaps checked bit-exactly against generator truth):
      sustained -- SUSTAINED_GRIDS back-to-back grids of SUSTAINED_STEPS batches each (~15 ms of
                   continuous verify): the clock the chip's power limit settles at under this load
                   (the K = 20 headline grid is a 0.22 ms burst at ~2.0 GHz; the XDP program it
                   replaces runs continuously); the median of the last half of the grids;
      per_call  -- the data-plane binding INTEGRATION.md section 2 documents, run in C through
                   hfv_debug_feed_loop on a resident grid: per RX batch one hfv_service_submit, and
                   hfv_service_wait on the ticket FEED_DEPTH batches back; host clock, steady state
                   (the grid was started and warmed before the clock)."""
    torch = W.torch
    batches, R = m["batches"], rotate
    truth = [torch.from_numpy(truth_bitmap(n, first + i * n)).cuda() for i in range(R)]
    out = {}
    # sustained
    K = SUSTAINED_STEPS
    bms = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(K)]
    posts = ctx.service_batches([(batches[k % R], n, bms[k]) for k in range(K)])
    W.sync()
    W.barrier()
    ctx.service_set_timing(True)
    grids = []
    for _ in range(SUSTAINED_GRIDS):
        _, g_ms = ctx.service_run(posts)
        grids.append((g_ms, ctx.service_shader_mhz() or 0.0))
    W.sync()
    for k in range(K):
        assert torch.equal(bms[k], truth[k % R]), f"sustained: bitmap {k} != generator truth"
    tail = sorted(grids[len(grids) // 2:])
    g_ms, mhz = tail[len(tail) // 2]
    g_all = W.gather(g_ms)
    ach = BYTES_PER_PACKET * n * K / (max(g_all) * 1e-3) / 1e9
    out["sustained"] = {"batches_per_grid": K, "grids": SUSTAINED_GRIDS, "grid_ms": round(g_ms, 4),
                        "mpkts": round(W.size * n * K / max(g_all) / 1e3, 1),
                        "frac": round(ach / HBM_PEAK_GBS / W.size, 4), "shader_mhz": round(mhz, 1) if mhz else None,
                        "all_grids_ms": [round(x[0], 4) for x in grids], "all_grids_mhz": [round(x[1], 1) for x in grids],
                        "per_rank_grid_ms": [round(x, 4) for x in g_all],
                        "note": f"{SUSTAINED_GRIDS} back-to-back service grids of {K} resident batches (k % {R}) each; "
                                f"median of the last {len(tail)}: the clock the power limit holds under continuous "
                                f"verify; frac per GPU"}
    # the same continuous load through the headline path: back-to-back hfv_verify_batches calls of
    # K batches each (one launch per 64 batches), each call timed by its launches' events
    bgrids = []
    for b in bms:
        b.zero_()
    for _ in range(SUSTAINED_GRIDS):
        b_ms = ctx.verify_batches_timed(posts)
        bgrids.append((b_ms, ctx.batches_shader_mhz() or 0.0))
    W.sync()
    for k in range(K):
        assert torch.equal(bms[k], truth[k % R]), f"sustained (batches): bitmap {k} != generator truth"
    btail = sorted(bgrids[len(bgrids) // 2:])
    bg_ms, bmhz = btail[len(btail) // 2]
    bg_all = W.gather(bg_ms)
    bach = BYTES_PER_PACKET * n * K / (max(bg_all) * 1e-3) / 1e9
    out["sustained_batches"] = {"batches_per_call": K, "calls": SUSTAINED_GRIDS, "kernel_ms": round(bg_ms, 4),
                                "launches_per_call": -(-K // 64),
                                "mpkts": round(W.size * n * K / max(bg_all) / 1e3, 1),
                                "frac": round(bach / HBM_PEAK_GBS / W.size, 4),
                                "shader_mhz": round(bmhz, 1) if bmhz else None,
                                "all_calls_ms": [round(x[0], 4) for x in bgrids],
                                "all_calls_mhz": [round(x[1], 1) for x in bgrids],
                                "per_rank_kernel_ms": [round(x, 4) for x in bg_all],
                                "note": f"{SUSTAINED_GRIDS} back-to-back hfv_verify_batches calls of {K} resident batches "
                                        f"each, one host wait between calls; median of the "
                                        f"last {len(btail)}; frac per GPU"}
    del bms
    # per_call: the documented feeder loop on a running grid
    bms = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(steps)]
    warm = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
    posts = ctx.service_batches([(batches[k % R], n, bms[k]) for k in range(steps)])
    W.sync()
    W.barrier()   # before the grid starts: no collective may need the CUs a resident grid holds
    ctx.service_start()
    ctx.feed_loop(ctx.service_batches([(batches[0], n, warm)]), depth=1)   # grid up, tables filled
    el = ctx.feed_loop(posts, depth=FEED_DEPTH)
    ctx.service_stop()
    W.sync()
    for k in range(steps):
        assert torch.equal(bms[k], truth[k % R]), f"per_call: bitmap {k} != generator truth"
    el_all = W.gather(el)
    out["per_call"] = {"mpkts": round(W.size * n * steps / max(el_all) / 1e6, 1),
                       "frac": round(BYTES_PER_PACKET * n * steps / max(el_all) / 1e9 / HBM_PEAK_GBS, 4),
                       "us_per_batch": round(max(el_all) / steps * 1e6, 2), "batches": steps, "depth": FEED_DEPTH,
                       "path": "INTEGRATION.md section 2: hfv_service_submit per batch + hfv_service_wait on the "
                               f"ticket {FEED_DEPTH} back, in C (hfv_debug_feed_loop), on a resident grid; host clock; "
                               "frac per GPU"}
    del bms
    return out


def cpu_baseline(recs_host, keysel, gpu_bits, budget_s):
    """The reference aes.c soft path (XDP's arithmetic) timed on this host's cores over a
    bounded sample of the same records (median of >= 5 timed passes); verdicts must equal
    the GPU's.  Threads: every CPU this process may run on, capped by OMP_NUM_THREADS when
    the environment sets one (the GPU box gives each GPU a share of its CPUs)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc   # test infrastructure: only this leg of the bench may use it

    raw = key_table_256() if keysel else KEY_1111
    hk, valid = orc.key_table(raw)
    raw256 = raw + bytes(16 * (256 - len(raw) // 16))
    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(affinity, omp) if omp > 0 else affinity
    n = len(recs_host)
    use_ref = orc.reference() is not None

    def run(nthreads, aesni=0):
        if use_ref:
            return orc.ref_verify_records(recs_host, raw256, hk, valid, keysel, nthreads=nthreads, aesni=aesni)
        return orc.verify_records(recs_host, hk, valid, keysel, nthreads=nthreads)

    def rate(nthreads, aesni, reps, budget):
        ts, bits = [], None
        t_all = 0.0
        while len(ts) < reps or t_all < budget:
            t0 = time.perf_counter()
            bits = run(nthreads, aesni)
            dt = time.perf_counter() - t0
            ts.append(dt)
            t_all += dt
            if len(ts) >= 50:
                break
        return n / statistics.median(ts) / 1e6, len(ts), bits

    # 1-core figures on a 2^16-record slice (one pass of the soft path over 2^20 takes ~0.25 s)
    m1 = min(n, 1 << 16)
    sub = recs_host[:m1]
    soft1 = [None]

    def run1(aesni):
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            b = orc.ref_verify_records(sub, raw256, hk, valid, keysel, nthreads=1, aesni=aesni) if use_ref else \
                orc.verify_records(sub, hk, valid, keysel, nthreads=1)
            ts.append(time.perf_counter() - t0)
            soft1[0] = b
        return m1 / statistics.median(ts) / 1e6

    one_soft = run1(0)
    one_aesni = run1(1) if use_ref else None
    v, reps, bitsN = rate(threads, 0, 5, budget_s)
    match = bool(np.array_equal(bitsN, gpu_bits))
    out = {"value": round(v, 3), "unit": "Mpkt/s", "cores": threads, "kind": "reference" if use_ref else "port",
           "sample": f"{n} records of the benched batch, median of {reps} timed passes, aes_cmac soft path "
                     f"(aes/src/aes.c, what XDP executes), {threads} threads",
           "nproc": os.cpu_count(), "affinity_cpus": affinity,
           "threads_note": "all CPUs of the process affinity" if not omp or omp >= affinity else
                           f"capped by OMP_NUM_THREADS={omp} (this GPU's share of the host CPUs)",
           "single_core_mpkts": round(one_soft, 3), "verdicts_match_gpu": match}
    if use_ref:
        va, reps_a, bitsA = rate(threads, 1, 5, 0.0)
        assert np.array_equal(bitsA, bitsN)
        out["aesni_mpkts"] = round(va, 3)
        out["aesni_single_core_mpkts"] = round(one_aesni, 3)
    return out


# ---- config 4 / 5: the full router path ---------------------------------------------------------

BR_SLOT = 2048
BR_KINDS = ("down", "up", "core", "seg_switch")


def br_templates():
    """Frames BR 1 of the reference topology receives in the PTF scenarios (as ingress from
    AS interfaces 1/2, and from sibling BR 2 over the internal link), each also with a
    corrupted hop-field MAC.  Returns (frames, ifindex, good, algorithmic bytes) lists."""
    from scion_hfv import packets as P
    from scion_hfv import topology as TP
    frames, ifis, good, abytes = [], [], [], []
    for ki, kind in enumerate(BR_KINDS):
        flows = [((1, 2), None), ((2, 1), None), ((1, 3), None), ((2, 4), None), ((3, 1), 5), ((4, 2), 5)]
        for fi, ((ing, egr), internal) in enumerate(flows):
            path = P.ptf_path(kind, ing, egr, TP.KEYS, seed=0x100 * ki + fi)
            if internal:   # BR 2 did the AS ingress and handed the frame over veth4 -> veth5
                path.ingress(TP.KEYS[1])
                enc, ifi = P.Encap(TP.MAC[4], TP.MAC[5], "10.2.0.0", "10.2.0.1", 31002, 31002), internal
            else:
                enc, _, _, ifi = TP.encaps(ing, egr)
            switch = kind == "seg_switch" and not internal
            for bad in (False, True):
                p = path.copy()
                if bad:
                    h = p.hops[p.curr_hf]
                    h.mac = bytes([h.mac[0] ^ 0x10]) + h.mac[1:]
                f = enc.frame(P.scion_header(p.pack()))
                # header bytes through the last hop field read, + bytes rewritten (Ethernet 12,
                # IPv4 11, UDP 6, PathMeta 4, SegID 2 per info field touched) + 12 B of per-frame
                # metadata (len, ifindex in; action, verdict, egress out)
                hf_end = 78 + 4 + 8 * len(p.infos) + 12 * (p.curr_hf + 1 + switch)
                frames.append(f)
                ifis.append(ifi)
                good.append(not bad)
                abytes.append(hf_end + 35 + 2 * (1 + switch) + 12)
    return frames, ifis, good, abytes


def br_batch(n, rank):
    """Host copy of the config-4 batch: frames [n, 2 KiB], lengths, ingress ifindex, #good."""
    frames, ifis, good, abytes = br_templates()
    nt = len(frames) // 2
    rng = np.random.default_rng(0x5C100004 + rank)
    tid = (np.arange(n) % nt) * 2 + corrupted(n, rank * n)
    hdr = np.array([len(f) for f in frames])
    lens = np.maximum(hdr[tid], rng.integers(64, 1501, n)).astype(np.uint16)
    tmpl = np.zeros((len(frames), BR_SLOT), dtype=np.uint8)
    for i, f in enumerate(frames):
        tmpl[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
    return tmpl, tid, lens, np.array(ifis, dtype=np.uint32)[tid], int(np.array(good)[tid].sum())


def br_cpu_baseline(frames_host, lens, ifidx, cfg, budget_s):
    """The oracle border router (a scalar C restatement of xdp.c; the BPF program itself cannot
    run here) on one host core over a sample of the same frames."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc   # test infrastructure: only the cpu_baseline leg may use it
    from scion_hfv import topology as TP
    hk = orc.hop_key(TP.KEYS[1])
    ts, n = [], len(frames_host)
    a = None
    while len(ts) < 5 or sum(ts) < budget_s:
        work = frames_host.copy()
        t0 = time.perf_counter()
        a, v, e, s = orc.br_process(work, lens, ifidx, cfg, hk)
        ts.append(time.perf_counter() - t0)
        if len(ts) >= 50:
            break
    return a, {"value": round(n / statistics.median(ts) / 1e6, 3), "unit": "Mpkt/s", "cores": 1, "kind": "port",
               "sample": f"{n} frames of the benched mix, median of {len(ts)} passes, oracle/hfv_br_oracle.c "
                         f"(scalar restatement of br/src/bpf/xdp.c process_packet + verify), 1 thread"}


def measure_br(hfv, W, n, steps, warmup, hf_check=True):
    """Config 4 on this rank: K pristine copies of the 2 KiB-slot batch resident in HBM, one
    hfv_br_process launch per step.  Returns (result fields, host frames sample, ...)."""
    from scion_hfv import topology as TP
    torch = W.torch
    ctx = hfv.Ctx(W.device)
    ctx.key_add(0, TP.KEYS[1])
    cfg = TP.br_config("br1")
    ctx.br_set_config(cfg)
    if not hf_check:
        ctx.br_set_hf_check(False)
    stream = torch.cuda.current_stream().cuda_stream
    frames, ifis, good, abytes = br_templates()
    tmpl, tid, lens, _, n_good = br_batch(n, W.rank)
    d_tid = torch.from_numpy(tid.astype(np.int64)).cuda()
    master = torch.from_numpy(tmpl).cuda()[d_tid]                    # n x 2 KiB, gathered on device
    d_len = torch.from_numpy(lens.view(np.int16)).cuda()
    d_if = torch.from_numpy(np.array(ifis, dtype=np.int32)).cuda()[d_tid]
    act = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ver = torch.zeros_like(act)
    egr = torch.zeros(n, dtype=torch.int32, device="cuda")
    stats = torch.zeros(64 * 2 * 11, dtype=torch.int64, device="cuda")
    alg = float(np.array(abytes)[tid].mean())
    work = torch.empty_like(master)
    for _ in range(max(1, warmup)):
        work.copy_(master)
        ctx.br_process(work, BR_SLOT, d_len, d_if, n, act, ver, egr, stats, stream=stream)
    W.sync()
    n_fwd = int((act == 4).sum())
    if hf_check:
        assert n_fwd == n_good and int((ver == hfv.VERDICT["INVALID_HF"]).sum()) == n - n_good
    else:
        assert n_fwd == n        # no MAC check: every scenario frame is forwarded
    del work
    copies = [master.clone() for _ in range(steps)]
    it = iter(copies)
    el, per_rank = W.timed(steps, lambda: ctx.br_process(next(it), BR_SLOT, d_len, d_if, n, act, ver, egr, stats,
                                                         stream=stream))
    ks = []
    for c in copies[: min(steps, 10)]:
        c.copy_(master)
        ks.append(ctx.br_process_timed(c, BR_SLOT, d_len, d_if, n, act, ver, egr, stats, stream=stream))
    ks.sort()
    k_mean = float(np.mean(ks))
    achieved = alg * n / (k_mean * 1e-3) / 1e9
    res = {"el": el, "per_rank_s": per_rank, "k_mean": k_mean, "k_med": ks[len(ks) // 2], "alg": alg,
           "achieved": achieved, "n_good": n_good}
    sample = None
    if W.rank == 0:
        m = min(n, 1 << 16)
        sample = (master[:m].cpu().numpy(), lens[:m], np.array(ifis, dtype=np.uint32)[tid[:m]], cfg,
                  act[:m].cpu().numpy())
    del copies, master
    ctx.close()
    return res, sample


def run_br(args, W):
    n, steps = args.n, args.steps
    if steps > 32:
        raise SystemExit("--workload br keeps one pristine 2 KiB-slot batch per timed step in HBM: use --steps <= 32")
    import scion_hfv as hfv
    r, sample = measure_br(hfv, W, n, steps, args.warmup, hf_check=not args.no_hf_check)
    result = {
        "metric": "Mpkt/s full border-router per-packet path (parse + hop-field MAC verify + rewrite), "
                  "mixed 64-1500 B frames",
        "value": round(W.size * n * steps / r["el"] / 1e6, 2),
        "unit": "Mpkt/s", "n_gpus": W.n_gpus, "ranks": W.size, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(r["el"] / steps * 1e3, 5), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (PTF scenario frames of the reference test topology for BR 1, 24 flows, 64-1500 B, "
                "2 KiB slots, 1/16 corrupted MACs)",
        "config": {"workload": f"config 4: {n} frames per GPU through hfv_br_process as br1-ff00_0_1-1"
                               + ("" if not args.no_hf_check else ", HF check off (ENABLE_HF_CHECK=OFF)"),
                   "frames_per_gpu": n, "slot_bytes": BR_SLOT, "parallelism": f"batch-sharded x{W.size}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(r["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(r["achieved"] / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(f"br:{n}"),
                     "kernel": "k_br_process", "kernel_ms_mean": round(r["k_mean"], 5),
                     "kernel_ms_median": round(r["k_med"], 5), "algorithmic_bytes_per_frame": round(r["alg"], 2),
                     "kernel_mpkts": round(n / r["k_mean"] / 1e3, 1)},
        "per_rank_ms": [round(x * 1e3, 4) for x in r["per_rank_s"]],
    }
    if W.rank == 0 and W.size == 1 and args.cpu_budget > 0 and sample is not None:
        hf, lens, ifx, cfg, act = sample
        a_cpu, result["cpu_baseline"] = br_cpu_baseline(hf, lens, ifx, cfg, min(args.cpu_budget, 5.0))
        result["cpu_baseline"]["actions_match_gpu"] = bool((a_cpu == act).all()) if not args.no_hf_check else None
    if W.rank == 0:
        print(json.dumps(result), flush=True)


def run_br_host(args, W):
    import scion_hfv as hfv
    from scion_hfv import topology as TP
    n, steps = args.n, args.steps
    ctx = hfv.Ctx(W.device)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    tb = apply_thread_budget(args, thread_budget(W, ctx))
    os.sched_setaffinity(0, ctx.numa_cpus())       # this GPU's host feeder runs on its NUMA node
    tmpl, tid, lens, ifidx, n_good = br_batch(n, W.rank)
    pristine = tmpl[tid]                                   # n x 2 KiB in host memory
    frames = hfv.host_array(pristine.shape, np.uint8)
    if not args.no_register:
        ctx.host_register(frames)   # mapped: zero-copy (the kernel reads header windows over PCIe)
    act = np.zeros(n, np.uint8)
    ver = np.zeros(n, np.uint8)
    egr = np.zeros(n, np.int32)
    hdr = 256
    for _ in range(max(1, args.warmup)):
        frames[:] = pristine
        ctx.br_process_host(frames, BR_SLOT, lens, ifidx, n, act, ver, egr, None, window=args.window)
    assert int((act == 4).sum()) == n_good and int((ver == hfv.VERDICT["INVALID_HF"]).sum()) == n - n_good
    total = 0.0
    for _ in range(steps):
        frames[:, :hdr] = pristine[:, :hdr]                # restore the rewritten headers (untimed)
        W.barrier()
        t0 = time.perf_counter()
        ctx.br_process_host(frames, BR_SLOT, lens, ifidx, n, act, ver, egr, None, window=args.window)
        total += max(W.gather(time.perf_counter() - t0))
    if not args.no_register:
        ctx.host_unregister(frames)
    path = ("DMA of %d-byte header windows (unregistered ring)" % (args.window or 256) if args.no_register else
            "zero-copy: registered ring, the kernel reads 128-byte header windows and writes back rewritten rows")
    result = {
        "metric": "Mpkt/s full border-router path with frames in host memory (H2D + kernel + D2H), "
                  "mixed 64-1500 B frames",
        "value": round(W.size * n * steps / total / 1e6, 2), "unit": "Mpkt/s", "n_gpus": W.n_gpus, "ranks": W.size, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(total / steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (the config-4 frame mix, 2 KiB slots in registered host memory)",
        "config": {"workload": f"config 5: {n} host-resident frames per GPU through hfv_br_process_host",
                   "frames_per_gpu": n, "slot_bytes": BR_SLOT, "path": path, "numa_node": ctx.numa_node(),
                   "parallelism": f"batch-sharded x{W.size}, no collective"},
        "host_threads": tb,
    }
    if W.rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()


def pcie_probe(W, nbytes=64 << 20, reps=5):
    """This box's host<->device copy rates, measured in the same run as the PCIe-inclusive legs
    (so a box-to-box swing of host_e2e / config5_loop can be told from a regression, VERDICT r05
    weak #8): pinned H2D, D2H, and both directions at once on two streams (scripts/pcie_probe.py),
    every rank at once."""
    torch = W.torch
    h1 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def rate(fn, moved):
        fn()
        torch.cuda.synchronize()
        W.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return moved * reps / (time.perf_counter() - t0) / 1e9

    def both():
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    out = {"h2d_gbs": round(rate(lambda: d1.copy_(h1, non_blocking=True), nbytes), 1),
           "d2h_gbs": round(rate(lambda: h2.copy_(d2, non_blocking=True), nbytes), 1),
           "both_gbs": round(rate(both, 2 * nbytes), 1), "bytes": nbytes,
           "note": "pinned 64 MiB copies through the copy engines, this rank, all ranks at once"}
    del h1, h2, d1, d2
    return out


def host_leg(hfv, W, ctx, recs, n, ref_bits):
    """PCIe-inclusive rates on this rank (every rank at once when N > 1), the rank's host
    threads on its GPU's NUMA node: pageable records through pinned staging, and a
    registered ring read in place by the kernel."""
    os.sched_setaffinity(0, ctx.numa_cpus())
    hrecs = recs.cpu().numpy()
    hbits = np.zeros((n + 63) // 64, dtype=np.uint64)
    ctx.verify_records_host(hrecs, n, hbits)     # warm the pinned staging
    reps = 5
    W.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.verify_records_host(hrecs, n, hbits)
    th = max(W.gather((time.perf_counter() - t0) / reps))
    assert np.array_equal(hbits, ref_bits)
    ring = hfv.host_array((n, hfv.REC_SIZE), np.uint8)
    ring[:] = hrecs
    rbits = hfv.host_array(((n + 63) // 64,), np.uint64)
    ctx.host_register(ring)
    ctx.host_register(rbits)
    ctx.verify_records_host(ring, n, rbits)
    W.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.verify_records_host(ring, n, rbits)
    tz = max(W.gather((time.perf_counter() - t0) / reps))
    assert np.array_equal(rbits, hbits)
    ctx.host_unregister(ring)
    ctx.host_unregister(rbits)
    return {"host_e2e": {"mpkts": round(W.size * n / th / 1e6, 1), "ms_per_batch": round(th * 1e3, 3),
                         "numa_node": ctx.numa_node(),
                         "path": "pageable host -> INF/HF gathered into 24 B pinned staging records (host threads "
                                 "on the GPU's NUMA node) -> H2D -> kernel -> D2H -> host, 2^18-record chunks on 2 "
                                 "streams; whole job (all ranks at once)"},
            "host_e2e_zero_copy": {"mpkts": round(W.size * n / tz / 1e6, 1), "ms_per_batch": round(tz * 1e3, 3),
                                   "path": "registered host ring read by the kernel over PCIe in place (PCIe moves "
                                           "whole 64 B lines), bitmap written to registered host memory"}}


def measure_loop(hfv, W, total, chunk, chunks, producers, consumers, slot=144, inflight=2, dma=2, digest=False):
    """Config 5 in one process (hfv_loop_run): gen_packets.py's 1000 frames cycled by producer
    threads into a pinned RX ring, the router (br1-ff00_0_1-2 of br/evaluation) over each chunk
    (dma: 0 zero-copy, 1 through HBM both ways, 2 copied in and the changes written back by the
    kernel), consumer threads counting transmitted frames and dropping the rest."""
    from scion_hfv import evaluation as E
    ctx = hfv.Ctx(W.device)
    E.setup_ctx(ctx)
    frames = E.frames(1000)
    lens = np.full(1000, E.FRAME_LEN, dtype=np.uint16)
    kw = dict(rx_ifindex=E.RX_IFINDEX, slot=slot, chunk=chunk, chunks=chunks, producers=producers,
              consumers=consumers, inflight=inflight, dma=dma, digest=digest)
    ctx.loop_run(frames, lens, 4 * chunk, **kw)                          # warm up
    W.barrier()
    # a failure on one rank must not leave the others waiting in the gather: every rank gets
    # to it, with a negative time if its loop failed
    try:
        r = ctx.loop_run(frames, lens, total, **kw)
        ok = r["rx"] == total and r["tx"] == total and r["verdicts"][1] == total   # every frame forwarded
        err = None if ok else f"counts {r['rx']}/{r['tx']}/{r['verdicts']}"
    except Exception as e:   # noqa: BLE001 -- reported in the line, not fatal to the headline
        r, err = None, str(e)
    times = W.gather(r["seconds"] if r and not err else -1.0)
    ctx_numa = ctx.numa_node()
    ctx.close()
    # every rank's counts (and, with digest, the order-free digest of its transmitted frames) and
    # where its producer / consumer threads ran
    mine = {"rank": W.rank, "error": err}
    if r:
        mine.update({k: r[k] for k in ("rx", "tx", "tx_bytes", "drop", "verdicts", "numa_node", "threads",
                                        "threads_on_node")})
        mine["tx_digest"] = f"{r['tx_digest']:016x}" if digest else None
        mine["seconds"] = round(r["seconds"], 4)
    per_rank = W.gather_obj(mine)
    if min(times) < 0:
        return {"error": err or "a rank's loop failed", "per_rank_s": times, "per_rank": per_rank}
    el = max(times)
    r["numa_node"] = ctx_numa
    return {"mpkts": round(W.size * total / el / 1e6, 2), "seconds": round(el, 4), "frames_per_gpu": total,
            "chunk": chunk, "chunks": chunks, "producers": producers, "consumers": consumers, "slot": slot,
            "inflight": inflight, "router_io": ("zero-copy over PCIe", "DMA through HBM both ways",
                          "DMA in, changed bytes written back by the kernel")[int(dma)],
            "tx_gbit_s": round(W.size * total * E.FRAME_LEN * 8 / el / 1e9, 1), "numa_node": r.get("numa_node"),
            "per_rank": per_rank,
            "stage_busy_frac": {"router": round(r["gpu_busy_s"] / r["seconds"], 3),
                                "router_waiting_for_rx": round(r["gpu_wait_s"] / r["seconds"], 3),
                                "producer": round(r["producer_busy_s"] / producers / r["seconds"], 3),
                                "consumer": round(r["consumer_busy_s"] / consumers / r["seconds"], 3)},
            "path": f"producer threads memcpy 138 B frames into a pinned, mapped host RX ring ({slot} B slots) -> "
                    "the router kernel per chunk (router_io) -> consumer threads count TX / drop; producers and "
                    "consumers on the GPU's NUMA node",
            "veth": "not used: the GPU box runs commands as an unprivileged user with user namespaces disabled "
                    "(unshare -Urn: ENOSPC) and no CAP_NET_RAW (AF_PACKET: EPERM), so no veth pair can be made "
                    "there (scripts/netns_gpu_probe.py, DESIGN.md)"}


def run_loop(args, W):
    import scion_hfv as hfv
    c = hfv.Ctx(W.device)
    tb = apply_thread_budget(args, thread_budget(W, c))
    c.close()
    r = measure_loop(hfv, W, args.loop_n, args.loop_chunk, args.loop_chunks, args.loop_threads, args.loop_consumers,
                     args.loop_slot, args.loop_inflight, args.loop_dma, args.loop_digest)
    result = {
        "metric": "Mpkt/s config-5 loop: RX ring -> border router on the GPU -> TX/drop, 138 B frames",
        "value": r.get("mpkts"), "unit": "Mpkt/s", "n_gpus": W.n_gpus, "ranks": W.size, "steps": 1, "warmup": 1,
        "ms_per_step": round(r["seconds"] * 1e3, 3) if "seconds" in r else None, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (gen_packets.py's 1000 frames, cycled like tcpreplay --loop)",
        "config": {"workload": f"config 5: {args.loop_n} frames per GPU through hfv_loop_run as br1-ff00_0_1-2",
                   "parallelism": f"one loop per GPU x{W.size}, no collective"},
        "loop": r,
        "host_threads": tb,
    }
    if W.rank == 0:
        print(json.dumps(result), flush=True)


def run_dry(args, W):
    """Launcher check without a GPU: every rank times K trivial CPU steps."""
    x = np.arange(1 << 12, dtype=np.uint64)
    el, per_rank = W.timed(args.steps, lambda: np.bitwise_xor.reduce(x))
    if W.rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mpkt/s", "n_gpus": W.n_gpus, "ranks": W.size, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "dry run: launcher check only, no GPU work", "config": {"workload": "dry run"},
                          "per_rank_ms": [round(t * 1e3, 4) for t in per_rank], "backend": W.backend}), flush=True)


def run_hf(args, W):
    import scion_hfv as hfv
    torch = W.torch
    keysel = hfv.KEYSEL_IFID if args.keysel == "ifid" else hfv.KEYSEL_ZERO
    n = args.n
    if args.strong:   # a fixed total, sliced over the ranks (scion_hfv.shard_range)
        a, b = hfv.shard_range(args.n, W.size, W.rank)
        n, total = b - a, args.n
        first = a * args.rotate
    else:             # weak: every rank verifies its own n records per step
        first, total = W.rank * args.n * args.rotate, W.size * args.n
    ctx = make_ctx(hfv, W.device, keysel)
    stream = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(W.device).multi_processor_count
    tb = apply_thread_budget(args, thread_budget(W, ctx))
    svc_blocks = 0
    if args.same_device and W.size > 1:
        # ranks sharing one GPU: each service grid takes its share of the CUs (one block per CU
        # holds the CU's LDS), so the grids run side by side instead of one after the other
        svc_blocks = max(1, cus // W.size)
        ctx.service_set_grid(svc_blocks)
    m = measure_hf(hfv, W, ctx, args.keysel, n, first, args.rotate, args.steps, args.warmup, stream, reps=args.svc_reps,
                   service=not args.launch_only)
    # every rank's median event-timed grid (the service's kernel time per rank), and no rank starts
    # an extra leg (host threads, PCIe copies) while another is still in its headline regions
    per_rank_grid = W.gather(m["grid_ms"] or 0.0)
    W.barrier()
    headline = "launch" if args.launch_only else args.mode
    elapsed = {"service": m["svc_el"], "launch": m["launch_el"], "batches": m["bat_el"]}[headline]
    if headline == "batches":
        m["per_rank_s"] = m["bat_per_rank_s"]
    bytes_per_batch = BYTES_PER_PACKET * n
    if headline == "batches":
        achieved = bytes_per_batch * args.steps / (m["bat_kernel_ms"] * 1e-3) / 1e9
        kern = {"kernel": "k_verify_batches", "kernel_ms": round(m["bat_kernel_ms"], 4),
                "batches_per_call": args.steps, "launches": -(-args.steps // 64),
                "kernel_ms_per_batch": round(m["bat_kernel_ms"] / args.steps, 5),
                "algorithmic_bytes_per_batch": int(bytes_per_batch),
                "timing": "dispatch start/stop events (hipExtLaunchKernel) of the call's launches, in calls identical "
                          "to the value's but for the events (median)"}
        traffic = pmc_traffic(f"bat:{args.keysel}:{n}:rot{args.rotate}")
    elif headline == "service":
        achieved = bytes_per_batch * args.steps / (m["grid_ms"] * 1e-3) / 1e9
        kern = {"kernel": "k_verify_service", "grid_ms": round(m["grid_ms"], 4), "batches_per_grid": args.steps,
                "kernel_ms_per_batch": round(m["grid_ms"] / args.steps, 5),
                "algorithmic_bytes_per_batch": int(bytes_per_batch),
                "timing": "dispatch start/stop events of the service grid (hipExtLaunchKernel) over all K batches, "
                          "in timed regions identical to the value's but for the events (median grid)"}
        traffic = pmc_traffic(f"svc:{args.keysel}:{n}:rot{args.rotate}")
    else:
        achieved = bytes_per_batch / (m["k_mean"] * 1e-3) / 1e9
        kern = {"kernel": "k_verify_batches (one batch per launch: hfv_verify_records)", "kernel_ms_mean": round(m["k_mean"], 5),
                "kernel_ms_median": round(m["k_med"], 5), "algorithmic_bytes_per_launch": int(bytes_per_batch)}
        traffic = pmc_traffic(f"{args.keysel}:{n}:rot{args.rotate}")
    result = {
        "metric": METRIC,
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "Mpkt/s",
        "n_gpus": W.n_gpus, "ranks": W.size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (64 B SCION records, splitmix64 seed 0x5C100001, 1/16 corrupted MACs; generated on device)",
        "config": {"workload": f"config {'3' if keysel else '2'}: "
                               f"{f'{total} x 64 B records per step in total' if args.strong else f'{n} x 64 B records per GPU per step'}, "
                               f"{'256 ingress-interface keys (KEYSEL_IFID)' if keysel else 'single AS key'}",
                   "records_per_gpu": n, "record_bytes": 64, "keysel": args.keysel,
                   "resident_batches_per_gpu": args.rotate,
                   "resident_bytes_per_gpu": args.rotate * n * 64,
                   "parallelism": f"batch-sharded x{W.size}, no collective"},
        "roofline": dict({"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic}, **kern,
                         achievable_peak=m["stream_read"]["gbs"],
                         frac_of_achievable=round(achieved / m["stream_read"]["gbs"], 4),
                         achievable_source="median of a dense streaming read of the same resident batches in this "
                                           "run (stream_read)",
                         variant=ctx.describe(),
                         note=f"step k verifies resident batch k % {args.rotate} ({args.rotate} x {n * 64 >> 20} MiB "
                              f"per GPU > 256 MiB Infinity Cache): records are read from HBM"),
        "stream_read": m["stream_read"],
        "ceilings": ceilings(args.keysel, n, m["bat_mhz"] if headline == "batches" else m["mhz"], cus,
                             "batches" if headline == "batches" else "service"),
        "path": {"service": "resident service: one persistent grid; the K batches and a stop descriptor posted "
                            "through the host descriptor ring by one hfv_service_run_async call, which launches the "
                            "grid after them; the timed region's closing device synchronize waits for the grid to "
                            "exit; posting, grid launch, table fill and drain inside the timed region",
                 "batches": "stream-ordered batch list: the K batches in one hfv_verify_batches call on the rank's "
                            "stream (one launch per 64 batches: table fill, ramp and tail paid once per launch); the "
                            "timed region's closing device synchronize waits for it",
                 "launch": "one hfv_verify_records launch per batch"}[headline],
        "batches": {"mpkts": round(total * args.steps / m["bat_el"] / 1e6, 2),
                    "ms_per_step": round(m["bat_el"] / args.steps * 1e3, 5),
                    "kernel_ms": round(m["bat_kernel_ms"], 4),
                    "frac": round(bytes_per_batch * args.steps / (m["bat_kernel_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "timed_regions_ms": m["bat_all_ms"], "kernel_ms_all": m["bat_all_kernel_ms"],
                    "shader_mhz": round(m["bat_mhz"], 1) if m["bat_mhz"] else None, "mhz_all": m["bat_all_mhz"],
                    "path": "hfv_verify_batches: K batches, one stream-ordered launch per 64"},
        "service": None if args.launch_only else {
            "mpkts": round(total * args.steps / m["svc_el"] / 1e6, 2),
            "ms_per_step": round(m["svc_el"] / args.steps * 1e3, 5), "grid_ms": round(m["grid_ms"], 4),
            "shader_mhz": round(m["mhz"], 1) if m["mhz"] else None,
            "timed_regions_ms": m.get("svc_all_ms"), "grids_ms": m.get("svc_all_grid_ms"),
            "event_timed_regions_ms": m.get("svc_timed_regions_ms"), "value_regions": m.get("svc_value_regions"),
            "service_run_call_us": m.get("svc_all_call_us"),
            "grids_mhz": m.get("svc_grid_mhz"), "weights": m.get("svc_weights"),
            "relay": m.get("svc_relay"),
            "note": f"value = the median of {args.svc_reps} timed regions of K steps each (each a fresh grid)"},
        "per_launch": {"mpkts": round(total * args.steps / m["launch_el"] / 1e6, 2),
                       "ms_per_step": round(m["launch_el"] / args.steps * 1e3, 5),
                       "kernel_ms_mean": round(m["k_mean"], 5), "kernel_ms_median": round(m["k_med"], 5),
                       "kernel_mpkts": round(n / m["k_mean"] / 1e3, 1),
                       "frac": round(bytes_per_batch / (m["k_mean"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "per_rank_ms": {"min": round(min(m["per_rank_s"]) * 1e3, 4), "max": round(max(m["per_rank_s"]) * 1e3, 4),
                        "all": [round(x * 1e3, 4) for x in m["per_rank_s"]],
                        "grid_ms": [round(x, 4) for x in per_rank_grid] if headline == "service" else None},
        "host_threads": tb,
    }
    if args.same_device:
        result["same_device"] = {"ranks": W.size, "physical_gpus": 1,
                                 "service_grid_blocks": svc_blocks,
                                 "note": "launcher rehearsal: every rank on GPU 0"}
    recs0, bits0 = m["batches"][0], m["bitmaps"][0]
    ref_bits = bits0.cpu().numpy().view(np.uint64).copy()   # the headline's own bitmap of batch 0
    if not args.no_extras and not args.launch_only:
        settle(args)
        result.update(service_legs(hfv, W, ctx, m, n, first, args.rotate, args.steps))
    extras = W.size == 1 and not args.no_extras

    if extras:   # the same batch re-posted: served from the Infinity Cache (diagnostic)
        for b in m["bitmaps"]:
            b.zero_()
        W.sync()
        g = service_grid(ctx, [recs0], args.steps, m["bitmaps"], n)
        result["mall_resident"] = {"records": n, "service_ms_per_batch": round(g / args.steps, 5),
                                   "service_mpkts": round(n * args.steps / g / 1e3, 1),
                                   "service_frac": round(bytes_per_batch * args.steps / (g * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "note": "one 64 MiB batch re-posted K times: Infinity-Cache bandwidth, not HBM"}
        W.sync()
        assert popcount(m["bitmaps"][0]) == expected_pass_count(n, first)

    if extras and args.big_n:
        settle(args)
        nb = args.big_n
        big = torch.empty((nb, 64), dtype=torch.uint8, device="cuda")
        ctx.gen_records(big, nb, SEED_RECORDS, first_index=0, stream=stream)
        bbits = [torch.zeros((nb + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(4)]
        for _ in range(3):
            ctx.verify_records(big, nb, bbits[0], stream=stream)
        W.sync()
        assert popcount(bbits[0]) == expected_pass_count(nb, 0)
        ks = sorted(ctx.verify_records_timed(big, nb, bbits[0], stream=stream) for _ in range(10))
        bm = float(np.mean(ks))
        ach = BYTES_PER_PACKET * nb / (bm * 1e-3) / 1e9
        for b in bbits:
            b.zero_()
        W.sync()
        sg = service_grid(ctx, [big], 4, bbits, nb)
        smhz = ctx.service_shader_mhz()
        for b in bbits:
            assert popcount(b) == expected_pass_count(nb, 0)
        sach = BYTES_PER_PACKET * nb * 4 / (sg * 1e-3) / 1e9
        result["hbm_resident"] = {"records": nb, "kernel_ms_mean": round(bm, 4), "mpkts": round(nb / bm / 1e3, 1),
                                  "achieved_GBs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                                  "traffic": pmc_traffic(f"{args.keysel}:{nb}"),
                                  "service_ms_per_batch": round(sg / 4, 4),
                                  "service_mpkts": round(nb * 4 / sg / 1e3, 1),
                                  "service_frac": round(sach / HBM_PEAK_GBS, 4),
                                  "service_traffic": pmc_traffic(f"svc:{args.keysel}:{nb}"),
                                  "service_shader_mhz": round(smhz, 1) if smhz else None}
        del big, bbits

    if extras and keysel == hfv.KEYSEL_ZERO:   # config 3 beside the config-2 headline
        settle(args)
        ctx3 = make_ctx(hfv, W.device, hfv.KEYSEL_IFID)
        m3 = measure_hf(hfv, W, ctx3, "ifid", n, first, args.rotate, args.steps, args.warmup, stream,
                        reps=args.svc_reps)
        a3 = bytes_per_batch * args.steps / (m3["grid_ms"] * 1e-3) / 1e9
        result["config3"] = {"workload": f"config 3: {n} x 64 B records per GPU per step, 256 ingress-interface "
                                         "keys (KEYSEL_IFID), same rotation and timing as the headline",
                             "mpkts": round(total * args.steps / m3["svc_el"] / 1e6, 2),
                             "ms_per_step": round(m3["svc_el"] / args.steps * 1e3, 5),
                             "grid_ms": round(m3["grid_ms"], 4), "frac": round(a3 / HBM_PEAK_GBS, 4),
                             "grids_ms": m3["svc_all_grid_ms"], "grids_mhz": m3["svc_grid_mhz"],
                             "per_launch_mpkts": round(total * args.steps / m3["launch_el"] / 1e6, 2),
                             "shader_mhz": round(m3["mhz"], 1) if m3["mhz"] else None,
                             "batches_kernel_ms": round(m3["bat_kernel_ms"], 4),
                             "batches_frac": round(bytes_per_batch * args.steps / (m3["bat_kernel_ms"] * 1e-3) / 1e9
                                                   / HBM_PEAK_GBS, 4),
                             "batches_mpkts": round(total * args.steps / m3["bat_el"] / 1e6, 2),
                             "ceilings": ceilings("ifid", n, m3["mhz"], cus, "service"),
                             "batches_ceilings": ceilings("ifid", n, m3["bat_mhz"], cus, "batches")}
        del m3
        ctx3.close()

    pcie = None
    if not args.no_host_e2e or (args.loop_n and not args.no_extras):
        pcie = pcie_probe(W)
        result["pcie_probe"] = pcie
    if not args.no_host_e2e:
        result.update(host_leg(hfv, W, ctx, recs0, n, ref_bits))
        # the leg against the same run's copy rate: 24 B staging records in (+ 1/8 B of verdicts out)
        result["host_e2e"]["h2d_frac"] = round(result["host_e2e"]["mpkts"] / W.size * 1e6 * 24.125 / 1e9
                                               / pcie["h2d_gbs"], 3)

    if extras and args.br_n:
        settle(args)
        W.sync()
        r4, sample = measure_br(hfv, W, args.br_n, 5, 2)
        r4off, _ = measure_br(hfv, W, args.br_n, 5, 2, hf_check=False)
        result["config4"] = {"workload": f"config 4: {args.br_n} mixed 64-1500 B frames (2 KiB slots) through "
                                         "hfv_br_process as br1 of the reference test topology",
                             "mpkts": round(args.br_n * 5 / r4["el"] / 1e6, 2),
                             "kernel_ms_mean": round(r4["k_mean"], 4),
                             "kernel_mpkts": round(args.br_n / r4["k_mean"] / 1e3, 1),
                             "frac": round(r4["achieved"] / HBM_PEAK_GBS, 4),
                             "algorithmic_bytes_per_frame": round(r4["alg"], 2),
                             "traffic": pmc_traffic(f"br:{args.br_n}"),
                             "hf_check_off_kernel_ms_mean": round(r4off["k_mean"], 4),
                             "hf_check_off_mpkts": round(args.br_n * 5 / r4off["el"] / 1e6, 2),
                             "hf_check_share": round(1 - r4off["k_mean"] / r4["k_mean"], 3),
                             "note": "hf_check_off = the reference's ENABLE_HF_CHECK=OFF build (br/CMakeLists.txt:8,"
                                     "48-64); hf_check_share = the part of the kernel time the MAC check costs"}

    if args.loop_n and not args.no_extras:   # config 5 runs on every rank (8x batch-sharded at N = 8)
        W.sync()
        result["config5_loop"] = measure_loop(hfv, W, args.loop_n, args.loop_chunk, args.loop_chunks, args.loop_threads,
                                              args.loop_consumers, args.loop_slot, args.loop_inflight, args.loop_dma,
                                              args.loop_digest)
        lp = result["config5_loop"]
        if "mpkts" in lp and pcie:   # the slot's bytes cross PCIe inward once per frame (DMA in)
            lp["h2d_frac"] = round(lp["mpkts"] / W.size * 1e6 * args.loop_slot / 1e9 / pcie["h2d_gbs"], 3)

    if extras:
        result["settle_s_before_extra_legs"] = args.settle_s
    # every rank's GPU work is done before the CPU baseline runs (it shares the host with them)
    W.barrier()
    if W.rank == 0 and args.cpu_budget > 0:
        result["cpu_baseline"] = cpu_baseline(recs0.cpu().numpy(), keysel, ref_bits, args.cpu_budget)
        if W.size > 1:
            result["cpu_baseline"]["note"] = (f"rank 0 after all {W.size} ranks finished their GPU legs, its "
                                              f"threads on GPU 0's share of the host")

    if W.rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 200 (hf), 10 (br), 5 (br-host)")
    ap.add_argument("--warmup", type=int, default=None, help="default 20 (hf), 3 (br), 1 (br-host)")
    ap.add_argument("--records", "--n", dest="n", type=int, default=1 << 20, help="records per GPU per step (config 2: 2^20); with --strong, in total")
    ap.add_argument("--rotate", type=int, default=8,
                    help="resident batches per GPU; step k verifies batch k %% R (8 x 64 MiB > the 256 MiB Infinity Cache)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --n records in total per step, sliced over the ranks on 64-record boundaries")
    ap.add_argument("--keysel", choices=["zero", "ifid"], default="zero")
    ap.add_argument("--big-n", type=int, default=1 << 24, help="HBM-resident single-batch run size (0 = skip)")
    ap.add_argument("--br-n", type=int, default=1 << 20, help="config-4 leg frames (0 = skip)")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of multi-thread CPU baseline (0 = skip)")
    ap.add_argument("--no-host-e2e", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline only (no config 3/4, 2^24, MALL legs)")
    ap.add_argument("--workload", choices=["hf", "br", "br-host", "loop"], default="hf",
                    help="hf: hop-field verify on 64 B records (configs 2/3, the headline); br: config 4; "
                         "br-host: config 5 router leg; loop: config 5 RX ring -> router -> TX loop")
    ap.add_argument("--loop-n", type=int, default=1 << 24, help="config-5 loop frames (0 = skip the leg)")
    ap.add_argument("--loop-chunk", type=int, default=1 << 16, help="config-5 loop frames per chunk")
    ap.add_argument("--loop-chunks", type=int, default=12, help="config-5 loop ring chunks")
    ap.add_argument("--loop-threads", type=int, default=8, help="config-5 loop producer threads")
    ap.add_argument("--loop-consumers", type=int, default=4, help="config-5 loop consumer threads")
    ap.add_argument("--loop-slot", type=int, default=144, help="config-5 loop ring slot bytes")
    ap.add_argument("--loop-inflight", type=int, default=2, help="config-5 loop chunks on the GPU at once")
    ap.add_argument("--loop-dma", type=int, default=2, choices=(0, 1, 2),
                    help="config-5 loop router I/O: 0 zero-copy over PCIe, 1 DMA through HBM both ways, "
                         "2 DMA in + the kernel writing its changes into the ring")
    ap.add_argument("--loop-digest", action="store_true",
                    help="config-5 loop: consumers sum a 64-bit digest of every transmitted frame (per rank in the line)")
    ap.add_argument("--mode", choices=["service", "launch", "batches"], default="batches",
                    help="hf headline: the K batches in one stream-ordered hfv_verify_batches call (default), "
                         "the resident service grid, or one launch per batch")
    ap.add_argument("--settle-s", type=float, default=0.5, help="idle seconds before each extra leg (untimed)")
    ap.add_argument("--svc-reps", type=int, default=5, help="timed service regions of K steps (median reported; 5: robust to two host hiccups)")
    ap.add_argument("--launch-only", action="store_true",
                    help="measure the launch path only (ranks sharing one GPU cannot each hold a service grid)")
    ap.add_argument("--window", type=int, default=256, help="br-host: header bytes per frame moved over PCIe")
    ap.add_argument("--no-register", action="store_true", help="br-host: leave the ring unregistered (DMA windows)")
    ap.add_argument("--no-hf-check", action="store_true", help="br: the ENABLE_HF_CHECK=OFF router")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on GPU 0 (launcher rehearsal on 1 GPU; gloo; service grids of cus/ranks blocks)")
    ap.add_argument("--dry-run", action="store_true", help="launcher check: gloo ranks, no GPU work")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = {"hf": 200, "br": 10, "br-host": 5, "loop": 1}[args.workload]
    if args.warmup is None:
        args.warmup = {"hf": 20, "br": 3, "br-host": 1, "loop": 1}[args.workload]
    if args.same_device:
        args.dist_backend = "gloo"   # one GPU: RCCL would not place two ranks on it
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))           # before anything touches a GPU
    W = World(args)
    try:
        if args.dry_run:
            run_dry(args, W)
        elif args.workload == "br":
            run_br(args, W)
        elif args.workload == "br-host":
            run_br_host(args, W)
        elif args.workload == "loop":
            run_loop(args, W)
        else:
            run_hf(args, W)
    finally:
        W.close()


if __name__ == "__main__":
    main()
