#!/usr/bin/env python3
"""Headline benchmark: Mpkt/s of device-resident hop-field AES-CMAC verify on 64 B SCION
records (BASELINE.json metric; config 2 = 2^20 records, single AS key, per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keysel zero|ifid] [--n N]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One process per GPU.  A "step" is one pass of the verifier over the rank's resident batch
of n records (weak scaling: every rank verifies its own n records, no collective on the
data path; RCCL is used only for the timing barrier and max-over-ranks).  By default
(--mode service) the K steps are K batches posted one by one to the resident service
(hfv_service_submit: the XDP program's counterpart, a grid that stays on the GPU), with
starting and stopping its grid inside the timed region; --mode launch times one
hfv_verify_records launch per step instead (both are always measured and reported:
`service`, `per_launch`).  Rank 0 prints one JSON line.  Besides
the contract fields it carries:
  roofline      -- the headline kernel's algorithmic bytes (64 B read + 1/8 B verdict per
                   record) / its duration from the dispatch's own start/stop events (the
                   service grid's lifetime over all K batches, or the mean launch), against
                   the 8 TB/s HBM3E peak; `traffic` is the PMC-measured HBM bytes per batch
                   from profiles/ when a matching pass exists.
  cpu_baseline  -- the reference's own aes.c soft path (oracle/_ref, built from
                   /root/reference) over a sample of the same records on this host's cores,
                   verdicts cross-checked against the GPU bitmap.
  hbm_resident  -- the same kernel on 2^24 records (1 GiB > 256 MiB Infinity Cache).
  host_e2e      -- rate including H2D/D2H through pinned staging (hfv_verify_records_host).

    python bench.py --workload br [--n 1048576] [--steps 10]

runs config 4 instead: the full border-router per-packet path (hfv_br_process: parse,
AS ingress/egress, next hop, rewrite, MAC check, counters) as BR 1 of the reference test
topology, over n frames of 64..1500 B in 2 KiB slots (PTF scenario traffic, 1/16 with a
corrupted hop-field MAC).  Frames are rewritten in place, so each timed step gets its own
pristine copy of the batch (K copies resident in HBM, made before the timed region).

    python bench.py --workload br-host [--n 1048576] [--steps 5] [--window 256]

runs config 5: the same frames start and end in (registered) host memory; per step one
hfv_br_process_host call moves the header windows over PCIe, processes them and writes the
rewritten windows back.  Each step's input is restored (untimed) before it runs.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import scion_hfv as hfv  # noqa: E402

SEED_RECORDS = 0x5C100001
SEED_KEYS = 0x5C100100
KEY_1111 = b"1111111111111111"   # br/test/run_tests:113
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
M64 = (1 << 64) - 1


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


def expected_pass_count(n, first_index):
    """Generator truth: record i is corrupted iff splitmix draw 4i+2 & 15 == 0."""
    i = np.arange(first_index, first_index + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(SEED_RECORDS) + (np.uint64(4) * i + np.uint64(3)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return int(((z & np.uint64(15)) != 0).sum())


def popcount(bits_t):
    b = bits_t.cpu().numpy().view(np.uint8)
    return int(np.unpackbits(b).sum())


def make_ctx(device, keysel):
    ctx = hfv.Ctx(device)
    if keysel == hfv.KEYSEL_IFID:
        ctx.key_add_batch(0, key_table_256())
    else:
        ctx.key_add(0, KEY_1111)
    ctx.set_keysel(keysel)
    return ctx


def kernel_ms(ctx, recs, n, bits, stream, reps):
    """Mean/median execution time of one verify launch on `stream`, from the dispatch's own
    start/stop timestamps (hipExtLaunchKernel events, hfv_verify_records_timed)."""
    ts = sorted(ctx.verify_records_timed(recs, n, bits, stream=stream) for _ in range(reps))
    return float(np.mean(ts)), float(ts[len(ts) // 2])


def timed_steps(world, steps, fn):
    """Run fn `steps` times between barrier + device sync on both sides; max over ranks."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def ceilings(keysel):
    """The other bounds beside HBM, per packet, from this repo's own measurements (DESIGN.md
    section 4): LDS lookups and VALU instructions per packet (PMC SQ_INSTS_LDS/VALU x 64 /
    records, profiles/r01/service/pmc_zero_svc), the chip's conflict-free ds_read_b32 rate
    (scripts/ubench/valu_rate.hip) and the streaming-read rate of the same access pattern
    without compute (scripts/ubench/stream_read.hip, 1 GiB)."""
    lds_per_pkt = 146.2 if keysel == "zero" else None
    lds_rate = 16.8e12
    out = {"lds_lookups_per_pkt": lds_per_pkt, "lds_peak_lookups_per_s": lds_rate,
           "valu_instr_per_pkt": 277.0 if keysel == "zero" else None,
           "streaming_read_GBs": 6552.0, "streaming_read_frac": round(6552.0 / HBM_PEAK_GBS, 3),
           "source": "profiles/r01/service/pmc_zero_svc/summary.json, profiles/r01/ubench/"}
    if lds_per_pkt:
        out["lds_bound_mpkts"] = round(lds_rate / lds_per_pkt / 1e6, 1)
    out["streaming_read_bound_mpkts"] = round(6552.0e9 / hfv.BYTES_PER_PACKET / 1e6, 1)
    return out


def lds_bound_at_clock(keysel, mhz):
    """The LDS-issue bound at the shader clock the service grid actually ran at (it is power
    limited: ~2.38 GHz with 32 CUs busy, ~1.5-1.6 GHz sustained with all 256, scripts/svc_probe.py):
    conflict-free ds_read_b32 retires 32 lanes per clock per CU."""
    if not mhz or keysel != "zero":
        return {}
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    # VALU: per 64-packet tile 145 v_perm_b32 (4 SIMD cycles per wave64 instruction, measured
    # half rate) + 132 full-rate instructions (2 cycles); 4 SIMDs per CU
    valu_cycles_per_pkt = (145 * 4 + 132 * 2) / 64.0
    return {"service_shader_mhz": round(mhz, 1),
            "lds_bound_mpkts_at_service_clock": round(cus * 32 * mhz * 1e6 / 146.2 / 1e6, 1),
            "valu_bound_mpkts_at_service_clock": round(cus * 4 * mhz * 1e6 / valu_cycles_per_pkt / 1e6, 1)}


def pmc_traffic(keysel, n, service=False):
    """HBM bytes per launch (per batch for the resident service) measured by rocprofv3 PMC
    passes (scripts/pmc_round.sh) for this exact configuration, committed in
    profiles/traffic.json; None if not measured."""
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        return json.load(open(tpath))[f"{'svc:' if service else ''}{keysel}:{n}"]["hbm_bytes_per_launch"]
    except Exception:
        return None


def cpu_baseline(recs_host, keysel, gpu_bits, budget_s):
    """The reference aes.c soft path (XDP's arithmetic) timed on this host's cores over a
    bounded sample of the same records; verdicts must equal the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc   # test infrastructure: only this leg of the bench may use it

    raw = key_table_256() if keysel == hfv.KEYSEL_IFID else KEY_1111
    hk, valid = orc.key_table(raw)
    raw256 = raw + bytes(16 * (256 - len(raw) // 16))
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    n = len(recs_host)
    use_ref = orc.reference() is not None

    def run(nthreads, aesni=0):
        if use_ref:
            return orc.ref_verify_records(recs_host, raw256, hk, valid, keysel, nthreads=nthreads, aesni=aesni)
        return orc.verify_records(recs_host, hk, valid, keysel, nthreads=nthreads)

    t0 = time.perf_counter()
    bits1 = run(1)
    t1c = time.perf_counter() - t0
    reps, t_all = 0, 0.0
    while t_all < budget_s or reps == 0:
        t0 = time.perf_counter()
        bitsN = run(cores)
        t_all += time.perf_counter() - t0
        reps += 1
    assert np.array_equal(bits1, bitsN)
    match = bool(np.array_equal(bitsN, gpu_bits))
    out = {"value": round(n * reps / t_all / 1e6, 3), "unit": "Mpkt/s", "cores": cores,
           "kind": "reference" if use_ref else "port",
           "sample": f"{n} records of the benched batch x {reps} passes, aes_cmac soft path (aes/src/aes.c), "
                     f"{cores} threads; 1-thread {round(n / t1c / 1e6, 3)} Mpkt/s",
           "single_core_mpkts": round(n / t1c / 1e6, 3),
           "verdicts_match_gpu": match}
    if use_ref:
        t0 = time.perf_counter()
        bitsA = run(cores, aesni=1)
        ta = time.perf_counter() - t0
        assert np.array_equal(bitsA, bitsN)
        out["aesni_mpkts"] = round(n / ta / 1e6, 3)
    return out


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


def corrupted(n, first_index=0):
    """Same 1/16 corruption draw as the 64 B records (splitmix64 draw 4i+2 & 15 == 0)."""
    i = np.arange(first_index, first_index + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(SEED_RECORDS) + (np.uint64(4) * i + np.uint64(3)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(15)) == 0


def br_cpu_baseline(frames_host, lens, ifidx, cfg, budget_s):
    """The oracle border router (a scalar C restatement of xdp.c; the BPF program itself cannot
    run here) on one host core over a sample of the same frames."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc   # test infrastructure: only the cpu_baseline leg may use it
    from scion_hfv import topology as TP
    hk = orc.hop_key(TP.KEYS[1])
    reps, t_all, n = 0, 0.0, len(frames_host)
    while t_all < budget_s or reps == 0:
        work = frames_host.copy()
        t0 = time.perf_counter()
        a, v, e, s = orc.br_process(work, lens, ifidx, cfg, hk)
        t_all += time.perf_counter() - t0
        reps += 1
    return a, {"value": round(n * reps / t_all / 1e6, 3), "unit": "Mpkt/s", "cores": 1, "kind": "port",
               "sample": f"{n} frames of the benched mix x {reps} passes, oracle/hfv_br_oracle.c (scalar restatement "
                         f"of br/src/bpf/xdp.c process_packet + verify), 1 thread"}


def run_br(args, rank, world, local):
    from scion_hfv import topology as TP
    n, steps = args.n, args.steps
    if steps > 32:
        raise SystemExit("--workload br keeps one pristine 2 KiB-slot batch per timed step in HBM: use --steps <= 32")
    ctx = hfv.Ctx(local)
    ctx.key_add(0, TP.KEYS[1])
    cfg = TP.br_config("br1")
    ctx.br_set_config(cfg)
    stream = torch.cuda.current_stream().cuda_stream
    frames, ifis, good, abytes = br_templates()
    tmpl, tid, lens, _, n_good = br_batch(n, rank)
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
    for _ in range(max(1, args.warmup)):
        work.copy_(master)
        ctx.br_process(work, BR_SLOT, d_len, d_if, n, act, ver, egr, stats, stream=stream)
    torch.cuda.synchronize()
    assert int((act == 4).sum()) == n_good and int((ver == hfv.VERDICT["INVALID_HF"]).sum()) == n - n_good
    del work
    copies = [master.clone() for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in copies:
        ctx.br_process(c, BR_SLOT, d_len, d_if, n, act, ver, egr, stats, stream=stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ks = []
    for c in copies[: min(steps, 10)]:
        c.copy_(master)
        ks.append(ctx.br_process_timed(c, BR_SLOT, d_len, d_if, n, act, ver, egr, stats, stream=stream))
    ks.sort()
    k_mean = float(np.mean(ks))
    achieved = alg * n / (k_mean * 1e-3) / 1e9
    result = {
        "metric": "Mpkt/s full border-router per-packet path (parse + hop-field MAC verify + rewrite), "
                  "mixed 64-1500 B frames",
        "value": round(world * n * steps / elapsed / 1e6, 2),
        "unit": "Mpkt/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 5), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (PTF scenario frames of the reference test topology for BR 1, 24 flows, 64-1500 B, "
                "2 KiB slots, 1/16 corrupted MACs)",
        "config": {"workload": f"config 4: {n} frames per GPU through hfv_br_process as br1-ff00_0_1-1",
                   "frames_per_gpu": n, "slot_bytes": BR_SLOT, "parallelism": f"batch-sharded x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("br", n), "kernel": "k_br_process",
                     "kernel_ms_mean": round(k_mean, 5), "kernel_ms_median": round(ks[len(ks) // 2], 5),
                     "algorithmic_bytes_per_frame": round(alg, 2),
                     "kernel_mpkts": round(n / k_mean / 1e3, 1)},
    }
    if rank == 0 and world == 1 and args.cpu_budget > 0:
        m = min(n, 1 << 16)
        hf = master[:m].cpu().numpy()
        a_cpu, result["cpu_baseline"] = br_cpu_baseline(hf, lens[:m], np.array(ifis, dtype=np.uint32)[tid[:m]],
                                                        cfg, min(args.cpu_budget, 5.0))
        result["cpu_baseline"]["actions_match_gpu"] = bool((a_cpu == act[:m].cpu().numpy()).all())
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


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


def run_br_host(args, rank, world, local):
    from scion_hfv import topology as TP
    n, steps = args.n, args.steps
    ctx = hfv.Ctx(local)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    tmpl, tid, lens, ifidx, n_good = br_batch(n, rank)
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
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        ctx.br_process_host(frames, BR_SLOT, lens, ifidx, n, act, ver, egr, None, window=args.window)
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        total += dt
    if not args.no_register:
        ctx.host_unregister(frames)
    path = ("DMA of %d-byte header windows (unregistered ring)" % (args.window or 256) if args.no_register else
            "zero-copy: registered ring, the kernel reads 128-byte header windows and writes back rewritten rows")
    result = {
        "metric": "Mpkt/s full border-router path with frames in host memory (H2D + kernel + D2H), "
                  "mixed 64-1500 B frames",
        "value": round(world * n * steps / total / 1e6, 2), "unit": "Mpkt/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(total / steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (the config-4 frame mix, 2 KiB slots in registered host memory)",
        "config": {"workload": f"config 5: {n} host-resident frames per GPU through hfv_br_process_host",
                   "frames_per_gpu": n, "slot_bytes": BR_SLOT, "path": path,
                   "parallelism": f"batch-sharded x{world}, no collective"},
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 200 (hf), 10 (br), 5 (br-host)")
    ap.add_argument("--warmup", type=int, default=None, help="default 20 (hf), 3 (br), 1 (br-host)")
    ap.add_argument("--n", type=int, default=1 << 20, help="records per GPU (config 2: 2^20); with --strong, in total")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --n records in total, sliced over the ranks on 64-record boundaries")
    ap.add_argument("--keysel", choices=["zero", "ifid"], default="zero")
    ap.add_argument("--big-n", type=int, default=1 << 24, help="HBM-resident run size (0 = skip)")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of multi-thread CPU baseline (0 = skip)")
    ap.add_argument("--no-host-e2e", action="store_true")
    ap.add_argument("--workload", choices=["hf", "br", "br-host"], default="hf",
                    help="hf: hop-field verify on 64 B records (configs 2/3, the headline); br: config 4; "
                         "br-host: config 5")
    ap.add_argument("--mode", choices=["service", "launch"], default="service",
                    help="hf headline: resident service grid (default) or one launch per batch")
    ap.add_argument("--window", type=int, default=256, help="br-host: header bytes per frame moved over PCIe")
    ap.add_argument("--no-register", action="store_true", help="br-host: leave the ring unregistered (DMA windows)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = {"hf": 200, "br": 10, "br-host": 5}[args.workload]
    if args.warmup is None:
        args.warmup = {"hf": 20, "br": 3, "br-host": 1}[args.workload]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.workload == "br":
        return run_br(args, rank, world, local)
    if args.workload == "br-host":
        return run_br_host(args, rank, world, local)
    keysel = hfv.KEYSEL_IFID if args.keysel == "ifid" else hfv.KEYSEL_ZERO
    if args.strong:   # a fixed total, sliced over the ranks (scion_hfv.shard_range)
        first, last = hfv.shard_range(args.n, world, rank)
        n, total = last - first, args.n
    else:             # weak: every rank verifies its own n records
        n, first, total = args.n, rank * args.n, world * args.n

    ctx = make_ctx(local, keysel)
    stream = torch.cuda.current_stream().cuda_stream   # int handle (0 = default stream)
    recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
    ctx.gen_records(recs, n, SEED_RECORDS, first_index=first, stream=stream)
    bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")

    # --- launch path (hfv_verify_records: one launch + table fill per batch) ---------------
    # W warmup steps (at least one untimed pass: the verdicts must be right before anything
    # is timed)
    for _ in range(max(1, args.warmup)):
        ctx.verify_records(recs, n, bits, stream=stream)
    torch.cuda.synchronize()
    assert popcount(bits) == expected_pass_count(n, first), "verify bitmap disagrees with generator truth"
    launch_elapsed = timed_steps(world, args.steps, lambda: ctx.verify_records(recs, n, bits, stream=stream))
    k_mean, k_med = kernel_ms(ctx, recs, n, bits, stream, max(20, min(args.steps, 200)))

    # --- resident service (hfv_service_*: persistent grid, host descriptor ring) ----------
    # The timed region starts the grid, posts the K batches one by one and stops it, so the
    # launch, the table fill and the drain are all inside it.
    bits.zero_()
    torch.cuda.synchronize()
    for _ in range(max(1, args.warmup)):
        ctx.service_submit(recs, n, bits)
    ctx.service_stop()
    assert popcount(bits) == expected_pass_count(n, first), "service bitmap disagrees with generator truth"
    svc = {}

    def service_run():
        ctx.service_start()
        for _ in range(args.steps):
            ctx.service_submit(recs, n, bits)
        svc["grid_ms"] = ctx.service_stop()

    svc_elapsed = timed_steps(world, 1, service_run)
    svc["shader_mhz"] = ctx.service_shader_mhz()   # diagnostics, outside the timed region
    assert popcount(bits) == expected_pass_count(n, first)
    headline = args.mode
    elapsed = svc_elapsed if headline == "service" else launch_elapsed

    bytes_per_launch = hfv.BYTES_PER_PACKET * n
    if headline == "service":
        # the grid's lifetime (dispatch start/stop events) covers all K batches
        grid_s = svc["grid_ms"] * 1e-3
        achieved = bytes_per_launch * args.steps / grid_s / 1e9
        kern = {"kernel": "k_verify_service", "grid_ms": round(svc["grid_ms"], 4),
                "batches_per_grid": args.steps, "kernel_ms_per_batch": round(svc["grid_ms"] / args.steps, 5),
                "algorithmic_bytes_per_grid": int(bytes_per_launch * args.steps)}
    else:
        achieved = bytes_per_launch / (k_mean * 1e-3) / 1e9
        kern = {"kernel": "k_verify_records", "kernel_ms_mean": round(k_mean, 5),
                "kernel_ms_median": round(k_med, 5), "algorithmic_bytes_per_launch": int(bytes_per_launch)}
    per_launch = {"mpkts": round(total * args.steps / launch_elapsed / 1e6, 2),
                  "ms_per_step": round(launch_elapsed / args.steps * 1e3, 5),
                  "kernel_ms_mean": round(k_mean, 5), "kernel_ms_median": round(k_med, 5),
                  "kernel_mpkts": round(n / k_mean / 1e3, 1),
                  "frac": round(bytes_per_launch / (k_mean * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    service = {"mpkts": round(total * args.steps / svc_elapsed / 1e6, 2),
               "ms_per_step": round(svc_elapsed / args.steps * 1e3, 5), "grid_ms": round(svc["grid_ms"], 4),
               "shader_mhz": round(svc["shader_mhz"], 1) if svc["shader_mhz"] else None}

    traffic = pmc_traffic(args.keysel, n, service=headline == "service")

    result = {
        "metric": "Mpkt/s device-resident hop-field AES-CMAC verify, 64 B SCION packets",
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (64 B SCION records, splitmix64 seed 0x5C100001, 1/16 corrupted MACs; generated on device)",
        "config": {"workload": f"config {'3' if keysel else '2'}: "
                               f"{f'{total} x 64 B records in total' if args.strong else f'{n} x 64 B records per GPU'}, "
                               f"{'256 ingress-interface keys (KEYSEL_IFID)' if keysel else 'single AS key'}",
                   "records_per_gpu": n, "record_bytes": 64, "keysel": args.keysel,
                   "parallelism": f"batch-sharded x{world}, no collective"},
        "roofline": dict({"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic}, **kern,
                         variant=ctx.describe(),
                         note="2^20 x 64 B = 64 MiB is Infinity-Cache resident; see hbm_resident"),
        "ceilings": dict(ceilings(args.keysel), **lds_bound_at_clock(args.keysel, svc["shader_mhz"])),
        "path": ("resident service: one persistent grid, the K batches posted one by one through the host "
                 "descriptor ring (hfv_service_submit); grid launch, table fill and drain inside the timed region"
                 if headline == "service" else "one hfv_verify_records launch per batch"),
        "service": service,
        "per_launch": per_launch,
    }

    if rank == 0 and world == 1 and args.big_n:
        nb = args.big_n
        big = torch.empty((nb, 64), dtype=torch.uint8, device="cuda")
        ctx.gen_records(big, nb, SEED_RECORDS, first_index=0, stream=stream)
        bbits = torch.zeros((nb + 63) // 64, dtype=torch.int64, device="cuda")
        for _ in range(3):
            ctx.verify_records(big, nb, bbits, stream=stream)
        torch.cuda.synchronize()
        assert popcount(bbits) == expected_pass_count(nb, 0)
        bm, bmed = kernel_ms(ctx, big, nb, bbits, stream, 20)
        ach = hfv.BYTES_PER_PACKET * nb / (bm * 1e-3) / 1e9
        # the same batch through the resident service, 10 batches per grid
        bbits.zero_()
        ctx.service_start()
        for _ in range(10):
            ctx.service_submit(big, nb, bbits)
        sg = ctx.service_stop()
        smhz = ctx.service_shader_mhz()
        assert popcount(bbits) == expected_pass_count(nb, 0)
        sach = hfv.BYTES_PER_PACKET * nb * 10 / (sg * 1e-3) / 1e9
        result["hbm_resident"] = {"records": nb, "kernel_ms_mean": round(bm, 4), "mpkts": round(nb / bm / 1e3, 1),
                                  "achieved_GBs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                                  "traffic": pmc_traffic(args.keysel, nb),
                                  "service_ms_per_batch": round(sg / 10, 4),
                                  "service_mpkts": round(nb * 10 / sg / 1e3, 1),
                                  "service_frac": round(sach / HBM_PEAK_GBS, 4),
                                  "service_traffic": pmc_traffic(args.keysel, nb, service=True),
                                  "service_shader_mhz": round(smhz, 1) if smhz else None}
        del big, bbits

    if rank == 0 and world == 1 and not args.no_host_e2e:
        hrecs = recs.cpu().numpy()
        hbits = np.zeros((n + 63) // 64, dtype=np.uint64)
        ctx.verify_records_host(hrecs, n, hbits)     # warm the pinned staging
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.verify_records_host(hrecs, n, hbits)
        th = (time.perf_counter() - t0) / reps
        assert np.array_equal(hbits, bits.cpu().numpy().view(np.uint64))
        result["host_e2e"] = {"mpkts": round(n / th / 1e6, 1), "ms_per_batch": round(th * 1e3, 3),
                              "path": "pageable host -> INF/HF gathered into 24 B pinned staging records (host threads) -> H2D -> "
                                      "kernel -> D2H -> host, 2^18-record chunks on 2 streams"}
        # the same batch in a registered (pinned, mapped) ring: the kernel reads the records'
        # INF/HF words across PCIe in place and writes the registered bitmap in place
        ring = hfv.host_array((n, hfv.REC_SIZE), np.uint8)
        ring[:] = hrecs
        rbits = hfv.host_array(((n + 63) // 64,), np.uint64)
        ctx.host_register(ring)
        ctx.host_register(rbits)
        ctx.verify_records_host(ring, n, rbits)
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.verify_records_host(ring, n, rbits)
        tz = (time.perf_counter() - t0) / reps
        assert np.array_equal(rbits, hbits)
        ctx.host_unregister(ring)
        ctx.host_unregister(rbits)
        result["host_e2e_zero_copy"] = {"mpkts": round(n / tz / 1e6, 1), "ms_per_batch": round(tz * 1e3, 3),
                                        "path": "registered host ring read by the kernel over PCIe in place (grid-stride "
                                                "tiles; PCIe moves whole 64 B lines), bitmap written to registered host memory"}

    if rank == 0 and world == 1 and args.cpu_budget > 0:
        result["cpu_baseline"] = cpu_baseline(recs.cpu().numpy(), keysel, bits.cpu().numpy().view(np.uint64),
                                              args.cpu_budget)

    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
