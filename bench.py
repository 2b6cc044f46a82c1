#!/usr/bin/env python3
"""Headline benchmark: Mpkt/s of device-resident hop-field AES-CMAC verify on 64 B SCION
records (BASELINE.json metric; config 2 = 2^20 records, single AS key, per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keysel zero|ifid] [--n N]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One process per GPU.  A "step" is one hfv_verify_records launch over the rank's resident
batch of n records (weak scaling: every rank verifies its own n records, no collective on
the data path; RCCL is used only for the timing barrier and max-over-ranks).  Rank 0
prints one JSON line.  Besides the contract fields it carries:
  roofline      -- the verify kernel's algorithmic bytes (64 B read + 1/8 B verdict per
                   record) per launch / its mean launch duration (HIP events on the launch
                   stream), against the 8 TB/s HBM3E peak; `traffic` is the PMC-measured HBM
                   bytes per launch from profiles/ when a matching pass exists.
  cpu_baseline  -- the reference's own aes.c soft path (oracle/_ref, built from
                   /root/reference) over a sample of the same records on this host's cores,
                   verdicts cross-checked against the GPU bitmap.
  hbm_resident  -- the same kernel on 2^24 records (1 GiB > 256 MiB Infinity Cache).
  host_e2e      -- rate including H2D/D2H through pinned staging (hfv_verify_records_host).
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


def pmc_traffic(keysel, n):
    """HBM bytes per launch measured by rocprofv3 PMC passes (scripts/pmc_round.sh) for this
    exact configuration, committed in profiles/traffic.json; None if not measured."""
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        return json.load(open(tpath))[f"{keysel}:{n}"]["hbm_bytes_per_launch"]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 20, help="records per GPU (config 2: 2^20)")
    ap.add_argument("--keysel", choices=["zero", "ifid"], default="zero")
    ap.add_argument("--big-n", type=int, default=1 << 24, help="HBM-resident run size (0 = skip)")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of multi-thread CPU baseline (0 = skip)")
    ap.add_argument("--no-host-e2e", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    keysel = hfv.KEYSEL_IFID if args.keysel == "ifid" else hfv.KEYSEL_ZERO
    n = args.n

    ctx = make_ctx(local, keysel)
    stream = torch.cuda.current_stream().cuda_stream   # int handle (0 = default stream)
    recs = torch.empty((n, 64), dtype=torch.uint8, device="cuda")
    ctx.gen_records(recs, n, SEED_RECORDS, first_index=rank * n, stream=stream)
    bits = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")

    for _ in range(args.warmup):
        ctx.verify_records(recs, n, bits, stream=stream)
    torch.cuda.synchronize()
    # the verdicts must be right before anything is timed
    assert popcount(bits) == expected_pass_count(n, rank * n), "verify bitmap disagrees with generator truth"

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.verify_records(recs, n, bits, stream=stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    k_mean, k_med = kernel_ms(ctx, recs, n, bits, stream, max(20, min(args.steps, 200)))
    bytes_per_launch = hfv.BYTES_PER_PACKET * n
    achieved = bytes_per_launch / (k_mean * 1e-3) / 1e9

    traffic = pmc_traffic(args.keysel, n)

    result = {
        "metric": "Mpkt/s device-resident hop-field AES-CMAC verify, 64 B SCION packets",
        "value": round(world * n * args.steps / elapsed / 1e6, 2),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (64 B SCION records, splitmix64 seed 0x5C100001, 1/16 corrupted MACs; generated on device)",
        "config": {"workload": f"config {'3' if keysel else '2'}: {n} x 64 B records per GPU, "
                               f"{'256 ingress-interface keys (KEYSEL_IFID)' if keysel else 'single AS key'}",
                   "records_per_gpu": n, "record_bytes": 64, "keysel": args.keysel,
                   "parallelism": f"batch-sharded x{world}, no collective"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "k_verify_records", "variant": ctx.describe(), "kernel_ms_mean": round(k_mean, 5),
                     "kernel_ms_median": round(k_med, 5),
                     "algorithmic_bytes_per_launch": int(bytes_per_launch),
                     "note": f"2^20 x 64 B = 64 MiB is Infinity-Cache resident; see hbm_resident"},
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
        result["hbm_resident"] = {"records": nb, "kernel_ms_mean": round(bm, 4), "mpkts": round(nb / bm / 1e3, 1),
                                  "achieved_GBs": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                                  "traffic": pmc_traffic(args.keysel, nb)}
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
                              "path": "pageable host -> pinned -> H2D -> kernel -> D2H -> host, 2 streams"}

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
