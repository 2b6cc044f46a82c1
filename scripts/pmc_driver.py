#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc passes: verify 2^20 and 2^24 records (config 2, and config 3
with --keysel ifid), `reps` launches each, after one untimed generation pass.  With a 4th
argument `bat` every size's `reps` batches go through one hfv_verify_batches call (twice; the
first is dropped as the warm-up).  With a 4th argument `svc` the batches go through the resident service instead: per size one 2-batch
grid (dropped by pmc_summary.py as the warm-up) and one grid of `reps` batches (`svcrun`: the
same grids through hfv_service_run, every batch in the kernel arguments).  With a 5th
argument `rotR` each size is held in R resident batches and batch k of a grid verifies
batch k % R, exactly as bench.py's headline does (R x 64 MiB > the Infinity Cache)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
from bench import KEY_1111, SEED_RECORDS, key_table_256  # noqa: E402


def run_br(reps, n=1 << 20, one=False):
    """Config 4: the bench frame mix through hfv_br_process, reps launches on fresh copies
    (one=True, `br1t`: every frame the bench mix's first template -- no divergence)."""
    from bench import BR_SLOT, br_batch
    from scion_hfv import topology as TP
    torch.cuda.set_device(0)
    ctx = hfv.Ctx(0)
    ctx.key_add(0, TP.KEYS[1])
    ctx.br_set_config(TP.br_config("br1"))
    tmpl, tid, lens, ifidx, _ = br_batch(n, 0)
    if one:
        tid[:], lens[:], ifidx[:] = tid[0], lens[0], ifidx[0]
    master = torch.from_numpy(tmpl).cuda()[torch.from_numpy(tid.astype("int64")).cuda()]
    d_len = torch.from_numpy(lens.view("int16")).cuda()
    d_if = torch.from_numpy(ifidx.view("int32")).cuda()
    act = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ver = torch.zeros_like(act)
    egr = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(64 * 2 * 11, dtype=torch.int64, device="cuda")
    work = torch.empty_like(master)
    for _ in range(reps + 1):
        work.copy_(master)
        ctx.br_process(work, BR_SLOT, d_len, d_if, n, act, ver, egr, st)
    torch.cuda.synchronize()
    ctx.close()


def main():
    keysel = sys.argv[1] if len(sys.argv) > 1 else "zero"
    if keysel in ("br", "br1t"):
        return run_br(int(sys.argv[2]) if len(sys.argv) > 2 else 10, one=keysel == "br1t")
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    sizes = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1048576,16777216").split(",")]
    svc = len(sys.argv) > 4 and sys.argv[4] in ("svc", "svcrun")
    bat = len(sys.argv) > 4 and sys.argv[4] == "bat"   # hfv_verify_batches: `reps` batches in one call
    run = len(sys.argv) > 4 and sys.argv[4] == "svcrun"   # the batches inline (hfv_service_run)
    rot = int(sys.argv[5][3:]) if len(sys.argv) > 5 and sys.argv[5].startswith("rot") else 1
    torch.cuda.set_device(0)
    ctx = hfv.Ctx(0)
    if keysel == "ifid":
        ctx.key_add_batch(0, key_table_256())
        ctx.set_keysel(hfv.KEYSEL_IFID)
    else:
        ctx.key_add(0, KEY_1111)
    for n in sizes:
        R = rot if n <= (1 << 20) else 1
        recs = [torch.empty((n, 64), dtype=torch.uint8, device="cuda") for _ in range(R)]
        bits = [torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda") for _ in range(max(R, reps, 2))]
        for i, r in enumerate(recs):   # consecutive generator dispatches = one size group (pmc_summary.py)
            ctx.gen_records(r, n, SEED_RECORDS, first_index=i * n)
        if bat:   # two calls of `reps` batches: the first is dropped by pmc_summary.py as the warm-up
            for _ in range(2):
                ctx.verify_batches([(recs[j % R], n, bits[j]) for j in range(reps)])
                torch.cuda.synchronize()
                print(f"batches n={n} reps={reps} shader_mhz={ctx.batches_shader_mhz()}", flush=True)
        elif svc:
            torch.cuda.synchronize()
            for k in (2, reps):
                if run:
                    ctx.service_run([(recs[j % R], n, bits[j]) for j in range(k)])
                    continue
                ctx.service_start()
                ctx.service_submitv([(recs[j % R], n, bits[j]) for j in range(k)])
                ctx.service_stop()
        else:
            for j in range(reps):
                ctx.verify_records(recs[j % R], n, bits[j])
        torch.cuda.synchronize()
        del recs, bits
    ctx.close()


if __name__ == "__main__":
    main()
