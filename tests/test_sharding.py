"""Multi-GPU partitioning on CPU (gloo, world_size 2): each rank owns a word-aligned slice
of the batch (scion_hfv.shard_range), verifies it, and the concatenated per-rank bitmaps
equal the single-device bitmap.  The per-rank verify here is the CPU checker; the GPU path
shards identically (bench.py, one process per GPU, no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import orc
import scion_hfv as hfv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, keysel, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    raw = orc.gen_key_table(256) if keysel else orc.KEY_1111
    hk, valid = orc.key_table(raw)
    a, b = hfv.shard_range(n, world, rank)
    recs = orc.gen_records(b - a, hk, keysel, first_index=a)        # this rank's slice only
    bits = orc.verify_records(recs, hk, valid, keysel)
    words = (n + 63) // 64
    mine = torch.zeros(words, dtype=torch.int64)
    mine[a // 64:a // 64 + len(bits)] = torch.from_numpy(bits.view(np.int64))
    dist.all_reduce(mine)                                            # disjoint slices: sum = concat
    if rank == 0:
        q.put(mine.numpy().view(np.uint64).copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("n,keysel", [(5000, 0), (4096 + 17, 1)])
def test_two_rank_shards_concatenate(n, keysel):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, keysel, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    raw = orc.gen_key_table(256) if keysel else orc.KEY_1111
    hk, valid = orc.key_table(raw)
    full = orc.verify_records(orc.gen_records(n, hk, keysel), hk, valid, keysel)
    assert np.array_equal(got, full)


def _br_worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import br_fuzz as F
    import br_topo as T
    mac = lambda k, m: orc.cmac(m, k)   # noqa: E731
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    frames, lens, ifidx = F.fuzz_batch(F.hop_inputs(brs, False, mac), "br1", False, n, seed=77, slot=256)
    a, b = hfv.shard_range(n, world, rank)
    act, ver, egr, st = brs["br1"].process(frames[a:b].copy(), lens[a:b], ifidx[a:b])   # this rank's frames
    out = torch.zeros((n, 6), dtype=torch.int64)
    out[a:b, 0], out[a:b, 1], out[a:b, 2] = torch.from_numpy(act.astype(np.int64)), \
        torch.from_numpy(ver.astype(np.int64)), torch.from_numpy(egr.astype(np.int64))
    stats = torch.from_numpy(st.view(np.int64).copy())
    dist.all_reduce(out)        # disjoint slices
    dist.all_reduce(stats)      # per-GPU verdict counters merge by summation (like per-CPU maps)
    if rank == 0:
        q.put((out.numpy().copy(), stats.numpy().view(np.uint64).copy()))
    dist.destroy_process_group()


def test_two_rank_router_shards():
    """Config 4 sharded over 2 ranks: per-frame results concatenate and the verdict counters
    of the ranks sum to the single-device counters."""
    import br_fuzz as F
    import br_topo as T
    n = 3001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_br_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    out, stats = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mac = lambda k, m: orc.cmac(m, k)   # noqa: E731
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    frames, lens, ifidx = F.fuzz_batch(F.hop_inputs(brs, False, mac), "br1", False, n, seed=77, slot=256)
    act, ver, egr, st = brs["br1"].process(frames, lens, ifidx)
    assert (out[:, 0] == act).all() and (out[:, 1] == ver).all() and (out[:, 2] == egr).all()
    assert (stats == st).all()
