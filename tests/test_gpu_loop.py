"""Config 5 in one process on the GPU: hfv_loop_run (producer threads -> registered RX ring ->
hfv_br_process_host zero-copy -> TX/drop consumers) against the oracle router over the same
frame sequence: packet, byte and verdict counts exact, and the sum of per-frame digests of
every transmitted (rewritten) frame with its egress port equal to the oracle's."""
import numpy as np
import pytest

import orc
import scion_hfv as hfv
from conftest import rerun_on_test_build
from scion_hfv import evaluation as E

pytestmark = pytest.mark.gpu
SLOT = 192
HOP1_MAC = 78 + 4 + 8 + 12 + 6   # path at 78: meta, info field, hop 0, then hop 1 flags..egress


def _frame_mix(n, bad_every=0):
    f = E.frames(n)
    if bad_every:
        f[::bad_every, HOP1_MAC] ^= 0x5A
    return f


def _oracle(frames, total, hf_check=True):
    """(rx, tx, tx_bytes, drop, digest, verdict counts) of the oracle router over the cyclic
    sequence the producers push."""
    n = frames.shape[0]
    slots = np.zeros((n, SLOT), dtype=np.uint8)
    slots[:, :frames.shape[1]] = frames
    lens = np.full(n, frames.shape[1], dtype=np.uint16)
    a, v, e, _ = orc.br_process(slots, lens, np.full(n, E.RX_IFINDEX, dtype=np.uint32), E.br_config()[0],
                                orc.hop_key(E.KEYS[1]), hf_check=hf_check)
    reps = np.bincount(np.arange(total) % n, minlength=n).astype(np.uint64)
    tx = a == 4
    M = (1 << 64) - 1
    digest = 0
    for i in np.nonzero(tx)[0]:
        digest = (digest + int(reps[i]) * hfv.loop_frame_digest(bytes(slots[i, :lens[i]]), int(e[i]))) & M
    verdicts = np.zeros(hfv.BR_COUNTERS, dtype=np.uint64)
    np.add.at(verdicts, v >> 3, reps)
    return {"rx": total, "tx": int(reps[tx].sum()), "tx_bytes": int((reps * lens)[tx].sum()),
            "drop": int(reps[~tx].sum()), "tx_digest": digest, "verdicts": [int(x) for x in verdicts]}


@pytest.mark.parametrize("dma", [0, 1, 2], ids=["zero_copy", "dma", "dma_in_zc_out"])
@pytest.mark.parametrize("hf_check", [True, False], ids=["hf_check", "hf_check_off"])
def test_loop_matches_oracle(gpu_ctx, hf_check, dma):
    frames = _frame_mix(97, bad_every=5)
    E.setup_ctx(gpu_ctx, hf_check=hf_check)
    total = 10007
    stats = np.zeros((hfv.BR_STATS_IFINDEX, 2, hfv.BR_COUNTERS), dtype=np.uint64)
    got = gpu_ctx.loop_run(frames, np.full(97, E.FRAME_LEN), total, rx_ifindex=E.RX_IFINDEX, slot=SLOT,
                           chunk=1000, chunks=3, producers=2, consumers=3, digest=True, stats=stats, dma=dma)
    want = _oracle(frames, total, hf_check)
    for k in want:
        assert got[k] == want[k], k
    assert (got["drop"] > 0) == hf_check
    # the kernel's per-ingress verdict counters (hfv_br_process_host's stats) agree with the consumers
    assert [int(x) for x in stats[E.RX_IFINDEX, 1]] == want["verdicts"]
    assert int(stats[E.RX_IFINDEX, 0].sum()) == total * E.FRAME_LEN


@pytest.mark.parametrize("dma", [0, 2], ids=["zero_copy", "dma_in_zc_out"])
def test_loop_publish_races_second_stream(request, gpu_ctx, dma):
    """The round-2 failure made deterministic: the table publish the loop's first chunk does on
    its stream is held 3 ms behind a spin kernel (hfv_debug_publish_delay), so chunk 1 on the
    loop's second stream launches while the copy of the new key and tables is still queued.
    It must wait for that copy (the publish fence); without it every MAC of chunk 1 fails
    against the stale key and tx falls short by one chunk (gpurun_out/r02c5)."""
    if rerun_on_test_build(request):   # uses a test hook: runs on lib/libscionhfv_test.so
        return
    import torch
    recs = torch.zeros((64, 64), dtype=torch.uint8, device="cuda:0")
    bits = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    frames = _frame_mix(97, bad_every=5)
    want = _oracle(frames, 10007, True)
    for wrong in (bytes(16), bytes(range(16))):   # both device tables: a wrong slot-0 key
        gpu_ctx.key_add(0, wrong)
        gpu_ctx.verify_records(recs, 64, bits)
        torch.cuda.synchronize()
    E.setup_ctx(gpu_ctx, hf_check=True)
    hfv.Ctx.debug_publish_delay(3000)
    try:
        got = gpu_ctx.loop_run(frames, np.full(97, E.FRAME_LEN), 10007, rx_ifindex=E.RX_IFINDEX, slot=SLOT,
                               chunk=1000, chunks=3, producers=2, consumers=3, digest=True, dma=dma)
    finally:
        hfv.Ctx.debug_publish_delay(0)
    for k in want:
        assert got[k] == want[k], k


@pytest.mark.parametrize("dma", [0, 2], ids=["zero_copy", "dma_in_zc_out"])
def test_loop_single_block_chunks(request, gpu_ctx, dma):
    """The round-2 failing shape, forced: each 1000-frame chunk runs as ONE 1024-thread block
    whose 16 waves are all active (hfv_debug_br_grid(1)), zero-copy on the mapped ring, fresh
    router tables and key published by the loop's first chunk (the loop's other streams must
    wait for that publish).  Repeated so chunk 1 races the publish more than once."""
    if rerun_on_test_build(request):   # uses a test hook: runs on lib/libscionhfv_test.so
        return
    frames = _frame_mix(97, bad_every=5)
    stats = np.zeros((hfv.BR_STATS_IFINDEX, 2, hfv.BR_COUNTERS), dtype=np.uint64)
    want = _oracle(frames, 10007, True)
    import torch
    recs = torch.zeros((64, 64), dtype=torch.uint8, device="cuda:0")
    bits = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    hfv.Ctx.debug_br_grid(1)
    try:
        for rep in range(3):
            # both device tables get a wrong slot-0 key first (one publish each), so a launch
            # reading a stale table fails every MAC
            for wrong in (bytes(16), bytes(range(16))):
                gpu_ctx.key_add(0, wrong)
                gpu_ctx.verify_records(recs, 64, bits)
                torch.cuda.synchronize()
            E.setup_ctx(gpu_ctx, hf_check=True)
            stats[:] = 0
            got = gpu_ctx.loop_run(frames, np.full(97, E.FRAME_LEN), 10007, rx_ifindex=E.RX_IFINDEX, slot=SLOT,
                                   chunk=1000, chunks=3, producers=2, consumers=3, digest=True, stats=stats,
                                   dma=dma)
            for k in want:
                assert got[k] == want[k], (rep, k)
            assert [int(x) for x in stats[E.RX_IFINDEX, 1]] == want["verdicts"]
    finally:
        hfv.Ctx.debug_br_grid(0)


def test_loop_more_threads_than_ring_chunks(gpu_ctx):
    """Producers and consumers outnumber the ring's chunks (chunks k and k + chunks share a slot
    and belong to different threads), three chunks in flight on the GPU."""
    frames = _frame_mix(31, bad_every=4)
    E.setup_ctx(gpu_ctx)
    got = gpu_ctx.loop_run(frames, np.full(31, E.FRAME_LEN), 20000, rx_ifindex=E.RX_IFINDEX, slot=144, chunk=500,
                           chunks=3, producers=5, consumers=4, digest=True, inflight=3, dma=True)
    want = _oracle(frames, 20000)
    assert {k: got[k] for k in want} == want


def test_loop_single_producer_ragged_tail(gpu_ctx):
    """One producer/consumer, total smaller than one chunk and not a multiple of n_frames."""
    frames = _frame_mix(7)
    E.setup_ctx(gpu_ctx)
    got = gpu_ctx.loop_run(frames, np.full(7, E.FRAME_LEN), 45, rx_ifindex=E.RX_IFINDEX, slot=SLOT, chunk=64,
                           chunks=2, producers=1, consumers=1, digest=True, inflight=1)
    want = _oracle(frames, 45)
    assert {k: got[k] for k in want} == want


def test_loop_rejects_bad_geometry(gpu_ctx):
    frames = _frame_mix(2)
    for kw in ({"slot": 136}, {"slot": 112}, {"slot": 128}, {"chunks": 1}, {"chunk": 0}, {"dma": 3}, {"dma": -1}):
        args = dict(rx_ifindex=E.RX_IFINDEX, slot=SLOT, chunk=16, chunks=2)
        args.update(kw)
        with pytest.raises(hfv.HfvError):
            gpu_ctx.loop_run(frames, np.full(2, E.FRAME_LEN), 10, **args)


@pytest.mark.parametrize("dma", [0, 1, 2], ids=["zero_copy", "dma", "dma_in_zc_out"])
def test_loop_ptf_mix_ipv4_ipv6(gpu_ctx, dma):
    """The loop over the config-4 frame mix (the reference test topology's BR 1: IPv4 and IPv6
    underlays, AS ingress, sibling hand-over, segment switch, corrupted MACs), frames of mixed
    length in 256-byte slots, several ingress interfaces: counts and transmitted-frame digests
    equal the oracle router's."""
    import br_topo as T
    sys_path_bench()
    import bench
    frames, ifis, good, _ = bench.br_templates()
    n = len(frames)
    stride = 256
    buf = np.zeros((n, stride), dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint16)
    for i, f in enumerate(frames):
        buf[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
        lens[i] = len(f)
    assert lens.max() <= stride
    # the loop takes one ingress ifindex per run: run it once per ingress interface of the mix
    cfg = T.br_config("br1")
    for ifx in sorted(set(ifis)):
        sel = np.array([i for i in range(n) if ifis[i] == ifx])
        gpu_ctx.br_set_config(cfg)
        gpu_ctx.key_add(0, T.KEYS[1])
        gpu_ctx.br_set_hf_check(True)
        total = 5 * len(sel) + 3
        got = gpu_ctx.loop_run(buf[sel], lens[sel], total, rx_ifindex=int(ifx), slot=stride, chunk=7, chunks=3,
                               producers=2, consumers=2, digest=True, dma=dma)
        slots = buf[sel].copy()
        a, v, e, _ = orc.br_process(slots, lens[sel], np.full(len(sel), ifx, dtype=np.uint32), cfg,
                                    orc.hop_key(T.KEYS[1]))
        reps = np.bincount(np.arange(total) % len(sel), minlength=len(sel)).astype(np.uint64)
        tx = a == 4
        digest = 0
        for i in np.nonzero(tx)[0]:
            digest = (digest + int(reps[i]) * hfv.loop_frame_digest(bytes(slots[i, :lens[sel][i]]), int(e[i]))) % 2**64
        assert got["rx"] == total and got["tx"] == int(reps[tx].sum()), ifx
        assert got["tx_digest"] == digest, ifx
        assert got["drop"] == int(reps[~tx].sum())


def sys_path_bench():
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
