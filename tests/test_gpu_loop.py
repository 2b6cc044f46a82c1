"""Config 5 in one process on the GPU: hfv_loop_run (producer threads -> registered RX ring ->
hfv_br_process_host zero-copy -> TX/drop consumers) against the oracle router over the same
frame sequence: packet, byte and verdict counts exact, and the sum of per-frame digests of
every transmitted (rewritten) frame with its egress port equal to the oracle's."""
import numpy as np
import pytest

import orc
import scion_hfv as hfv
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


@pytest.mark.parametrize("dma", [False, True], ids=["zero_copy", "dma"])
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
    for kw in ({"slot": 136}, {"slot": 112}, {"slot": 128}, {"chunks": 1}, {"chunk": 0}):
        args = dict(rx_ifindex=E.RX_IFINDEX, slot=SLOT, chunk=16, chunks=2)
        args.update(kw)
        with pytest.raises(hfv.HfvError):
            gpu_ctx.loop_run(frames, np.full(2, E.FRAME_LEN), 10, **args)
