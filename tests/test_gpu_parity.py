"""Parity of the MI355X kernels (through the C ABI) against the CPU checker and the
committed reference fixtures.  Integer work: every comparison is bit-exact."""
import os

import numpy as np
import pytest

import orc
import scion_hfv as hfv

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def dev(a):
    return torch.from_numpy(np.array(a, copy=True)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def new_bits(n):
    return torch.zeros(max(1, (n + 63) // 64), dtype=torch.int64, device=DEV)


def bits_np(t, n):
    return host(t).view(np.uint64)[: (n + 63) // 64]


def install(ctx, raw_keys, nkeys=256):
    for k in range(nkeys):
        ctx.key_add(k, raw_keys[16 * k:16 * k + 16])


@pytest.fixture()
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = hfv.Ctx(0)
    yield c
    c.synchronize()
    c.close()


@pytest.mark.parametrize("name,keysel", [("hf_single.npz", 0), ("hf_ifid256.npz", 1)])
def test_golden_tags_and_verdicts(ctx, name, keysel):
    g = orc.load_golden(name)
    n = len(g["records"])
    install(ctx, g["raw_keys"].reshape(-1).tobytes(), int(g["nkeys"]))
    ctx.set_keysel(keysel)
    # full 16-byte tags (parity mode) against the reference's aes_cmac
    tags = torch.zeros((n, 16), dtype=torch.uint8, device=DEV)
    kidx = dev(g["key_index"]) if keysel else None
    ctx.cmac_tags(dev(g["macinputs"]), n, tags, key_index=kidx)
    assert np.array_equal(host(tags), g["tags"])
    # fused record verify
    bits = new_bits(n)
    ctx.verify_records(dev(g["records"]), n, bits)
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])
    # verify_hop_field form: macinput + expected 48-bit MAC
    expected = np.frombuffer(np.pad(g["records"][:, 54:60], ((0, 0), (0, 2))).tobytes(), dtype=np.uint64)
    bits2 = new_bits(n)
    ctx.verify_macinputs(dev(g["macinputs"]), dev(expected), n, bits2, key_index=kidx)
    assert np.array_equal(bits_np(bits2, n), g["pass_bits"])


@pytest.mark.parametrize("keysel", [0, 1])
def test_random_records_vs_oracle(ctx, keysel):
    rng = np.random.default_rng(11 + keysel)
    raw = orc.gen_key_table(256)
    hk, valid = orc.key_table(raw)
    install(ctx, raw)
    ctx.set_keysel(keysel)
    recs = orc.gen_records(20000, hk, keysel, seed=99)
    # sprinkle fully random records (garbage flags, IFIDs 0 and >255) between valid ones
    junk = rng.random(len(recs)) < 0.2
    recs[junk] = rng.integers(0, 256, size=(int(junk.sum()), 64), dtype=np.uint8)
    d = dev(recs)
    for n in (1, 2, 63, 64, 65, 127, 4097, 20000):
        bits = new_bits(n)
        ctx.verify_records(d, n, bits)
        want = orc.verify_records(recs[:n], hk, valid, keysel)
        assert np.array_equal(bits_np(bits, n), want), n


def test_strides_and_layouts(ctx):
    raw = orc.KEY_1111
    hk, valid = orc.key_table(raw)
    ctx.key_add(0, raw)
    base = orc.gen_records(3000, hk, 0, seed=5)
    want = orc.verify_records(base, hk, valid, 0)
    for stride in (64, 72, 128, 200):
        recs = np.zeros((3000, stride), dtype=np.uint8)
        recs[:, :64] = base
        bits = new_bits(3000)
        ctx.verify_records(dev(recs), 3000, bits, stride=stride)
        assert np.array_equal(bits_np(bits, 3000), want), stride
    # a compact layout: INF at 0, HF at 8, 24-byte stride
    ctx.set_record_layout(0, 8)
    compact = np.zeros((3000, 24), dtype=np.uint8)
    compact[:, 0:8] = base[:, 40:48]
    compact[:, 8:20] = base[:, 48:60]
    bits = new_bits(3000)
    ctx.verify_records(dev(compact), 3000, bits, stride=24)
    assert np.array_equal(bits_np(bits, 3000), want)
    ctx.set_record_layout(40, 48)


def test_key_remove_add_fail_closed(ctx):
    g = orc.load_golden("hf_single.npz")
    n = len(g["records"])
    d = dev(g["records"])
    bits = new_bits(n)
    ctx.verify_records(d, n, bits)              # no key installed yet
    assert not bits_np(bits, n).any()
    ctx.key_add_b64(0, "MTExMTExMTExMTExMTExMQ==")  # br/test/run_tests:113
    ctx.verify_records(d, n, bits)
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])
    ctx.key_remove(0)
    ctx.verify_records(d, n, bits)
    assert not bits_np(bits, n).any()
    with pytest.raises(hfv.HfvError):
        ctx.key_remove(0)                        # erase of a missing element fails
    with pytest.raises(hfv.HfvError):
        ctx.key_add(256, orc.KEY_1111)
    ctx.key_set_hop_key(0, g["hop_keys"][0].tobytes())
    assert ctx.key_get(0) == g["hop_keys"][0].tobytes()
    ctx.verify_records(d, n, bits)
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])


def test_key_update_is_stream_ordered(ctx):
    """Batches enqueued before a key change keep the old table (RCU-like)."""
    g = orc.load_golden("hf_single.npz")
    n = len(g["records"])
    d = dev(g["records"])
    ctx.key_add(0, orc.KEY_1111)
    s = torch.cuda.Stream()
    outs = [new_bits(n) for _ in range(3)]
    torch.cuda.synchronize()
    ctx.verify_records(d, n, outs[0], stream=s)
    ctx.key_remove(0)
    ctx.verify_records(d, n, outs[1], stream=s)
    ctx.key_add(0, orc.KEY_1111)
    ctx.verify_records(d, n, outs[2], stream=s)
    s.synchronize()
    assert np.array_equal(bits_np(outs[0], n), g["pass_bits"])
    assert not bits_np(outs[1], n).any()
    assert np.array_equal(bits_np(outs[2], n), g["pass_bits"])


def test_key_publish_visible_on_other_streams(ctx):
    """A table published by a launch on stream A, its copy queued behind earlier work on A, is
    the table a launch on stream B then reads: B waits for A's publish copy.  Round 2 had no
    such fence; the config-5 loop published on its chunk-0 stream and its chunk-1 kernel, on a
    second stream, could read the previous table (loop parity failure)."""
    g = orc.load_golden("hf_single.npz")
    n = len(g["records"])
    d = dev(g["records"])
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    scratch = new_bits(n)
    # two publishes of wrong keys: both device tables hold a key that fails these records
    for wrong in (bytes(16), bytes(range(16))):
        ctx.key_add(0, wrong)
        ctx.verify_records(d, n, scratch, stream=a)
        torch.cuda.synchronize()
        assert not bits_np(scratch, n).any() or not np.array_equal(bits_np(scratch, n), g["pass_bits"])
    ctx.key_add(0, orc.KEY_1111)
    outs = [new_bits(n) for _ in range(3)]
    torch.cuda.synchronize()
    with torch.cuda.stream(a):
        torch.cuda._sleep(20_000_000)   # stream A busy for milliseconds before the publish copy
    ctx.verify_records(d, n, outs[0], stream=a)    # publishes: copy queued on A behind the sleep
    ctx.verify_records(d, n, outs[1], stream=b)    # must not run before that copy lands
    ctx.verify_records(d, n, outs[2], stream=0)    # nor on HIP's default stream
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(bits_np(o, n), g["pass_bits"])


def test_partial_key_table_ifid(ctx):
    g = orc.load_golden("hf_ifid256.npz")
    n = len(g["records"])
    raw = g["raw_keys"].reshape(-1).tobytes()
    install(ctx, raw)
    for k in range(0, 256, 3):
        ctx.key_remove(k)
    ctx.set_keysel(1)
    bits = new_bits(n)
    ctx.verify_records(dev(g["records"]), n, bits)
    valid = g["valid"].copy()
    for k in range(0, 256, 3):
        valid[k >> 5] &= np.uint32(~(1 << (k & 31)) & 0xFFFFFFFF)
    want = orc.verify_records(g["records"], g["hop_keys"].reshape(-1), valid, 1)
    assert np.array_equal(bits_np(bits, n), want)


@pytest.mark.parametrize("keysel", [0, 1])
def test_generator_matches_oracle(ctx, keysel):
    raw = orc.gen_key_table(256) if keysel else orc.KEY_1111
    hk, _ = orc.key_table(raw)
    install(ctx, raw, len(raw) // 16)
    ctx.set_keysel(keysel)
    for first in (0, 123456789):
        n = 5000
        recs = torch.zeros((n, 64), dtype=torch.uint8, device=DEV)
        ctx.gen_records(recs, n, orc.SEED_RECORDS, first_index=first)
        want = orc.gen_records(n, hk, keysel, first_index=first)
        assert np.array_equal(host(recs), want)


def test_device_key_expansion(ctx):
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 256, size=(1000, 16), dtype=np.uint8)
    out = torch.zeros((1000, 192), dtype=torch.uint8, device=DEV)
    ctx.expand_keys(dev(keys), 1000, out)
    got = host(out)
    for i in range(1000):
        assert got[i].tobytes() == orc.hop_key(keys[i].tobytes()), i
    # bulk install through the device expansion, then verify the 256-key fixture
    g = orc.load_golden("hf_ifid256.npz")
    ctx.key_add_batch(0, g["raw_keys"].reshape(-1).tobytes())
    for k in (0, 1, 77, 255):
        assert ctx.key_get(k) == g["hop_keys"][k].tobytes()
    ctx.set_keysel(1)
    n = len(g["records"])
    bits = new_bits(n)
    ctx.verify_records(dev(g["records"]), n, bits)
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])


@pytest.mark.parametrize("n", [1 << 20, 1 << 24])
def test_full_size_properties(ctx, n):
    """At BASELINE sizes: verdicts equal the generator's truth (uncorrupted <=> pass), and a
    random sample re-verified by the oracle agrees."""
    ctx.key_add(0, orc.KEY_1111)
    recs = torch.empty((n, 64), dtype=torch.uint8, device=DEV)
    ctx.gen_records(recs, n, orc.SEED_RECORDS)
    bits = new_bits(n)
    ctx.verify_records(recs, n, bits)
    got = hfv.bits_to_bool(bits_np(bits, n), n)
    truth = orc.expected_pass_rule(n)
    assert np.array_equal(got, truth)
    idx = np.sort(np.random.default_rng(1).choice(n, 4096, replace=False))
    sample = recs[torch.from_numpy(idx).to(DEV)].cpu().numpy()
    hk, valid = orc.key_table(orc.KEY_1111)
    want = hfv.bits_to_bool(orc.verify_records(sample, hk, valid, 0), 4096)
    assert np.array_equal(got[idx], want)
    # idempotence: a second pass over the same batch gives the same bitmap
    bits2 = new_bits(n)
    ctx.verify_records(recs, n, bits2)
    assert torch.equal(bits, bits2)
    del recs


@pytest.mark.parametrize("service", [False, True], ids=["launch", "service"])
def test_full_size_properties_ifid(ctx, service):
    """Config 3 at its BASELINE size (2^20 records, 256 ingress-interface keys, KEYSEL_IFID):
    verdicts equal the generator's truth, an oracle-verified sample agrees, and the launch and
    the resident-service paths give the same bitmap."""
    n = 1 << 20
    raw = orc.gen_key_table(256)
    hk, valid = orc.key_table(raw)
    install(ctx, raw)
    ctx.set_keysel(1)
    recs = torch.empty((n, 64), dtype=torch.uint8, device=DEV)
    ctx.gen_records(recs, n, orc.SEED_RECORDS)
    bits = new_bits(n)
    if service:
        t = ctx.service_submit(recs, n, bits)
        ctx.service_wait(t, 10000)
        ctx.service_stop()
    else:
        ctx.verify_records(recs, n, bits)
    torch.cuda.synchronize()
    got = hfv.bits_to_bool(bits_np(bits, n), n)
    assert np.array_equal(got, orc.expected_pass_rule(n))
    idx = np.sort(np.random.default_rng(3).choice(n, 4096, replace=False))
    sample = recs[torch.from_numpy(idx).to(DEV)].cpu().numpy()
    want = hfv.bits_to_bool(orc.verify_records(sample, hk, valid, 1), 4096)
    assert np.array_equal(got[idx], want)
    # the IFIDs really spread over the key table (not one slot)
    ifids = np.where(sample[:, 40] & 1, sample[:, 51], sample[:, 53])   # Cons ? ConsIngress : ConsEgress (big-endian low byte)
    assert len(np.unique(ifids)) > 200
    del recs


def test_host_path_matches_device(ctx):
    ctx.key_add(0, orc.KEY_1111)
    n = (1 << 21) + 777   # 8 full 2^18-record staging chunks and a ragged ninth
    recs = torch.empty((n, 64), dtype=torch.uint8, device=DEV)
    ctx.gen_records(recs, n, orc.SEED_RECORDS)
    dbits = new_bits(n)
    ctx.verify_records(recs, n, dbits)
    hrecs = recs.cpu().numpy()
    hbits = np.zeros((n + 63) // 64, dtype=np.uint64)
    ctx.verify_records_host(hrecs, n, hbits)
    assert np.array_equal(hbits, bits_np(dbits, n))
    # a wider stride: the host threads gather INF/HF from 128-byte slots
    m = 300001
    wide = np.zeros((m, 128), dtype=np.uint8)
    wide[:, :64] = hrecs[:m]
    wbits = np.zeros((m + 63) // 64, dtype=np.uint64)
    ctx.verify_records_host(wide, m, wbits, stride=128)
    want = bits_np(dbits, n)[: (m + 63) // 64].copy()
    want[-1] &= np.uint64((1 << (m % 64)) - 1) if m % 64 else np.uint64(~0)
    assert np.array_equal(wbits, want)


def test_host_zero_copy_ring(ctx):
    """Records in a registered host ring are verified in place (zero-copy), with the bitmap
    either registered (written in place) or pageable (copied back); both equal the device
    path, also for a ragged count and a record range that starts inside the ring."""
    ctx.key_add(0, orc.KEY_1111)
    n = 100_003
    recs = torch.empty((n, 64), dtype=torch.uint8, device=DEV)
    ctx.gen_records(recs, n, orc.SEED_RECORDS)
    dbits = new_bits(n)
    ctx.verify_records(recs, n, dbits)
    want = bits_np(dbits, n)
    ring = hfv.host_array((n, 64), np.uint8)
    ring[:] = recs.cpu().numpy()
    rbits = hfv.host_array(((n + 63) // 64,), np.uint64)
    ctx.host_register(ring)
    ctx.host_register(rbits)
    try:
        ctx.verify_records_host(ring, n, rbits)
        assert np.array_equal(rbits, want)
        pbits = np.zeros_like(want)
        ctx.verify_records_host(ring, n, pbits)
        assert np.array_equal(pbits, want)
        sub = ring[333:]                         # a window starting inside the ring
        m = len(sub)
        sbits = np.zeros((m + 63) // 64, dtype=np.uint64)
        ctx.verify_records_host(sub, m, sbits)
        dsub = new_bits(m)
        ctx.verify_records(recs[333:], m, dsub)
        assert np.array_equal(sbits, bits_np(dsub, m))
        hk, valid = orc.key_table(orc.KEY_1111)
        assert np.array_equal(sbits[:64], orc.verify_records(np.array(sub[:4096]), hk, valid, 0))
    finally:
        ctx.host_unregister(ring)
        ctx.host_unregister(rbits)


def test_empty_and_bad_arguments(ctx):
    ctx.key_add(0, orc.KEY_1111)
    bits = new_bits(1)
    ctx.verify_records(0, 0, 0)                  # n == 0: nothing to do
    recs = torch.zeros((4, 64), dtype=torch.uint8, device=DEV)
    with pytest.raises(hfv.HfvError):
        ctx.verify_records(recs.data_ptr() + 4, 3, bits)   # misaligned
    with pytest.raises(hfv.HfvError):
        ctx.verify_records(recs, 4, bits, stride=40)        # HF beyond the stride
    with pytest.raises(hfv.HfvError):
        ctx.set_keysel(7)


def test_pinned_keymap_attach(ctx, tmp_path, monkeypatch):
    """A data plane attached to the pinned map sees `hfv-loader key add/remove` from another
    process at its next batch (reusePinnedMap + RCU-like update, br_loader.cpp:119-126)."""
    import subprocess
    monkeypatch.setenv("HFV_PIN_DIR", str(tmp_path))
    loader = os.path.join(hfv.PKG_ROOT, "bin", "hfv-loader")
    path = hfv.keymap_path("br1")
    ctx.attach_keymap(path)                       # creates an empty map
    g = orc.load_golden("hf_single.npz")
    n = len(g["records"])
    d = dev(g["records"])
    bits = new_bits(n)
    ctx.verify_records(d, n, bits)
    assert not bits_np(bits, n).any()
    assert subprocess.run([loader, "key", "add", "br1", "0", "MTExMTExMTExMTExMTExMQ=="]).returncode == 0
    ctx.verify_records(d, n, bits)
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])
    assert subprocess.run([loader, "key", "remove", "br1", "0"]).returncode == 0
    ctx.verify_records(d, n, bits)
    assert not bits_np(bits, n).any()
    ctx.key_add(0, orc.KEY_1111)                  # write-through from the attached ctx
    assert hfv.keymap_read(path)[0] == orc.hop_key(orc.KEY_1111)
    ctx.verify_records(d, n, bits)
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])


def test_table_update_after_reader_stream_destroyed(ctx):
    """A key update after the stream that last read the key table was destroyed: the publish
    fences on an event recorded after that stream's launch, never on the dead stream."""
    import gc
    raw = orc.KEY_1111
    hk, valid = orc.key_table(raw)
    ctx.key_add(0, raw)
    recs = orc.gen_records(3000, hk, 0, seed=8)
    want = orc.verify_records(recs, hk, valid, 0)
    d = dev(recs)
    for _ in range(3):
        s = torch.cuda.Stream()
        bits = new_bits(3000)
        ctx.verify_records(d, 3000, bits, stream=s)
        s.synchronize()
        assert np.array_equal(bits_np(bits, 3000), want)
        del s
        gc.collect()
        ctx.key_add(7, orc.KEY_1111)   # dirty: the next launch publishes a new table
    bits = new_bits(3000)
    ctx.verify_records(d, 3000, bits, stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    assert np.array_equal(bits_np(bits, 3000), want)


@pytest.mark.parametrize("keysel", [0, 1])
def test_verdict_counters(ctx, keysel):
    """record_verdict for the verify-only paths: per AS-ingress IFID & 0xff, verified and
    INVALID_HF packets, from records + bitmap of the launch path and of the service; equal to
    the counts derived from the oracle's verdicts; counters are added to."""
    rng = np.random.default_rng(21 + keysel)
    raw = orc.gen_key_table(256)
    hk, valid = orc.key_table(raw)
    install(ctx, raw)
    ctx.set_keysel(keysel)
    recs = orc.gen_records(30011, hk, keysel, seed=123)
    junk = rng.random(len(recs)) < 0.1
    recs[junk] = rng.integers(0, 256, size=(int(junk.sum()), 64), dtype=np.uint8)
    n = len(recs)
    want_bits = orc.verify_records(recs, hk, valid, keysel)
    passed = hfv.bits_to_bool(want_bits, n)
    slot = np.where(recs[:, 40] & 1, recs[:, 51], recs[:, 53]).astype(np.int64)
    want = np.zeros((256, 2), dtype=np.uint64)
    np.add.at(want, (slot, (~passed).astype(np.int64)), 1)
    d = dev(recs)
    bits = new_bits(n)
    ctx.verify_records(d, n, bits)
    counters = torch.zeros((256, 2), dtype=torch.int64, device=DEV)
    ctx.verdict_counters(d, n, bits, counters)
    assert np.array_equal(host(counters).view(np.uint64), want)
    # the service's bitmap, counted into the same (added-to) counters
    sbits = new_bits(n)
    t = ctx.service_submit(d, n, sbits)
    ctx.service_wait(t, 20000)
    ctx.verdict_counters(d, n, sbits, counters)
    assert np.array_equal(host(counters).view(np.uint64), 2 * want)
    assert int(want[:, 1].sum()) == int((~passed).sum()) and int(want.sum()) == n
