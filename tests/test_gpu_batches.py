"""hfv_verify_batches (the stream-ordered multi-batch launch) against the CPU checker and the
reference fixtures, and config 1's known-answer vectors through the HIP CMAC kernel.
Integer work: every comparison is bit-exact."""
import json
import os

import numpy as np
import pytest

import orc
import scion_hfv as hfv

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda:0"
KAT = json.load(open(os.path.join(orc.GOLDEN, "kat.json")))


def dev(a):
    return torch.from_numpy(np.array(a, copy=True)).to(DEV)


def bits_np(t, n):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)[: (n + 63) // 64]


def new_bits(n, fill=0):
    return torch.full((max(1, (n + 63) // 64),), fill, dtype=torch.int64, device=DEV)


@pytest.fixture()
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = hfv.Ctx(0)
    yield c
    c.synchronize()
    c.close()


def test_config1_kats_through_the_cmac_kernel(ctx):
    """Config 1 on the GPU: RFC 4493's one-block vector (aes/src/test/aes_test.cpp:156-245, key
    2b7e1516...) and the three blocks of aes/test/test.py:121-126 through hfv_cmac_tags
    (aes_cmac_16bytes, one lane per block), bit-exact against tests/golden/kat.json; the 48-bit
    verify form (verify_hop_field's compare) passes on the true tag and fails on a flipped bit."""
    key = bytes.fromhex(KAT["key"])
    ctx.key_add(0, key)
    msg = bytes.fromhex(KAT["cmac_msg"])
    cases = [(msg[:16], next(v["tag"] for v in KAT["cmac"] if v["len"] == 16))]
    cases += [(bytes.fromhex(v["data"]), v["tag"]) for v in KAT["testpy_blocks"]]
    n = len(cases)
    mi = np.frombuffer(b"".join(d for d, _ in cases), dtype=np.uint8).reshape(n, 16)
    tags = torch.zeros((n, 16), dtype=torch.uint8, device=DEV)
    ctx.cmac_tags(dev(mi), n, tags)
    torch.cuda.synchronize()
    got = [bytes(t).hex() for t in tags.cpu().numpy()]
    assert got == [t for _, t in cases]
    exp = np.array([int.from_bytes(bytes.fromhex(t)[:6], "little") for _, t in cases], dtype=np.uint64)
    bits = new_bits(n)
    ctx.verify_macinputs(dev(mi), dev(exp), n, bits)
    assert int(bits_np(bits, n)[0]) == (1 << n) - 1
    bad = exp ^ np.uint64(1 << 40)
    ctx.verify_macinputs(dev(mi), dev(bad), n, bits)
    assert int(bits_np(bits, n)[0]) == 0


@pytest.mark.parametrize("name,keysel", [("hf_single.npz", 0), ("hf_ifid256.npz", 1)])
def test_batches_golden(ctx, name, keysel):
    """The reference fixtures cut into ragged batches (and empty ones) of one launch."""
    g = orc.load_golden(name)
    n = len(g["records"])
    raw = g["raw_keys"].reshape(-1).tobytes()
    for k in range(int(g["nkeys"])):
        ctx.key_add(k, raw[16 * k:16 * k + 16])
    ctx.set_keysel(keysel)
    d = dev(g["records"])
    want = hfv.bits_to_bool(g["pass_bits"], n)
    cuts = [0, 1, 64, 64, 129, 500, 937, n]
    outs, batches = [], []
    for a, b in zip(cuts, cuts[1:]):
        bits = new_bits(b - a, fill=-1)
        outs.append((a, b, bits))
        batches.append((d[a:] if a < n else d, b - a, bits))
    ctx.verify_batches(batches)
    for a, b, bits in outs:
        if b > a:
            assert np.array_equal(hfv.bits_to_bool(bits_np(bits, b - a), b - a), want[a:b]), (a, b)
            assert int(bits_np(bits, b - a)[-1]) >> ((b - a) % 64 or 64) == 0   # no bit past n
        else:
            assert int(bits_np(bits, 1)[0]) == -1 & 0xFFFFFFFFFFFFFFFF   # an empty batch writes nothing


@pytest.mark.parametrize("keysel", [0, 1])
def test_batches_random_vs_oracle(ctx, keysel):
    """More batches than one launch holds (split into launches of 64), ragged sizes, strides
    64/72/128 and garbage records, against the oracle."""
    rng = np.random.default_rng(31 + keysel)
    raw = orc.gen_key_table(256)
    hk, valid = orc.key_table(raw)
    for k in range(256):
        ctx.key_add(k, raw[16 * k:16 * k + 16])
    ctx.set_keysel(keysel)
    base = orc.gen_records(40000, hk, keysel, seed=7)
    junk = rng.random(len(base)) < 0.2
    base[junk] = rng.integers(0, 256, size=(int(junk.sum()), 64), dtype=np.uint8)
    sizes = [int(x) for x in rng.choice([0, 1, 2, 63, 64, 65, 127, 300, 1000, 4097], size=150)]
    batches, checks, off = [], [], 0
    for i, m in enumerate(sizes):
        stride = (64, 72, 128)[i % 3]
        m = min(m, len(base) - off)
        recs = np.zeros((max(m, 1), stride), dtype=np.uint8)
        recs[:m, :64] = base[off:off + m]
        d = dev(recs)
        bits = new_bits(m, fill=-1)
        batches.append((d, m, bits, stride))
        checks.append((off, m, bits, d))
        off += m
    ctx.verify_batches(batches)
    for o, m, bits, _ in checks:
        if m:
            assert np.array_equal(bits_np(bits, m), orc.verify_records(base[o:o + m], hk, valid, keysel)), (o, m)


def test_batches_stream_ordered(ctx):
    """Producer, verify and consumer all on one stream with no host synchronisation between
    them: a kernel writes the records, hfv_verify_batches reads them in stream order, and a
    torch op on the same stream reads the bitmaps -- bit-exact against the generator truth."""
    ctx.key_add(0, orc.KEY_1111)
    s = torch.cuda.Stream()
    n, k = 1 << 18, 6
    with torch.cuda.stream(s):
        recs = [torch.empty((n, 64), dtype=torch.uint8, device=DEV) for _ in range(k)]
        bits = [torch.full(((n + 63) // 64,), -1, dtype=torch.int64, device=DEV) for _ in range(k)]
        torch.cuda._sleep(5_000_000)                     # the producer runs late
        for i in range(k):
            ctx.gen_records(recs[i], n, orc.SEED_RECORDS, first_index=i * n, stream=s)
        ctx.verify_batches([(recs[i], n, bits[i]) for i in range(k)], stream=s)
        joined = torch.cat(bits)                         # the consumer
    s.synchronize()
    got = hfv.bits_to_bool(joined.cpu().numpy().view(np.uint64), k * n)
    assert np.array_equal(got, orc.expected_pass_rule(k * n))


def test_batches_fail_closed_and_bad_arguments(ctx):
    g = orc.load_golden("hf_single.npz")
    n = len(g["records"])
    d = dev(g["records"])
    bits = new_bits(n, fill=-1)
    ctx.verify_batches([(d, n, bits)])                   # no key in slot 0
    assert not bits_np(bits, n).any()
    ctx.key_add_b64(0, "MTExMTExMTExMTExMTExMQ==")
    ctx.verify_batches([(d, n, bits)])
    assert np.array_equal(bits_np(bits, n), g["pass_bits"])
    ctx.verify_batches([])                               # nothing to do
    with pytest.raises(hfv.HfvError):
        ctx.verify_batches([(d.data_ptr() + 4, 3, bits)])    # misaligned
    with pytest.raises(hfv.HfvError):
        ctx.verify_batches([(d, n, bits), (d, 4, bits, 40)])  # HF beyond the stride
    with pytest.raises(hfv.HfvError):
        ctx.verify_batches([(d, n, 0)])                      # null bitmap


def test_batches_full_size_rotation(ctx):
    """The bench's shape: 20 batches of 2^20 records over 8 resident buffers, one call, timed
    form too; every bitmap equals its buffer's truth; the launch and the service agree."""
    ctx.key_add(0, orc.KEY_1111)
    n, R, K = 1 << 20, 8, 20
    recs = [torch.empty((n, 64), dtype=torch.uint8, device=DEV) for _ in range(R)]
    for i in range(R):
        ctx.gen_records(recs[i], n, orc.SEED_RECORDS, first_index=i * n)
    bits = [new_bits(n, fill=-1) for _ in range(K)]
    ms = ctx.verify_batches_timed([(recs[k % R], n, bits[k]) for k in range(K)])
    assert ms > 0
    for k in range(K):
        got = hfv.bits_to_bool(bits_np(bits[k], n), n)
        assert np.array_equal(got, orc.expected_pass_rule(n, first_index=(k % R) * n)), k
    sbits = new_bits(n)
    t = ctx.service_submit(recs[3], n, sbits)
    ctx.service_wait(t, 10000)
    ctx.service_stop()
    assert torch.equal(sbits, bits[3])
