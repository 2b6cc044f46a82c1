"""Config 4 on the GPU: hfv_br_process (hfv_br_kernel.hip) against the oracle border router,
bit-exact on frames (every byte of every slot), XDP action, verdict, redirect target and the
verdict counters; plus the PTF scenarios end to end through chained GPU routers."""
import numpy as np
import pytest

import br_fuzz as F
import br_topo as T
import orc
import scion_hfv as hfv
from conftest import rerun_on_test_build

pytestmark = pytest.mark.gpu
MAC = lambda k, m: orc.cmac(m, k)   # noqa: E731


def _gpu_brs(ctx, v6, key0=T.KEYS[1]):
    return {b: T.GpuBR(ctx, T.br_config(b, v6), key0=key0) for b in ("br1", "br2", "br3")}


@pytest.mark.parametrize("v6", [False, True], ids=["ipv4", "ipv6"])
def test_ptf_scenarios_gpu(gpu_ctx, v6):
    brs = _gpu_brs(gpu_ctx, v6)
    for name, kind, frame, first, ifi, want, veth_out in F.ptf_cases(v6, MAC):
        out, last, egress, trace = T.run_chain(brs, frame, first, ifi)
        assert out == want, (name, kind)
        assert egress == veth_out
        for br, a, v, _ in trace:
            assert (a, v) == (4, hfv.VERDICT["SCION_FORWARD"])
        s = trace[0][3]
        assert s[ifi, 0, 1] == len(frame) and s[ifi, 1, 1] == 1 and s.sum() == len(frame) + 1


def _compare(gpu_ctx, frames, lens, ifidx, cfg, key0, hf_check=True, feat_off=0):
    ref = frames.copy()
    oa, ov, oe, os_ = orc.br_process(ref, lens, ifidx, cfg, orc.hop_key(key0) if key0 is not None else None,
                                     hf_check=hf_check, feat_off=feat_off)
    got = frames.copy()
    ga, gv, ge, gs = T.GpuBR(gpu_ctx, cfg, key0=key0, hf_check=hf_check, feat_off=feat_off).process(got, lens, ifidx)
    bad = np.nonzero((ga != oa) | (gv != ov) | (ge != oe) | (got != ref).any(axis=1))[0]
    assert bad.size == 0, "first mismatch at frame %d: gpu (%d,%d,%d) oracle (%d,%d,%d)" % (
        bad[0], ga[bad[0]], gv[bad[0]], ge[bad[0]], oa[bad[0]], ov[bad[0]], oe[bad[0]])
    assert (gs == os_).all()
    return ov


@pytest.mark.parametrize("v6", [False, True], ids=["ipv4", "ipv6"])
def test_segid_rewrite_inside_checked_hop_field(gpu_ctx, v6):
    """The kernel reads the macinput at the MAC check, after the rewrite: a frame whose rewritten
    SegID lies in the checked hop field (br_fuzz.overlap_frame) must still verify against the
    bytes from before the rewrite, like the oracle; in a 64-frame tile with ordinary frames."""
    frame, first, ifi, want = F.overlap_frame(v6)
    cfg = T.br_config(first, v6)
    brs = {b: T.OracleBR(T.br_config(b, v6)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, v6, MAC)
    rest = [(f, i) for b, i, f in hops if b == first][:63]
    frames, lens = T.to_slots([frame] + [f for f, _ in rest])
    ifidx = np.array([ifi] + [i for _, i in rest], dtype=np.uint32)
    v = _compare(gpu_ctx, frames, lens, ifidx, cfg, T.KEYS[1])
    assert v[0] == hfv.VERDICT["SCION_FORWARD"] and frames[0, :len(want)].tobytes() != want   # input untouched
    got = frames.copy()
    T.GpuBR(gpu_ctx, cfg).process(got, lens, ifidx)
    assert got[0, :len(want)].tobytes() == want


def test_ipv4_options_across_the_window(gpu_ctx):
    """IPv4 options (IHL 6..15) move PathMeta, the info and hop fields and the rewritten SegIDs
    4..40 bytes further, so the kernel's reads and writes fall inside, across and past its
    128-byte staging window: bit-exact against the oracle, and routed like the unshifted frames."""
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    frames, lens, ifidx, m = F.options_shift_batch(F.hop_inputs(brs, False, MAC))
    v = _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1"), T.KEYS[1]).reshape(11, m)
    assert (v == v[0]).all() and (v[0] == hfv.VERDICT["SCION_FORWARD"]).sum() >= m // 2


@pytest.mark.parametrize("hdrlen", [0, 23, 255])
def test_hdrlen_hint_across_the_window(gpu_ctx, hdrlen):
    """The kernel loads bytes 128-135 early for a frame whose SCION header, by its HdrLen, runs
    past the staging window (a hint only: the router never checks HdrLen).  With every frame's
    HdrLen forced to 0 (no early load: every read past the window goes to HBM), 23 (92 bytes:
    the load for the frames shifted by IPv4 options) or 255 (the load for every frame) the
    results stay bit-exact against the oracle, frames inside, across and past the window."""
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    frames, lens, ifidx, m = F.options_shift_batch(F.hop_inputs(brs, False, MAC))
    for i in range(len(frames)):
        sc = 14 + 4 * (frames[i, 14] & 15) + 8
        frames[i, sc + 5] = hdrlen
    _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1"), T.KEYS[1])


@pytest.mark.parametrize("v6", [False, True], ids=["ipv4", "ipv6"])
@pytest.mark.parametrize("br", ["br1", "br2", "br3"])
def test_fuzz_parity(gpu_ctx, br, v6):
    brs = {b: T.OracleBR(T.br_config(b, v6)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, v6, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, br, v6, 20000, seed=100 + v6, payload_max=1500)
    verdicts = _compare(gpu_ctx, frames, lens, ifidx, T.br_config(br, v6), T.KEYS[1])
    assert len(np.unique(verdicts)) >= 6


def test_fuzz_parity_no_key_and_foreign_key(gpu_ctx):
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, 4000, seed=7)
    v = _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1"), None)
    # no key: every frame that reaches a hop-field check fails it; internal -> internal IP
    # forwarding checks none and still forwards (fib_ip_forward path, xdp.c:235-238)
    assert hfv.VERDICT["INVALID_HF"] in v
    fwd = np.nonzero(v == hfv.VERDICT["SCION_FORWARD"])[0]
    assert np.isin(ifidx[fwd], [5, 7]).all()          # BR 1's internal interfaces
    _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1"), T.KEYS[5])


@pytest.mark.parametrize("v6", [False, True], ids=["ipv4", "ipv6"])
def test_fuzz_parity_hf_check_off(gpu_ctx, v6):
    """ENABLE_HF_CHECK=OFF (br/CMakeLists.txt:8): no frame is dropped for its hop-field MAC,
    everything else as with the check; bit-exact against the oracle built the same way."""
    brs = {b: T.OracleBR(T.br_config(b, v6)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, v6, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", v6, 20000, seed=200 + v6, payload_max=1500)
    v = _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1", v6), T.KEYS[1], hf_check=False)
    assert hfv.VERDICT["INVALID_HF"] not in v
    _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1", v6), None, hf_check=False)   # no key: still forwarded
    gpu_ctx.br_set_hf_check(True)


@pytest.mark.parametrize("opt", ["no_ipv6", "no_ipv4", "no_scion_path"])
def test_fuzz_parity_build_options(gpu_ctx, opt):
    """The reference's ENABLE_IPV4 / ENABLE_IPV6 / ENABLE_SCION_PATH builds (br/CMakeLists.txt:5-7):
    an IPv4-only (IPv6-only) router over a mix of IPv4 and IPv6 frames passes the other family
    up the stack as NOT_SCION; without the SCION path type every SCION frame is NOT_IMPLEMENTED.
    Bit-exact against the oracle built the same way."""
    v6cfg = opt == "no_ipv4"
    mix = []
    for v6 in (False, True):
        brs = {b: T.OracleBR(T.br_config(b, v6)) for b in ("br1", "br2", "br3")}
        mix.append(F.fuzz_batch(F.hop_inputs(brs, v6, MAC), "br1", v6, 4000, seed=300 + v6))
    frames = np.concatenate([mix[0][0], mix[1][0]])
    lens = np.concatenate([mix[0][1], mix[1][1]])
    ifidx = np.concatenate([mix[0][2], mix[1][2]])
    order = np.random.default_rng(5).permutation(len(frames))
    frames, lens, ifidx = np.ascontiguousarray(frames[order]), lens[order], ifidx[order]
    feat = {"no_ipv6": hfv.BR_NO_IPV6, "no_ipv4": hfv.BR_NO_IPV4, "no_scion_path": hfv.BR_NO_SCION_PATH}[opt]
    v = _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1", v6cfg), T.KEYS[1], feat_off=feat)
    if opt == "no_scion_path":
        assert hfv.VERDICT["SCION_FORWARD"] not in v and hfv.VERDICT["NOT_IMPLEMENTED"] in v
    else:
        assert hfv.VERDICT["SCION_FORWARD"] in v and hfv.VERDICT["NOT_SCION"] in v
    gpu_ctx.br_set_build_options(0)


def test_large_batch_mixed_sizes(gpu_ctx):
    """2^17 frames of 64..1500 B in 2 KiB slots (the config-4 shape): parity with the oracle."""
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, 1 << 17, seed=3, payload_max=1500)
    _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1"), T.KEYS[1])


@pytest.mark.parametrize("hf_check", [True, False], ids=["hf_check", "hf_check_off"])
def test_bench_batch_full_size_bit_exact(gpu_ctx, hf_check):
    """the batch the config-4 bench times -- 2^20 frames in 2 KiB slots,
    i.e. 16384 tiles, every one of the 256 x 16 waves running 4 of them -- compared with the
    oracle byte for byte (every slot byte), with action, verdict, egress and the counters
    (xdp.c:250-283 over the whole batch)."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n = 1 << 20
    tmpl, tid, lens, ifidx, n_good = bench.br_batch(n, 0)
    frames = tmpl[tid]                                     # n x 2 KiB
    cfg = T.br_config("br1")
    want = frames.copy()
    oa, ov, oe, os_ = orc.br_process(want, lens, ifidx, cfg, orc.hop_key(T.KEYS[1]), hf_check=hf_check)
    gpu_ctx.br_set_config(cfg)
    gpu_ctx.key_add(0, T.KEYS[1])
    gpu_ctx.br_set_hf_check(hf_check)
    d = torch.from_numpy(frames).cuda()
    dl = torch.from_numpy(lens.view(np.int16)).cuda()
    di = torch.from_numpy(ifidx.view(np.int32)).cuda()
    a = torch.zeros(n, dtype=torch.uint8, device="cuda")
    v = torch.zeros_like(a)
    e = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(64 * 2 * 11, dtype=torch.int64, device="cuda")
    gpu_ctx.br_process(d, bench.BR_SLOT, dl, di, n, a, v, e, st)
    torch.cuda.synchronize()
    ga, gv, ge = a.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy()
    bad = np.nonzero((ga != oa) | (gv != ov) | (ge != oe))[0]
    assert bad.size == 0, (bad[:8], ga[bad[:4]], oa[bad[:4]], gv[bad[:4]], ov[bad[:4]])
    dw = torch.from_numpy(want).cuda()
    rows = torch.nonzero((d != dw).any(dim=1)).flatten().cpu().numpy()
    assert rows.size == 0, ("frame bytes differ", rows[:8])
    assert (st.cpu().numpy().view(np.uint64).reshape(64, 2, 11) == os_).all()
    assert int((ga == 4).sum()) == (n_good if hf_check else n)
    gpu_ctx.br_set_hf_check(True)


def test_split_launch_counters(request, gpu_ctx):
    """The block counters are 32-bit in LDS (HFV_BR_STATS32); a launch whose blocks could count
    2^32 bytes is split into pieces that add into the same 64-bit counters.  Forced here with a
    small piece size (hfv_debug_br_split): a ragged 2^14 + 37-frame fuzz batch in pieces of 1000
    frames must give the oracle's frames, outputs and counters exactly."""
    if rerun_on_test_build(request):   # uses a test hook: runs on lib/libscionhfv_test.so
        return
    hops = F.hop_inputs({b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, (1 << 14) + 37, seed=11, payload_max=1500)
    hfv.Ctx.debug_br_split(1000)
    try:
        _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1"), T.KEYS[1])
    finally:
        hfv.Ctx.debug_br_split(0)


def test_stats_accumulate_and_bad_args(gpu_ctx):
    import torch
    ing_enc, egr_enc, first, ifi = T.encaps(1, 2, False)
    from scion_hfv import packets as P
    frame = ing_enc.frame(P.scion_header(P.ptf_path("down", 1, 2, T.KEYS, seed=9, mac_fn=MAC).pack()))
    buf, lens = T.to_slots([frame] * 100)
    gpu_ctx.br_set_config(T.br_config("br1"))
    gpu_ctx.key_add(0, T.KEYS[1])
    d = torch.from_numpy(buf).cuda()
    dl = torch.from_numpy(lens.view(np.int16)).cuda()
    di = torch.full((100,), ifi, dtype=torch.int32, device="cuda")
    a = torch.zeros(100, dtype=torch.uint8, device="cuda")
    v = torch.zeros_like(a)
    e = torch.zeros(100, dtype=torch.int32, device="cuda")
    s = torch.zeros(64 * 2 * 11, dtype=torch.int64, device="cuda")
    gpu_ctx.br_process(d, T.SLOT, dl, di, 100, a, v, e, s)
    gpu_ctx.br_process(d, T.SLOT, dl, di, 100, a, v, e, s)   # second pass: now addressed to the next AS
    torch.cuda.synchronize()
    st = s.cpu().numpy().reshape(64, 2, 11)
    assert st[ifi, 1, 1] == 100 and st[ifi, 1, 5] == 100          # FORWARD, then NO_INTERFACE
    assert st[ifi, 0, 1] == 100 * len(frame)
    with pytest.raises(hfv.HfvError):
        gpu_ctx.br_process(d, 60, dl, di, 100, a, v, e, s)       # slot < 64
    with pytest.raises(hfv.HfvError):
        gpu_ctx.br_process(d, 2044, dl, di, 100, a, v, e, s)     # slot % 8
    cfg = T.br_config("br1")
    cfg.n_routes = 65
    with pytest.raises(hfv.HfvError):
        gpu_ctx.br_set_config(cfg)


@pytest.mark.parametrize("window,register", [(64, False), (256, False), (0, False), (0, True)],
                         ids=["win64", "win256", "windefault", "zerocopy"])
def test_host_path_matches_oracle(gpu_ctx, window, register):
    """Config 5 (hfv_br_process_host): frames in host memory.  Unregistered: only a header
    window crosses PCIe by DMA; frames whose headers pass the window (long paths, and for
    window 64 nearly all) are re-run whole.  Registered: zero-copy, the kernel reads the
    mapped ring itself.  Result identical to the oracle on the full frames either way."""
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, 70000, seed=21, payload_max=1500)
    longf = F.long_path_frames(False, MAC)
    for k, (f, ifi) in enumerate(longf):   # sprinkle long-path frames over both chunks
        i = 1000 + k * 8191
        frames[i] = 0
        frames[i, :len(f)] = np.frombuffer(f, dtype=np.uint8)
        lens[i], ifidx[i] = len(f), ifi
    ref = frames.copy()
    oa, ov, oe, os_ = orc.br_process(ref, lens, ifidx, T.br_config("br1"), orc.hop_key(T.KEYS[1]))
    gpu_ctx.br_set_config(T.br_config("br1"))
    gpu_ctx.key_add(0, T.KEYS[1])
    n = len(frames)
    got = hfv.host_array(frames.shape, np.uint8) if register else frames.copy()
    got[:] = frames
    a = hfv.host_array(n, np.uint8) if register else np.zeros(n, np.uint8)
    v = np.zeros(n, np.uint8)
    e = np.zeros(n, np.int32)
    st = np.zeros((64, 2, 11), np.uint64)
    if register:
        gpu_ctx.host_register(got)
        gpu_ctx.host_register(a)      # an output array used in place as well
    try:
        gpu_ctx.br_process_host(got, T.SLOT, lens, ifidx, n, a, v, e, st, window=window)
    finally:
        if register:
            gpu_ctx.host_unregister(got)
            gpu_ctx.host_unregister(a)
    assert (a == oa).all() and (v == ov).all() and (e == oe).all()
    assert (got == ref).all()
    assert (st == os_).all()
    assert (a[[1000 + k * 8191 for k in range(len(longf))]] == 4).all()


def test_host_path_pageable_and_args(gpu_ctx):
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, 3000, seed=5, slot=512)
    ref = frames.copy()
    oa, ov, oe, _ = orc.br_process(ref, lens, ifidx, T.br_config("br1"), orc.hop_key(T.KEYS[1]))
    gpu_ctx.br_set_config(T.br_config("br1"))
    gpu_ctx.key_add(0, T.KEYS[1])
    a = np.zeros(3000, np.uint8)
    v = np.zeros(3000, np.uint8)
    e = np.zeros(3000, np.int32)
    gpu_ctx.br_process_host(frames, 512, lens, ifidx, 3000, a, v, e, None, window=128)   # not registered
    assert (a == oa).all() and (v == ov).all() and (e == oe).all() and (frames == ref).all()
    for bad in (60, 1024, 100):
        with pytest.raises(hfv.HfvError):
            gpu_ctx.br_process_host(frames, 512, lens, ifidx, 3000, a, v, e, None, window=bad)


def test_fuzz_parity_unstaged_slot(gpu_ctx):
    """slot % 16 != 0 selects the direct-from-HBM kernel variant (no LDS header staging)."""
    brs = {b: T.OracleBR(T.br_config(b, True)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, True, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", True, 6000, seed=9, slot=1032, payload_max=1000)
    _compare(gpu_ctx, frames, lens, ifidx, T.br_config("br1", True), T.KEYS[1])


def test_host_path_survives_keymap_attach(gpu_ctx, tmp_path, monkeypatch):
    """Attaching the pinned key map after the host path ran must leave the host path's
    staging buffers alone (regression: the attach once freed them without forgetting them,
    so the next host batch or ctx destruction used freed memory)."""
    monkeypatch.setenv("HFV_PIN_DIR", str(tmp_path))
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, 2000, seed=17, slot=512)
    ref = frames.copy()
    oa, ov, oe, _ = orc.br_process(ref, lens, ifidx, T.br_config("br1"), orc.hop_key(T.KEYS[1]))
    gpu_ctx.br_set_config(T.br_config("br1"))
    gpu_ctx.key_add(0, T.KEYS[1])
    for attach in (False, True):
        got = frames.copy()
        a = np.zeros(2000, np.uint8)
        v = np.zeros(2000, np.uint8)
        e = np.zeros(2000, np.int32)
        gpu_ctx.br_process_host(got, 512, lens, ifidx, 2000, a, v, e, None, window=128)
        assert (a == oa).all() and (v == ov).all() and (e == oe).all() and (got == ref).all()
        if not attach:
            gpu_ctx.attach_keymap(hfv.keymap_path("br1"))   # an empty map: re-add the key through it
            gpu_ctx.key_add(0, T.KEYS[1])


def test_attached_pinned_brconfig_reloads(gpu_ctx, tmp_path, monkeypatch):
    """hfv_ctx_attach_brconfig: the data plane takes its router tables from the pinned file
    `hfv-loader attach` publishes and picks up a republished version at the next batch."""
    monkeypatch.setenv("HFV_PIN_DIR", str(tmp_path))
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    hops = F.hop_inputs(brs, False, MAC)
    frames, lens, ifidx = F.fuzz_batch(hops, "br1", False, 3000, seed=31)
    path = hfv.brconfig_path("br1-ff00_0_1-1")
    hfv.brconfig_publish(path, T.br_config("br1"))
    import ctypes
    import torch

    class Pinned(T.GpuBR):   # like GpuBR, but without installing tables itself
        def process(self, frames, lens, ifidx):
            ctx = self.ctx
            ctx.key_add(0, T.KEYS[1])
            n, slot = frames.shape
            d = torch.from_numpy(frames).cuda()
            dl = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).cuda()
            di = torch.from_numpy(ifidx.astype(np.uint32).view(np.int32)).cuda()
            a = torch.zeros(n, dtype=torch.uint8, device="cuda")
            v = torch.zeros_like(a)
            e = torch.zeros(n, dtype=torch.int32, device="cuda")
            ctx.br_process(d, slot, dl, di, n, a, v, e)
            torch.cuda.synchronize()
            frames[:] = d.cpu().numpy()
            return a.cpu().numpy(), v.cpu().numpy(), e.cpu().numpy()

    gpu_ctx.br_set_config(hfv.BrConfig())          # empty tables: the attach must replace them
    gpu_ctx.br_set_hf_check(True)
    gpu_ctx.attach_brconfig(path)
    for cfg_name in ("br1", "br2"):
        hfv.brconfig_publish(path, T.br_config(cfg_name))
        ref = frames.copy()
        oa, ov, oe, _ = orc.br_process(ref, lens, ifidx, T.br_config(cfg_name), orc.hop_key(T.KEYS[1]))
        got = frames.copy()
        ga, gv, ge = Pinned(gpu_ctx, None).process(got, lens, ifidx)
        assert (ga == oa).all() and (gv == ov).all() and (ge == oe).all() and (got == ref).all(), cfg_name
    assert ctypes.sizeof(hfv.BrConfig) > 0
    # `hfv-loader detach`: the attached data plane sees the detached state at its
    # next batch and passes every frame untouched, as an interface without the XDP program does
    hfv.brconfig_detach(path)
    got = frames.copy()
    ga, gv, ge = Pinned(gpu_ctx, None).process(got, lens, ifidx)
    assert (ga == 2).all() and (gv == 0).all() and (ge == -1).all() and (got == frames).all()
    # a later attach republishes into the same file: the data plane routes again
    hfv.brconfig_publish(path, T.br_config("br1"))
    ref = frames.copy()
    oa, ov, oe, _ = orc.br_process(ref, lens, ifidx, T.br_config("br1"), orc.hop_key(T.KEYS[1]))
    got = frames.copy()
    ga, gv, ge = Pinned(gpu_ctx, None).process(got, lens, ifidx)
    assert (ga == oa).all() and (gv == ov).all() and (ge == oe).all() and (got == ref).all()
