"""The same 2^24 records (one 1 GiB buffer) verified as one hfv_verify_records launch and by the
resident service in 16, 4 and 1 batches: per-2^20 time and shader clock of each, interleaved
over reps, to size what the service loop costs against a plain launch at equal work.
Usage: python scripts/svc_vs_launch.py [reps]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scion-xdp-br_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import scion_hfv as hfv  # noqa: E402
import bench  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
N = 1 << 24
torch.cuda.set_device(0)
ctypes.CDLL("libamdhip64.so").hipSetDeviceFlags(ctypes.c_uint(1))
ctx = bench.make_ctx(hfv, 0, hfv.KEYSEL_ZERO)
sh = torch.cuda.current_stream().cuda_stream
big = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
ctx.gen_records(big, N, bench.SEED_RECORDS, first_index=0, stream=sh)
want = bench.expected_pass_count(N, 0)
bits = torch.zeros((N + 63) // 64, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()


def check():
    torch.cuda.synchronize()
    got = bench.popcount(bits)
    assert got == want, (got, want)
    bits.zero_()


posts = {}
for k in (16, 4, 1):
    m = N // k
    posts[k] = ctx.service_batches([(big[i * m:(i + 1) * m], m, bits[i * m // 64:(i + 1) * m // 64]) for i in range(k)])
L = hfv.lib()
stamped = L.hfv_debug_verify_stamped
stamped.restype = ctypes.c_int
stamped.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_size_t] + [ctypes.c_void_p] * 3 + [ctypes.POINTER(ctypes.c_int)]
stamps = torch.zeros((256 * 2 * 16, 16), dtype=torch.int64, device="cuda")


def launch_mhz():
    """shader clock of the launch kernel over its waves' lives (STAMP build of the same loop)"""
    stamps.zero_()
    grid = ctypes.c_int()
    assert stamped(ctx._h, big.data_ptr(), N, bits.data_ptr(), stamps.data_ptr(), sh, ctypes.byref(grid)) == 0
    check()
    st = stamps.cpu().numpy()[: grid.value * 16]
    st = st[st[:, 0] != 0]
    m = (st[:, 13] - st[:, 12]) / np.maximum(1, st[:, 15] - st[:, 1]) * 100.0
    xcc = (st[:, 14].astype(np.uint64) >> np.uint64(32)) & np.uint64(0xf)
    launch_xcd.append([round(float(np.median(m[xcc == x])), 0) if (xcc == x).any() else None for x in range(8)])
    return float(np.median(m))


blk = (ctypes.c_uint64 * 4096)()
L.hfv_debug_service_blocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]


def blocks():
    """last grid: (median block finish - first fill, max - min finish) in us"""
    g = ctypes.c_int()
    assert L.hfv_debug_service_blocks(ctx._h, blk, 4096, ctypes.byref(g)) == 0
    G = g.value
    a = np.array(blk[:4 * G], dtype=np.int64)
    st, fin, c0, c1 = a[:G], a[G:2 * G], a[2 * G:3 * G], a[3 * G:]
    mhz = (c1 - c0) / np.maximum(1, fin - st) * 100.0
    f = (fin - st.min()) / 100.0
    detail.append({"block0": round(float(f[0] - np.median(f)), 2),
                   "xcd_mhz": [round(float(np.median(mhz[x::8])), 0) for x in range(8)],
                   "xcd_median": [round(float(np.median(f[x::8]) - np.median(f)), 2) for x in range(8)],
                   "slowest": [(int(k), round(float(f[k] - np.median(f)), 2)) for k in np.argsort(f)[-6:]],
                   "fastest": [(int(k), round(float(f[k] - np.median(f)), 2)) for k in np.argsort(f)[:3]]})
    return (np.median(fin) - st.min()) / 100.0, (fin.max() - fin.min()) / 100.0, (st.max() - st.min()) / 100.0


spans = {16: [], 4: [], 1: []}
detail = []
launch_xcd = []
rows = {"launch": [], 16: [], 4: [], 1: []}
for rep in range(REPS + 1):
    ms = ctx.verify_records_timed(big, N, bits, stream=sh)
    check()
    mhz = launch_mhz()
    if rep:
        rows["launch"].append((ms, mhz))
    for k in (16, 4, 1):
        g = ctx.service_run(posts[k])[1]
        mhz = ctx.service_shader_mhz() or 0.0
        check()
        if rep:
            rows[k].append((g, mhz))
            spans[k].append(blocks())
for key, r in rows.items():
    a = np.array(r)
    print(f"{str(key):>6}: ms {np.median(a[:, 0]):.4f} (per 2^20 {np.median(a[:, 0]) / 16 * 1e3:6.2f} us, "
          f"frac {bench.BYTES_PER_PACKET * N / (np.median(a[:, 0]) * 1e-3) / 8e12:.3f})  mhz {np.median(a[:, 1]):6.0f}  "
          f"all {[round(x, 4) for x in a[:, 0]]}", flush=True)
for k, r in spans.items():
    a = np.array(r)
    print(f"{k:>6}: block finish median {np.median(a[:, 0]):7.1f} us after the first fill, finish spread "
          f"{np.median(a[:, 1]):6.1f} us, fill spread {np.median(a[:, 2]):5.1f} us", flush=True)
for d in detail[-6:]:
    print(d)
for x in launch_xcd[-3:]:
    print("launch xcd_mhz", x)
ctx.close()
