"""Python binding of libscionhfv.so (include/scion_hfv.h) -- SCION hop-field AES-CMAC
verification on MI355X.

Thin ctypes layer over the C ABI; every data-path call goes to the HIP kernels.  There is
no CPU fallback: if the shared library or a GPU is missing, calls raise HfvError.

Device buffers may be given as torch CUDA tensors (``data_ptr()`` is used) or raw integer
device pointers.  torch is imported before the library is loaded so that both share one
HIP runtime in the process (device pointers and streams then interoperate).
"""
import ctypes
import errno
import os
import sys

try:  # load torch's HIP runtime first (same soname as /opt/rocm's), see module docstring
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for C-style use
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libscionhfv.so")
# the test build: the same library plus the test hooks (hfv_debug_relay_delay, _publish_delay,
# _br_grid, _br_split, _loop_host_stage); loaded only by tests (HFV_LIB), never by the product path
TEST_LIB_PATH = os.path.join(PKG_ROOT, "lib", "libscionhfv_test.so")

KEYSEL_ZERO = 0
KEYSEL_IFID = 1
MAX_KEYS = 256
REC_INF_OFF = 40
REC_HF_OFF = 48
REC_SIZE = 64
SVC_RING = 128   # resident-service descriptor ring (kSvcRing, csrc/hfv_internal.h)
SVC_INLINE = 64  # descriptors a service grid gets in its kernel arguments (kSvcInline)
BYTES_PER_PACKET = 64 + 1.0 / 8  # algorithmic HBM bytes per verified record


class HfvError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (rc={code} {errno.errorcode.get(-code, '')})")
        self.code = code


_lib = None


def lib():
    """Load libscionhfv.so once; raise HfvError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("HFV_LIB") or LIB_PATH   # HFV_LIB: another build (A/B measurements)
    if not os.path.exists(path):
        raise HfvError(-errno.ENOENT, f"{path} not built (run `make -C {PKG_ROOT}`)")
    L = ctypes.CDLL(path)
    vp, sz, u32, u64, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sigs = {
        "hfv_ctx_create": (i32, [i32, ctypes.POINTER(vp)]),
        "hfv_ctx_destroy": (i32, [vp]),
        "hfv_ctx_device": (i32, [vp]),
        "hfv_ctx_numa_node": (i32, [vp]),
        "hfv_ctx_stream": (vp, [vp]),
        "hfv_ctx_set_keysel": (i32, [vp, i32]),
        "hfv_ctx_set_record_layout": (i32, [vp, u32, u32]),
        "hfv_ctx_synchronize": (i32, [vp]),
        "hfv_key_add": (i32, [vp, u32, vp]),
        "hfv_key_add_b64": (i32, [vp, u32, ctypes.c_char_p]),
        "hfv_key_set_hop_key": (i32, [vp, u32, vp]),
        "hfv_key_remove": (i32, [vp, u32]),
        "hfv_key_get": (i32, [vp, u32, vp]),
        "hfv_key_add_batch": (i32, [vp, u32, vp, sz]),
        "hfv_verify_records": (i32, [vp, vp, sz, sz, vp, vp]),
        "hfv_verify_records_timed": (i32, [vp, vp, sz, sz, vp, vp, ctypes.POINTER(ctypes.c_float)]),
        "hfv_verify_batches": (i32, [vp, vp, sz, vp]),
        "hfv_verify_batches_timed": (i32, [vp, vp, sz, vp, ctypes.POINTER(ctypes.c_float)]),
        "hfv_ctx_describe": (i32, [vp, ctypes.c_char_p, sz]),
        "hfv_ctx_attach_keymap": (i32, [vp, ctypes.c_char_p]),
        "hfv_keymap_path": (i32, [ctypes.c_char_p, ctypes.c_char_p, sz]),
        "hfv_keymap_update": (i32, [ctypes.c_char_p, u32, vp]),
        "hfv_keymap_erase": (i32, [ctypes.c_char_p, u32]),
        "hfv_keymap_read": (i32, [ctypes.c_char_p, vp, vp]),
        "hfv_keymap_create_mode": (i32, [ctypes.c_char_p, i32]),
        "hfv_keymap_mode": (i32, [ctypes.c_char_p]),
        "hfv_keymap_list": (i32, [ctypes.c_char_p, vp, vp, sz, ctypes.POINTER(sz)]),
        "hfv_verify_macinputs": (i32, [vp, vp, vp, vp, sz, vp, vp]),
        "hfv_verdict_counters": (i32, [vp, vp, sz, sz, vp, vp, vp]),
        "hfv_br_set_config": (i32, [vp, vp]),
        "hfv_br_set_hf_check": (i32, [vp, i32]),
        "hfv_br_set_build_options": (i32, [vp, u32]),
        "hfv_br_config_check_options": (i32, [vp, u32]),
        "hfv_brconfig_publish_opts": (i32, [ctypes.c_char_p, vp, u32]),
        "hfv_br_config_load": (i32, [ctypes.c_char_p, vp, sz, vp, sz, vp, ctypes.c_char_p, sz, ctypes.c_char_p, sz,
                                     ctypes.c_char_p, sz]),
        "hfv_br_load_config": (i32, [vp, ctypes.c_char_p, vp, sz]),
        "hfv_brconfig_path": (i32, [ctypes.c_char_p, ctypes.c_char_p, sz]),
        "hfv_brconfig_publish": (i32, [ctypes.c_char_p, vp]),
        "hfv_brconfig_read": (i32, [ctypes.c_char_p, vp]),
        "hfv_brconfig_detach": (i32, [ctypes.c_char_p]),
        "hfv_ctx_attach_brconfig": (i32, [vp, ctypes.c_char_p]),
        "hfv_br_process": (i32, [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp, vp]),
        "hfv_br_process_timed": (i32, [vp, vp, sz, vp, vp, sz, vp, vp, vp, vp, vp, ctypes.POINTER(ctypes.c_float)]),
        "hfv_br_process_host": (i32, [vp, vp, sz, vp, vp, sz, sz, vp, vp, vp, vp]),
        "hfv_host_register": (i32, [vp, vp, sz]),
        "hfv_loop_run": (i32, [vp, vp, vp]),
        "hfv_statsmap_path": (i32, [ctypes.c_char_p, ctypes.c_char_p, sz]),
        "hfv_statsmap_add": (i32, [ctypes.c_char_p, vp]),
        "hfv_statsmap_read": (i32, [ctypes.c_char_p, vp]),
        "hfv_host_unregister": (i32, [vp, vp]),
        "hfv_cmac_tags": (i32, [vp, vp, vp, sz, vp, vp]),
        "hfv_verify_records_host": (i32, [vp, vp, sz, sz, vp]),
        "hfv_service_start": (i32, [vp, u32]),
        "hfv_service_submit": (i32, [vp, vp, sz, sz, vp, ctypes.POINTER(u64)]),
        "hfv_service_submitv": (i32, [vp, vp, sz, ctypes.POINTER(u64)]),
        "hfv_service_run": (i32, [vp, vp, sz, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_float)]),
        "hfv_service_run_async": (i32, [vp, vp, sz, ctypes.POINTER(u64)]),
        "hfv_service_poll": (i32, [vp, u64]),
        "hfv_service_wait": (i32, [vp, u64, i32]),
        "hfv_service_stop": (i32, [vp, ctypes.POINTER(ctypes.c_float)]),
        "hfv_service_running": (i32, [vp]),
        "hfv_expand_keys": (i32, [vp, vp, sz, vp, vp]),
        "hfv_gen_records": (i32, [vp, vp, sz, sz, u64, u64, vp]),
        "hfv_verify_macinput": (i32, [vp, u64, vp]),
        "hfv_decode_key_b64": (i32, [ctypes.c_char_p, vp]),
        "hfv_dev_alloc": (i32, [vp, sz, ctypes.POINTER(vp)]),
        "hfv_dev_free": (i32, [vp, vp]),
        "hfv_memcpy_h2d": (i32, [vp, vp, vp, sz]),
        "hfv_memcpy_d2h": (i32, [vp, vp, vp, sz]),
        "hfv_last_error": (ctypes.c_char_p, []),
        "hfv_abi_version": (i32, []),
        "hfv_service_set_timing": (i32, [vp, i32]),
        "hfv_service_set_grid": (i32, [vp, i32]),
        "aes_key_expansion": (None, [vp, vp]),
        "aes_cypher": (i32, [vp, vp, vp]),
        "aes_cmac_subkeys": (None, [vp, vp]),
        "aes_cmac": (None, [vp, sz, vp, vp, vp]),
        "aes_cmac_no_loops": (None, [vp, sz, vp, vp, vp]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise HfvError(rc, lib().hfv_last_error().decode(errors="replace"))
    return rc


def _ptr(x):
    """Device/host pointer from a torch tensor, numpy array, ctypes buffer or int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return ctypes.cast(x, ctypes.c_void_p).value


def _stream(stream):
    """hipStream_t for a call: an explicit int/torch stream, else torch's current stream
    (so work stays ordered with torch ops on the same buffers), else HIP's default stream."""
    if stream is None:
        if torch is not None and torch.cuda.is_initialized():
            return torch.cuda.current_stream().cuda_stream or None
        return None
    if isinstance(stream, int):
        return stream          # 0 is the NULL (default) stream
    return stream.cuda_stream  # torch.cuda.Stream


# ---- aes.h surface (host, control plane) ---------------------------------------------------

def aes_key_expansion(key: bytes) -> bytes:
    out = ctypes.create_string_buffer(176)
    lib().aes_key_expansion(bytes(key), out)
    return out.raw


def aes_cypher(block: bytes, sched: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().aes_cypher(bytes(block), bytes(sched), out)
    return out.raw


def aes_cmac_subkeys(sched: bytes):
    out = ctypes.create_string_buffer(32)
    lib().aes_cmac_subkeys(bytes(sched), out)
    return out.raw[:16], out.raw[16:]


def aes_cmac(data: bytes, key: bytes, no_loops=False) -> bytes:
    sched = aes_key_expansion(key)
    k1, k2 = aes_cmac_subkeys(sched)
    out = ctypes.create_string_buffer(16)
    fn = lib().aes_cmac_no_loops if no_loops else lib().aes_cmac
    fn(bytes(data), len(data), sched, k1 + k2, out)
    return out.raw


def hop_key(key: bytes) -> bytes:
    """192-byte struct hop_key image (br/src/bpf/common.h:87-91) for a raw 16-byte key."""
    sched = aes_key_expansion(key)
    k1, _ = aes_cmac_subkeys(sched)
    return sched + k1


def decode_key_b64(s: str) -> bytes:
    out = ctypes.create_string_buffer(16)
    _check(lib().hfv_decode_key_b64(s.encode(), out))
    return out.raw


def verify_macinput(macinput: bytes, expected: int, hop_key_bytes) -> bool:
    return bool(lib().hfv_verify_macinput(bytes(macinput), expected, None if hop_key_bytes is None else bytes(hop_key_bytes)))


# ---- context --------------------------------------------------------------------------------

class HfvBatch(ctypes.Structure):
    """struct hfv_batch (hfv_service_submitv)"""
    _fields_ = [("recs", ctypes.c_void_p), ("stride", ctypes.c_size_t), ("n", ctypes.c_size_t),
                ("pass_bits", ctypes.c_void_p)]


class LoopConfig(ctypes.Structure):
    """struct hfv_loop_config"""
    _fields_ = [("frames", ctypes.c_void_p), ("lens", ctypes.c_void_p), ("n_frames", ctypes.c_size_t),
                ("frame_stride", ctypes.c_size_t), ("rx_ifindex", ctypes.c_uint32), ("slot", ctypes.c_uint32),
                ("chunk", ctypes.c_size_t), ("chunks", ctypes.c_size_t), ("total", ctypes.c_uint64),
                ("producers", ctypes.c_int), ("consumers", ctypes.c_int), ("digest", ctypes.c_int),
                ("inflight", ctypes.c_int), ("dma", ctypes.c_int), ("stats", ctypes.c_void_p),
                ("rx_ifname", ctypes.c_char_p), ("tx_ifname", ctypes.c_char_p), ("idle_ms", ctypes.c_int)]


class LoopStats(ctypes.Structure):
    """struct hfv_loop_stats"""
    _fields_ = [("rx_pkts", ctypes.c_uint64), ("tx_pkts", ctypes.c_uint64), ("tx_bytes", ctypes.c_uint64),
                ("drop_pkts", ctypes.c_uint64), ("tx_digest", ctypes.c_uint64),
                ("verdict_pkts", ctypes.c_uint64 * 11), ("seconds", ctypes.c_double),
                ("gpu_busy_s", ctypes.c_double), ("gpu_wait_s", ctypes.c_double),
                ("producer_busy_s", ctypes.c_double), ("consumer_busy_s", ctypes.c_double),
                ("rx_truncated", ctypes.c_uint64), ("tx_errors", ctypes.c_uint64),
                ("numa_node", ctypes.c_int32), ("threads", ctypes.c_uint32), ("threads_on_node", ctypes.c_uint32),
                ("pad_", ctypes.c_uint32)]


def loop_run(handle, frames, lens, total, rx_ifindex=1, slot=192, chunk=65536, chunks=8, producers=2,
             consumers=2, digest=False, stats=None, inflight=2, dma=0, rx_ifname=None, tx_ifname=None, idle_ms=0):
    """hfv_loop_run on ctx handle `handle` (None only with a host stage, debug_loop_host_stage)."""
    import numpy as np
    if frames is not None:
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
    cfg = LoopConfig(frames=frames.ctypes.data if frames is not None else None,
                     lens=lens.ctypes.data if lens is not None else None,
                     n_frames=frames.shape[0] if frames is not None else 0,
                     frame_stride=frames.shape[1] if frames is not None else 0, rx_ifindex=rx_ifindex, slot=slot,
                     chunk=chunk, chunks=chunks, total=total, producers=producers, consumers=consumers,
                     digest=1 if digest else 0, inflight=inflight, dma=int(dma), stats=_ptr(stats),
                     rx_ifname=rx_ifname.encode() if rx_ifname else None,
                     tx_ifname=tx_ifname.encode() if tx_ifname else None, idle_ms=idle_ms)
    st = LoopStats()
    _check(lib().hfv_loop_run(handle, ctypes.byref(cfg), ctypes.byref(st)))
    return {"rx": st.rx_pkts, "tx": st.tx_pkts, "tx_bytes": st.tx_bytes, "drop": st.drop_pkts,
            "tx_digest": st.tx_digest, "verdicts": list(st.verdict_pkts), "seconds": st.seconds,
            "gpu_busy_s": st.gpu_busy_s, "gpu_wait_s": st.gpu_wait_s, "producer_busy_s": st.producer_busy_s,
            "consumer_busy_s": st.consumer_busy_s, "rx_truncated": st.rx_truncated, "tx_errors": st.tx_errors,
            "numa_node": st.numa_node, "threads": st.threads, "threads_on_node": st.threads_on_node}


# Test-only host router stage for hfv_loop_run (see hfv_loop.cpp): fn(frames, slot, len,
# ingress_ifindex, n, action, verdict, egress) on raw pointers; keep the returned object alive.
LOOP_HOST_STAGE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)


def debug_loop_host_stage(fn):
    """Install fn (a LOOP_HOST_STAGE) as hfv_loop_run's router stage, None to remove it."""
    L = lib()
    L.hfv_debug_loop_host_stage.argtypes = [LOOP_HOST_STAGE, ctypes.c_void_p]
    L.hfv_debug_loop_host_stage.restype = ctypes.c_int
    _check(L.hfv_debug_loop_host_stage(fn if fn is not None else LOOP_HOST_STAGE(), None))


def loop_frame_digest(frame: bytes, egress: int) -> int:
    """The digest hfv_loop_run sums over transmitted frames (hfv_loop.cpp frame_hash)."""
    M = (1 << 64) - 1
    n = len(frame)
    h = 0x9E3779B97F4A7C15 ^ ((egress & 0xFFFFFFFF) << 32) ^ n
    i = 0
    while i + 8 <= n:
        h = ((h ^ int.from_bytes(frame[i:i + 8], "little")) * 0xBF58476D1CE4E5B9) & M
        h ^= h >> 29
        i += 8
    h = ((h ^ int.from_bytes(frame[i:], "little")) * 0x94D049BB133111EB) & M
    return h ^ (h >> 31)


class Ctx:
    """One per GPU (hfv_ctx).  Mirrors the br-loader key commands and the XDP verify step."""

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        _check(lib().hfv_ctx_create(device, ctypes.byref(self._h)))
        self.device = device

    def close(self):
        if self._h:
            lib().hfv_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def numa_node(self):
        """NUMA node of this GPU (-1 if unknown)."""
        return lib().hfv_ctx_numa_node(self._h)

    def numa_cpus(self):
        """CPUs of this GPU's NUMA node that this process may run on (all allowed CPUs if the
        node is unknown): where a per-GPU host feeder thread belongs."""
        allowed = os.sched_getaffinity(0)
        node = self.numa_node()
        if node < 0:
            return sorted(allowed)
        try:
            txt = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
        except OSError:
            return sorted(allowed)
        cpus = set()
        for part in txt.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        return sorted(cpus & allowed) or sorted(allowed)

    @property
    def stream(self):
        return lib().hfv_ctx_stream(self._h)

    def set_keysel(self, keysel):
        _check(lib().hfv_ctx_set_keysel(self._h, keysel))

    def set_record_layout(self, inf_off, hf_off):
        _check(lib().hfv_ctx_set_record_layout(self._h, inf_off, hf_off))

    def synchronize(self):
        _check(lib().hfv_ctx_synchronize(self._h))

    # key table (br-loader key add / remove)
    def key_add(self, index, key: bytes):
        _check(lib().hfv_key_add(self._h, index, bytes(key)))

    def key_add_b64(self, index, b64: str):
        _check(lib().hfv_key_add_b64(self._h, index, b64.encode()))

    def key_set_hop_key(self, index, hk: bytes):
        _check(lib().hfv_key_set_hop_key(self._h, index, bytes(hk)))

    def key_remove(self, index):
        _check(lib().hfv_key_remove(self._h, index))

    def key_get(self, index) -> bytes:
        out = ctypes.create_string_buffer(192)
        _check(lib().hfv_key_get(self._h, index, out))
        return out.raw

    def key_add_batch(self, first, keys: bytes):
        assert len(keys) % 16 == 0
        _check(lib().hfv_key_add_batch(self._h, first, bytes(keys), len(keys) // 16))

    # data path (device buffers)
    def verify_records(self, recs, n, pass_bits, stride=REC_SIZE, stream=None):
        _check(lib().hfv_verify_records(self._h, _ptr(recs), stride, n, _ptr(pass_bits), _stream(stream)))

    def verify_records_timed(self, recs, n, pass_bits, stride=REC_SIZE, stream=None):
        """Launch, wait, and return the kernel's own execution time in ms (dispatch events)."""
        ms = ctypes.c_float()
        _check(lib().hfv_verify_records_timed(self._h, _ptr(recs), stride, n, _ptr(pass_bits), _stream(stream),
                                              ctypes.byref(ms)))
        return ms.value

    def verify_batches(self, batches, stream=None):
        """hfv_verify_batches: every batch of the list ([(recs, n, pass_bits[, stride]), ...] or a
        service_batches array) in one stream-ordered launch (64 batches per launch)."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        _check(lib().hfv_verify_batches(self._h, arr, len(arr), _stream(stream)))

    def verify_batches_fn(self, batches, stream=None):
        """verify_batches as a prepared zero-argument call (one foreign-function call per use)."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        f, h, n, st = lib().hfv_verify_batches, self._h, len(arr), _stream(stream)

        def run():
            rc = f(h, arr, n, st)
            if rc:
                _check(rc)
        return run

    def batches_shader_mhz(self):
        """Diagnostic: block 0's shader clock over the last verify_batches launch (s_memtime
        against the 100 MHz s_memrealtime), or None."""
        v = (ctypes.c_uint64 * 4)()
        L = lib()
        if not hasattr(L, "hfv_debug_batches_clock"):
            return None
        L.hfv_debug_batches_clock.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        if L.hfv_debug_batches_clock(self._h, v, 4) != 0:
            return None
        t0, r0, t1, r1 = (int(x) for x in v)
        return (t1 - t0) / ((r1 - r0) / 100.0) if r1 > r0 and t1 > t0 else None

    def batches_block_span(self, grid):
        """Diagnostic: per block of the last timed verify_batches launch, (entered, finished) in
        us after the earliest entry; None if unavailable."""
        v = (ctypes.c_uint64 * (4 + 2 * 1024))()
        L = lib()
        L.hfv_debug_batches_clock.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        if L.hfv_debug_batches_clock(self._h, v, len(v)) != 0:
            return None
        st = [int(v[4 + k]) for k in range(grid)]
        fin = [int(v[4 + 1024 + k]) for k in range(grid)]
        t0 = min(st)
        return [((a - t0) / 100.0, (b - t0) / 100.0) for a, b in zip(st, fin)]

    def stream_read_ms(self, bufs, stream=None):
        """Diagnostic (hfv_debug_stream_read): one dense non-temporal read of the device tensors
        `bufs` (<= 64); returns its kernel time in ms."""
        L = lib()
        L.hfv_debug_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
        ptrs = (ctypes.c_void_p * len(bufs))(*[_ptr(b) for b in bufs])
        sizes = (ctypes.c_size_t * len(bufs))(*[b.numel() * b.element_size() for b in bufs])
        ms = ctypes.c_float(0.0)
        _check(L.hfv_debug_stream_read(self._h, ptrs, sizes, len(bufs), _stream(stream), ctypes.byref(ms)))
        return ms.value

    def verify_batches_timed(self, batches, stream=None):
        """verify_batches, waited for; returns the launches' execution time in ms."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        ms = ctypes.c_float(0.0)
        _check(lib().hfv_verify_batches_timed(self._h, arr, len(arr), _stream(stream), ctypes.byref(ms)))
        return ms.value

    def verdict_counters(self, recs, n, pass_bits, counters, stride=REC_SIZE, stream=None):
        """record_verdict for the verify-only paths: counters (device u64[256][2]) +=
        [verified, INVALID_HF] per AS-ingress IFID & 0xff (hfv_verdict_counters)."""
        _check(lib().hfv_verdict_counters(self._h, _ptr(recs), stride, n, _ptr(pass_bits), _ptr(counters),
                                          _stream(stream)))

    def describe(self):
        buf = ctypes.create_string_buffer(512)
        _check(lib().hfv_ctx_describe(self._h, buf, 512))
        return buf.value.decode()

    def attach_keymap(self, path):
        _check(lib().hfv_ctx_attach_keymap(self._h, path.encode()))

    def br_set_config(self, cfg):
        _check(lib().hfv_br_set_config(self._h, ctypes.byref(cfg)))

    def attach_brconfig(self, path):
        """Use the pinned router tables at `path` (hfv-loader attach), reloaded when republished."""
        _check(lib().hfv_ctx_attach_brconfig(self._h, path.encode()))

    def br_set_hf_check(self, enable: bool):
        """ENABLE_HF_CHECK on/off (br/CMakeLists.txt:8): off skips the hop-field MAC check."""
        _check(lib().hfv_br_set_hf_check(self._h, 1 if enable else 0))

    def br_set_build_options(self, disabled):
        """HFV_BR_NO_IPV4 | HFV_BR_NO_IPV6 | HFV_BR_NO_SCION_PATH: the reference's build options
        switched off (br/CMakeLists.txt:5-7)."""
        _check(lib().hfv_br_set_build_options(self._h, disabled))

    def br_process(self, pkts, slot, lens, ingress_ifindex, n, action, verdict, egress_ifindex, stats=None,
                   stream=None):
        _check(lib().hfv_br_process(self._h, _ptr(pkts), slot, _ptr(lens), _ptr(ingress_ifindex), n, _ptr(action),
                                    _ptr(verdict), _ptr(egress_ifindex), _ptr(stats), _stream(stream)))

    def br_process_host(self, frames, slot, lens, ingress_ifindex, n, action, verdict, egress_ifindex, stats=None,
                        window=0):
        """Config 5: numpy host arrays in, results in place (hfv_br_process_host)."""
        _check(lib().hfv_br_process_host(self._h, _ptr(frames), slot, _ptr(lens), _ptr(ingress_ifindex), n, window,
                                         _ptr(action), _ptr(verdict), _ptr(egress_ifindex), _ptr(stats)))

    def loop_run(self, frames, lens, total, **kw):
        """Config 5 in one process (hfv_loop_run): `frames` (n x stride uint8) cycled into a
        registered RX ring, the router over each chunk, TX/drop consumers.  dma: 0 zero-copy,
        1 (or True) copies both ways, 2 copies in and the kernel writes its changes back.
        rx_ifname / tx_ifname: packet-socket I/O on those interfaces instead (frames unused).
        Returns a dict."""
        return loop_run(self._h, frames, lens, total, **kw)

    @staticmethod
    def debug_publish_delay(us):
        """Test-only: every key/table publish copy waits behind a `us`-microsecond spin kernel on
        its stream (0 = off)."""
        _check(lib().hfv_debug_publish_delay(ctypes.c_uint32(us)))

    @staticmethod
    def debug_br_grid(blocks):
        """Test-only: cap k_br_process launches at `blocks` blocks (0 = default geometry)."""
        _check(lib().hfv_debug_br_grid(ctypes.c_uint(blocks)))

    @staticmethod
    def debug_br_split(frames):
        """Test-only: split counting k_br_process launches into pieces of at most `frames`
        frames (0 = only where the 32-bit block counters could overflow)."""
        _check(lib().hfv_debug_br_split(ctypes.c_size_t(frames)))

    def host_register(self, buf):
        _check(lib().hfv_host_register(self._h, _ptr(buf), buf.nbytes))

    def host_unregister(self, buf):
        _check(lib().hfv_host_unregister(self._h, _ptr(buf)))

    def br_process_timed(self, pkts, slot, lens, ingress_ifindex, n, action, verdict, egress_ifindex, stats=None,
                         stream=None):
        ms = ctypes.c_float(0.0)
        _check(lib().hfv_br_process_timed(self._h, _ptr(pkts), slot, _ptr(lens), _ptr(ingress_ifindex), n,
                                          _ptr(action), _ptr(verdict), _ptr(egress_ifindex), _ptr(stats),
                                          _stream(stream), ctypes.byref(ms)))
        return ms.value

    def verify_macinputs(self, mi, expected, n, pass_bits, key_index=None, stream=None):
        _check(lib().hfv_verify_macinputs(self._h, _ptr(mi), _ptr(expected), _ptr(key_index), n, _ptr(pass_bits),
                                          _stream(stream)))

    def cmac_tags(self, mi, n, tags, key_index=None, stream=None):
        _check(lib().hfv_cmac_tags(self._h, _ptr(mi), _ptr(key_index), n, _ptr(tags), _stream(stream)))

    def expand_keys(self, keys, n, out, stream=None):
        _check(lib().hfv_expand_keys(self._h, _ptr(keys), n, _ptr(out), _stream(stream)))

    def gen_records(self, recs, n, seed, first_index=0, stride=REC_SIZE, stream=None):
        _check(lib().hfv_gen_records(self._h, _ptr(recs), stride, n, seed, first_index, _stream(stream)))

    # resident verify service (persistent grid fed through a host descriptor ring)
    def service_start(self, idle_ms=0):
        _check(lib().hfv_service_start(self._h, idle_ms))

    def service_submit(self, recs, n, pass_bits, stride=REC_SIZE):
        """Post one batch (device buffers); returns its ticket."""
        t = ctypes.c_uint64()
        _check(lib().hfv_service_submit(self._h, _ptr(recs), stride, n, _ptr(pass_bits), ctypes.byref(t)))
        return t.value

    @staticmethod
    def service_batches(batches):
        """A struct hfv_batch array for service_submitv, built once (batches = [(recs, n,
        pass_bits[, stride]), ...]): posting it then costs one C call."""
        arr = (HfvBatch * len(batches))()
        for i, b in enumerate(batches):
            recs, n, bits = b[0], b[1], b[2]
            arr[i].recs, arr[i].n, arr[i].pass_bits = _ptr(recs), n, _ptr(bits)
            arr[i].stride = b[3] if len(b) > 3 else REC_SIZE
        return arr

    def service_submitv(self, batches):
        """Post several batches in one call (a list as for service_batches, or its result);
        starts the service if needed, launching its grid after the batches are in the ring.
        Returns their tickets."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        t = ctypes.c_uint64()
        _check(lib().hfv_service_submitv(self._h, arr, len(arr), ctypes.byref(t)))
        return list(range(t.value, t.value + len(arr)))

    def service_run(self, batches):
        """One-shot: the batches on a fresh grid with the stop posted behind them; returns
        (tickets, grid lifetime in ms) once every batch is verified (hfv_service_run)."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        t = ctypes.c_uint64()
        ms = ctypes.c_float(0.0)
        _check(lib().hfv_service_run(self._h, arr, len(arr), ctypes.byref(t), ctypes.byref(ms)))
        return list(range(t.value, t.value + len(arr))), ms.value

    def service_run_async(self, batches):
        """hfv_service_run without the wait: the grid is launched with the batches and the stop
        behind them; a device synchronize (or service_wait) covers it, service_stop reaps it and
        returns its lifetime.  Returns the tickets."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        t = ctypes.c_uint64()
        _check(lib().hfv_service_run_async(self._h, arr, len(arr), ctypes.byref(t)))
        return list(range(t.value, t.value + len(arr)))

    def service_run_async_fn(self, batches):
        """service_run_async as a prepared zero-argument call (the C function, the ctx handle, the
        batch array and the ticket out-parameter bound once): what a timed loop calls, so that
        the Python side of each call is one foreign-function call and a return-code check."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        f = lib().hfv_service_run_async
        h, n, t = self._h, len(arr), ctypes.c_uint64()
        tp = ctypes.byref(t)

        def run():
            rc = f(h, arr, n, tp)
            if rc:
                _check(rc)
        return run

    def service_poll(self, ticket):
        rc = lib().hfv_service_poll(self._h, ticket)
        if rc < 0:
            _check(rc)
        return bool(rc)

    def service_wait(self, ticket, timeout_ms=-1):
        _check(lib().hfv_service_wait(self._h, ticket, timeout_ms))

    def service_stop(self):
        """Finish posted batches, stop the grid; returns its lifetime in ms."""
        ms = ctypes.c_float(0.0)
        _check(lib().hfv_service_stop(self._h, ctypes.byref(ms)))
        return ms.value

    def service_shader_mhz(self):
        """Diagnostic: block 0's shader clock over the last service grid's life (s_memtime
        against the 100 MHz s_memrealtime), or None."""
        clk = (ctypes.c_uint64 * (2 * SVC_RING + 4))()
        L = lib()
        L.hfv_debug_service_clocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        if L.hfv_debug_service_clocks(self._h, clk) != 0:
            return None
        t0, r0, t1, r1 = (int(x) for x in clk[SVC_RING:SVC_RING + 4])
        return (t1 - t0) / ((r1 - r0) / 100.0) if r1 > r0 and t1 > t0 else None

    def service_weights(self):
        """Diagnostic: the block weights the next service grid will use (per XCD 0..7, then
        block 0's), in 1/1024 of an equal share (svc_balance, hfv_api.cpp)."""
        w = (ctypes.c_uint32 * 9)()
        L = lib()
        L.hfv_debug_service_weights.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        if L.hfv_debug_service_weights(self._h, w) != 0:
            return None
        return [int(x) for x in w]

    def service_timeline(self, nbatches):
        """Diagnostic: per batch of the last grid, (relay published, block 0 loaded) in us
        after block 0's loop start, and the grid's loop span."""
        clk = (ctypes.c_uint64 * (2 * SVC_RING + 4))()
        L = lib()
        L.hfv_debug_service_clocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        if L.hfv_debug_service_clocks(self._h, clk) != 0:
            return None
        r0, r1 = int(clk[SVC_RING + 1]), int(clk[SVC_RING + 3])
        us = lambda t: round((int(t) - r0) / 100.0, 2) if t else None   # noqa: E731
        return {"loop_us": us(r1), "relay_us": [us(clk[SVC_RING + 4 + i]) for i in range(nbatches + 1)],
                "load_us": [us(clk[i]) for i in range(nbatches + 1)]}

    def service_relay(self):
        """Diagnostic: the last service grid's relay counters (hfv_debug_service_relay) -- how the
        host link behaved for it: the PCIe round trip probed at grid start and the longest host
        read (us), host reads, descriptors relayed beyond the inline ones, completions forwarded,
        waits of a block for a descriptor, descriptors in the kernel arguments."""
        v = (ctypes.c_uint64 * 8)()
        L = lib()
        if not hasattr(L, "hfv_debug_service_relay"):   # an older build (A/B runs)
            return None
        L.hfv_debug_service_relay.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        if L.hfv_debug_service_relay(self._h, v) != 0:
            return None
        x = [int(t) for t in v]
        return {"probe_rtt_us": round(x[0] / 100.0, 2), "host_reads": x[1],
                "read_rtt_mean_us": round(x[2] / 100.0 / x[1], 2) if x[1] else None,
                "read_rtt_max_us": round(x[3] / 100.0, 2), "relayed": x[4], "forwarded": x[5],
                "block_waits": x[6], "inline": x[7]}

    @staticmethod
    def debug_relay_delay(us):
        """Test-only: every host read of later service grids' relay wave takes `us` microseconds
        longer (a slow PCIe link); 0 = off."""
        L = lib()
        L.hfv_debug_relay_delay.argtypes = [ctypes.c_uint32]
        _check(L.hfv_debug_relay_delay(us))

    def service_set_timing(self, enable):
        """Launch later service grids with (True) or without the dispatch timing events."""
        _check(lib().hfv_service_set_timing(self._h, 1 if enable else 0))

    def service_set_grid(self, blocks):
        """Later service grids use `blocks` blocks (0: one per CU) -- for ranks sharing one GPU."""
        _check(lib().hfv_service_set_grid(self._h, int(blocks)))

    def feed_loop(self, batches, depth=4):
        """Diagnostic (hfv_debug_feed_loop): INTEGRATION.md section 2's data-plane loop run in C --
        per batch one hfv_service_submit, hfv_service_wait on the ticket `depth` batches back --
        returns its host wall time in seconds."""
        arr = batches if isinstance(batches, ctypes.Array) else self.service_batches(batches)
        L = lib()
        L.hfv_debug_feed_loop.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint64)]
        ns = ctypes.c_uint64(0)
        _check(L.hfv_debug_feed_loop(self._h, arr, len(arr), depth, ctypes.byref(ns)))
        return ns.value * 1e-9

    @property
    def service_running(self):
        return bool(lib().hfv_service_running(self._h))

    # host buffers (pinned staging, H2D/kernel/D2H overlapped)
    def verify_records_host(self, recs, n, pass_bits, stride=REC_SIZE):
        _check(lib().hfv_verify_records_host(self._h, _ptr(recs), stride, n, _ptr(pass_bits)))


# ---- full BR path (config 4): router tables --------------------------------------------------

AF_INET, AF_INET6 = 2, 10
BR_MAX_IFACES, BR_MAX_ROUTES, BR_MAX_TXPORTS, BR_COUNTERS, BR_STATS_IFINDEX = 16, 64, 128, 11, 64


class BrIntIface(ctypes.Structure):
    _fields_ = [("ifindex", ctypes.c_uint32), ("family", ctypes.c_uint32), ("addr", ctypes.c_uint8 * 16),
                ("port", ctypes.c_uint8 * 2), ("pad", ctypes.c_uint8 * 2)]


class BrIngress(ctypes.Structure):
    _fields_ = [("ifindex", ctypes.c_uint32), ("family", ctypes.c_uint32), ("addr", ctypes.c_uint8 * 16),
                ("port", ctypes.c_uint8 * 2), ("pad", ctypes.c_uint8 * 2), ("ifid", ctypes.c_uint32)]


class BrEgress(ctypes.Structure):
    _fields_ = [("ifid", ctypes.c_uint32), ("fwd_external", ctypes.c_uint32), ("family", ctypes.c_uint32),
                ("remote", ctypes.c_uint8 * 16), ("local", ctypes.c_uint8 * 16),
                ("remote_port", ctypes.c_uint8 * 2), ("local_port", ctypes.c_uint8 * 2)]


class BrRoute(ctypes.Structure):
    _fields_ = [("family", ctypes.c_uint32), ("prefix", ctypes.c_uint8 * 16), ("prefix_len", ctypes.c_uint32),
                ("ret", ctypes.c_int32), ("ifindex", ctypes.c_uint32), ("smac", ctypes.c_uint8 * 6),
                ("dmac", ctypes.c_uint8 * 6)]


class BrConfig(ctypes.Structure):
    """struct hfv_br_config: the reference's BPF maps (int_iface_map, ingress_map, egress_map,
    tx_port_map) plus the static next-hop table that replaces bpf_fib_lookup."""
    _fields_ = [("n_int_ifaces", ctypes.c_uint32), ("n_ingress", ctypes.c_uint32), ("n_egress", ctypes.c_uint32),
                ("n_routes", ctypes.c_uint32), ("n_tx_ports", ctypes.c_uint32),
                ("int_ifaces", BrIntIface * BR_MAX_IFACES), ("ingress", BrIngress * BR_MAX_IFACES),
                ("egress", BrEgress * BR_MAX_IFACES), ("routes", BrRoute * BR_MAX_ROUTES),
                ("tx_ports", ctypes.c_uint32 * BR_MAX_TXPORTS)]

    @staticmethod
    def _ip(addr):
        import ipaddress
        a = ipaddress.ip_address(addr)
        b = a.packed + bytes(16 - len(a.packed))
        return (AF_INET if a.version == 4 else AF_INET6), (ctypes.c_uint8 * 16)(*b)

    @staticmethod
    def _port(p):
        return (ctypes.c_uint8 * 2)(p >> 8, p & 0xff)

    @staticmethod
    def _mac(m):
        return (ctypes.c_uint8 * 6)(*bytes.fromhex(m.replace(":", "")))

    def add_int_iface(self, ifindex, addr, port):
        e = self.int_ifaces[self.n_int_ifaces]
        e.ifindex = ifindex
        e.family, e.addr = self._ip(addr)
        e.port = self._port(port)
        self.n_int_ifaces += 1

    def add_ingress(self, ifindex, addr, port, ifid):
        e = self.ingress[self.n_ingress]
        e.ifindex = ifindex
        e.family, e.addr = self._ip(addr)
        e.port = self._port(port)
        e.ifid = ifid
        self.n_ingress += 1

    def add_egress_link(self, ifid, local, local_port, remote, remote_port):
        e = self.egress[self.n_egress]
        e.ifid, e.fwd_external = ifid, 1
        e.family, e.remote = self._ip(remote)
        _, e.local = self._ip(local)
        e.remote_port, e.local_port = self._port(remote_port), self._port(local_port)
        self.n_egress += 1

    def add_egress_sibling(self, ifid, addr, port):
        e = self.egress[self.n_egress]
        e.ifid, e.fwd_external = ifid, 0
        e.family, e.remote = self._ip(addr)
        e.remote_port = self._port(port)
        self.n_egress += 1

    def add_route(self, prefix, prefix_len, ifindex, smac, dmac, ret=0):
        e = self.routes[self.n_routes]
        e.family, e.prefix = self._ip(prefix)
        e.prefix_len, e.ret, e.ifindex = prefix_len, ret, ifindex
        e.smac, e.dmac = self._mac(smac), self._mac(dmac)
        self.n_routes += 1

    def add_tx_port(self, ifindex):
        self.tx_ports[self.n_tx_ports] = ifindex
        self.n_tx_ports += 1


class BrIfAddr(ctypes.Structure):
    """struct hfv_br_ifaddr: one address of the getifaddrs view."""
    _fields_ = [("ifname", ctypes.c_char * 16), ("ifindex", ctypes.c_uint32), ("family", ctypes.c_uint32),
                ("addr", ctypes.c_uint8 * 16)]


class BrNextHop(ctypes.Structure):
    """struct hfv_br_next_hop: one static FIB entry (replaces bpf_fib_lookup)."""
    _fields_ = [("family", ctypes.c_uint32), ("prefix", ctypes.c_uint8 * 16), ("prefix_len", ctypes.c_uint32),
                ("ifname", ctypes.c_char * 16), ("smac", ctypes.c_uint8 * 6), ("dmac", ctypes.c_uint8 * 6),
                ("ret", ctypes.c_int32)]


def br_config_load(toml_path, if_addrs=None, ifindex_of=None, next_hops=()):
    """br-loader's loadConfig + initializeMaps in the C library (hfv_br_config_load).
    if_addrs: {ip: ifname} (None: this namespace); ifindex_of: ifname -> ifindex for if_addrs;
    next_hops: (prefix, prefix_len, ifname, smac, dmac[, ret]).
    Returns (rc, BrConfig, self, listing, diag)."""
    ifs = None
    n_ifs = 0
    if if_addrs is not None:
        ifs = (BrIfAddr * max(1, len(if_addrs)))()
        for k, (ip, name) in enumerate(if_addrs.items()):
            fam, a = BrConfig._ip(str(ip))
            ifs[k].ifname, ifs[k].family, ifs[k].addr = name.encode(), fam, a
            ifs[k].ifindex = ifindex_of(name) if ifindex_of else 0
        n_ifs = len(if_addrs)
    hops = (BrNextHop * max(1, len(next_hops)))()
    for k, h in enumerate(next_hops):
        prefix, plen, ifname, smac, dmac = h[:5]
        hops[k].family, hops[k].prefix = BrConfig._ip(prefix)
        hops[k].prefix_len, hops[k].ifname = plen, ifname.encode()
        hops[k].smac, hops[k].dmac = BrConfig._mac(smac), BrConfig._mac(dmac)
        hops[k].ret = h[5] if len(h) > 5 else 0
    cfg = BrConfig()
    selfb, lst, diag = (ctypes.create_string_buffer(256), ctypes.create_string_buffer(16384),
                        ctypes.create_string_buffer(16384))
    rc = lib().hfv_br_config_load(str(toml_path).encode(), ifs, n_ifs, hops, len(next_hops), ctypes.byref(cfg),
                                  selfb, 256, lst, 16384, diag, 16384)
    return rc, cfg, selfb.value.decode(), lst.value.decode(), diag.value.decode()


def brconfig_path(br: str) -> str:
    buf = ctypes.create_string_buffer(4096)
    _check(lib().hfv_brconfig_path(br.encode(), buf, 4096))
    return buf.value.decode()


def brconfig_publish(path: str, cfg):
    _check(lib().hfv_brconfig_publish(path.encode(), ctypes.byref(cfg)))


def brconfig_read(path: str):
    cfg = BrConfig()
    _check(lib().hfv_brconfig_read(path.encode(), ctypes.byref(cfg)))
    return cfg


BR_NO_IPV4, BR_NO_IPV6, BR_NO_SCION_PATH = 1, 2, 4


def br_config_check_options(cfg, disabled):
    _check(lib().hfv_br_config_check_options(ctypes.byref(cfg), disabled))


def brconfig_publish_opts(path: str, cfg, disabled):
    _check(lib().hfv_brconfig_publish_opts(path.encode(), ctypes.byref(cfg), disabled))


def brconfig_detach(path: str):
    """`hfv-loader detach`: attached data planes pass every frame from their next batch."""
    _check(lib().hfv_brconfig_detach(path.encode()))


# enum verdict (br/src/bpf/common.h:55-70)
VERDICT = {"ABORT": 0, "SCION_FORWARD": 12, "PARSE_ERROR": 17, "NOT_SCION": 26, "NOT_IMPLEMENTED": 34,
           "NO_INTERFACE": 41, "UNDERLAY_MISMATCH": 50, "ROUTER_ALERT": 58, "FIB_LKUP_DROP": 65,
           "FIB_LKUP_PASS": 74, "INVALID_HF": 81}


# ---- pinned key map (bpffs mac_key_map analogue) --------------------------------------------

def keymap_path(br: str) -> str:
    buf = ctypes.create_string_buffer(4096)
    _check(lib().hfv_keymap_path(br.encode(), buf, 4096))
    return buf.value.decode()


def keymap_update(path: str, index: int, hop_key_bytes: bytes):
    _check(lib().hfv_keymap_update(path.encode(), index, bytes(hop_key_bytes)))


def keymap_erase(path: str, index: int):
    _check(lib().hfv_keymap_erase(path.encode(), index))


KEYMAP_SLOTS, KEYMAP_HASH8 = 0, 1


def keymap_create(path: str, mode=KEYMAP_SLOTS):
    _check(lib().hfv_keymap_create_mode(path.encode(), mode))


def keymap_mode(path: str) -> int:
    rc = lib().hfv_keymap_mode(path.encode())
    _check(min(rc, 0))
    return rc


def keymap_list(path: str):
    """Every entry of the map, index ascending: [(index, 192-byte hop_key)]."""
    cap = MAX_KEYS + 8
    idx = (ctypes.c_uint32 * cap)()
    keys = ctypes.create_string_buffer(192 * cap)
    n = ctypes.c_size_t(0)
    _check(lib().hfv_keymap_list(path.encode(), idx, keys, cap, ctypes.byref(n)))
    return [(int(idx[i]), keys.raw[192 * i:192 * i + 192]) for i in range(min(n.value, cap))]


def keymap_read(path: str):
    """(dict slot -> 192-byte hop_key, for the occupied slots)"""
    slots = ctypes.create_string_buffer(192 * MAX_KEYS)
    valid = (ctypes.c_uint32 * 8)()
    _check(lib().hfv_keymap_read(path.encode(), slots, valid))
    return {k: slots.raw[192 * k:192 * k + 192] for k in range(MAX_KEYS) if (valid[k >> 5] >> (k & 31)) & 1}


# ---- batch sharding across GPUs ------------------------------------------------

def host_array(shape, dtype):
    """Zero-filled numpy array in page-aligned anonymous memory, suitable for Ctx.host_register
    (an RX ring, or the per-frame metadata arrays of br_process_host)."""
    import mmap
    import numpy as np
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    buf = mmap.mmap(-1, max(1, count * dt.itemsize))
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


def statsmap_path(br: str) -> str:
    buf = ctypes.create_string_buffer(4096)
    _check(lib().hfv_statsmap_path(br.encode(), buf, 4096))
    return buf.value.decode()


def statsmap_add(path: str, stats):
    """Add a [64, 2, 11] u64 counter block (hfv_br_process stats) to the pinned stats map."""
    import numpy as np
    a = np.ascontiguousarray(np.asarray(stats.cpu().numpy() if hasattr(stats, "cpu") else stats).view(np.uint64))
    assert a.size == BR_STATS_IFINDEX * 2 * BR_COUNTERS
    _check(lib().hfv_statsmap_add(path.encode(), a.ctypes.data))


def statsmap_read(path: str):
    import numpy as np
    a = np.zeros((BR_STATS_IFINDEX, 2, BR_COUNTERS), dtype=np.uint64)
    _check(lib().hfv_statsmap_read(path.encode(), a.ctypes.data))
    return a


def shard_range(n, world, rank):
    """Contiguous slice of n packets for `rank`, cut on 64-packet boundaries so each rank's
    verdict bitmap is a whole-word slice of the global bitmap."""
    words = (n + 63) // 64
    w0 = words * rank // world
    w1 = words * (rank + 1) // world
    return min(64 * w0, n), min(64 * w1, n)


def bits_to_bool(words, n):
    """Expand a uint64 verdict bitmap (numpy) to a bool array of n entries."""
    import numpy as np
    b = np.unpackbits(np.ascontiguousarray(words).view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


__all__ = [n for n in dir() if not n.startswith("_")]
if sys.version_info < (3, 8):  # pragma: no cover
    raise RuntimeError("python >= 3.8 required")
