"""Host-side mirror of the reference's verify API over the C ABI.

Loads ``firedancer_amd/libfdgpu_ed25519.so`` (HIP kernels + C runtime, see
include/fd_ed25519_gpu.h) with ctypes.  The module-level functions mirror
the reference's ``fd_ed25519_verify`` / ``fd_ed25519_verify_batch_single_msg``
(src/ballet/ed25519/fd_ed25519.h:96-130): same argument meaning, same
FD_ED25519_* result codes.  :class:`Engine` is the batch API used by the
verify-stage offload and the bench.

There is no CPU fallback: if the shared library or the GPU is missing,
every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FDGPU_LIB") or os.path.join(PKG_DIR, "libfdgpu_ed25519.so")

FD_ED25519_SUCCESS = 0
FD_ED25519_ERR_SIG = -1
FD_ED25519_ERR_PUBKEY = -2
FD_ED25519_ERR_MSG = -3
SEMANTICS_AVX512 = 0
SEMANTICS_REF = 1

DESC_DTYPE = np.dtype([("payload_off", "<u4"), ("sig_base", "<u4"), ("payload_sz", "<u2"),
                       ("message_off", "<u2"), ("acct_addr_off", "<u2"), ("signature_off", "u1"),
                       ("sig_cnt", "u1")])
assert DESC_DTYPE.itemsize == 16
RAW_DTYPE = np.dtype([("payload_off", "<u4"), ("sig_base", "<u4"), ("payload_sz", "<u2"), ("sig_lanes", "u1"),
                      ("_pad", "u1", (5,))])
assert RAW_DTYPE.itemsize == 16
FDGPU_ERR_PARSE = -16
FDGPU_ERR_OVERRUN = -17
TXN_IMG_STRIDE = 864

# every symbol include/fd_ed25519_gpu.h declares
EXPORTS = ("fd_ed25519_verify", "fd_ed25519_verify_batch_single_msg", "fd_ed25519_strerror",
           "fdgpu_ed25519_ctx_new", "fdgpu_ed25519_ctx_delete", "fdgpu_ed25519_verify_txns_device",
           "fdgpu_ed25519_verify_txns_host", "fdgpu_txn_parse_device", "fdgpu_ed25519_verify_raw_device",
           "fdgpu_ed25519_verify_raw_host", "fdgpu_ed25519_submit", "fdgpu_ed25519_flush",
           "fdgpu_ed25519_poll", "fdgpu_ed25519_submit_raw", "fdgpu_ed25519_poll_raw", "fdgpu_ed25519_submit_raw_ref",
           "fdgpu_host_alloc", "fdgpu_host_free", "fdgpu_host_register", "fdgpu_host_unregister", "fdgpu_device_numa_node",
           "fdgpu_ed25519_submit_raw_gather", "fdgpu_ed25519_submit_raw_gather_chk", "fdgpu_ed25519_gather",
           "fdgpu_ed25519_gathered", "fdgpu_ed25519_gather_launched", "fdgpu_ed25519_gather_wait", "fdgpu_host_dev_ptr", "fdgpu_host_register_shared",
           "fdgpu_ed25519_reserve_gather_cus", "fdgpu_ed25519_reserve_cus", "fdgpu_ed25519_set_cu_exclusive", "fdgpu_ed25519_get_cu_exclusive", "fdgpu_ed25519_set_lat_share", "fdgpu_ed25519_gather_stats", "fdgpu_ed25519_phase_stats", "fdgpu_ed25519_prepare", "fdgpu_ed25519_submit_raw_gather_dev", "fdgpu_host_region",
           "fdgpu_ed25519_dropin_init", "fdgpu_debug_set_opts", "fdgpu_debug_gather_pauses",
           "fdgpu_ed25519_pipeline_state", "fdgpu_ed25519_verify_many_host", "fdgpu_sha512_batch_device", "fdgpu_sha512_batch_host", "fdgpu_ed25519_set_timing", "fdgpu_ed25519_set_small_batch_max", "fdgpu_ed25519_kernel_ms", "fdgpu_mad_peak_per_s",
           "fdgpu_ed25519_faulted", "fdgpu_ed25519_debug_fault", "fdgpu_ed25519_slow_count", "fdgpu_ed25519_set_dedup",
           "fdgpu_ed25519_set_record_fp_off", "fdgpu_ed25519_batch_stats", "fdgpu_ed25519_launch_stats", "fdgpu_ed25519_front_remaining", "fdgpu_ed25519_front_batch", "fdgpu_ed25519_verify_txn_ptrs",
           "fdgpu_ed25519_submit_raw_gather_dev_f", "fdgpu_launcher_new", "fdgpu_launcher_delete", "fdgpu_launcher_stats", "fdgpu_ed25519_set_launcher",
           "fdgpu_ed25519_submit_raw_gather_to", "fdgpu_ed25519_set_dedup_seeds", "fdgpu_ed25519_debug_fail_launch",
           "fdgpu_last_error")

_lib = None
_lock = threading.Lock()
_u8p = ctypes.POINTER(ctypes.c_uint8)


def load_library():
    """dlopen the engine.  Raises if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch-ROCm ships its own libamdhip64 with the same SONAME
        # (libamdhip64.so.7).  Load it first so this library binds to that
        # one HIP runtime: torch tensors/streams and the engine then share
        # one runtime (two runtimes in one process do not see each other's
        # streams, and the second fails to enumerate GPUs).
        try:
            import torch  # noqa: F401
            if getattr(torch.version, "hip", None):
                torch.cuda.device_count()
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.fd_ed25519_verify.restype = ctypes.c_int
        L.fd_ed25519_verify.argtypes = [_u8p, ctypes.c_ulong, _u8p, _u8p, ctypes.c_void_p]
        L.fd_ed25519_verify_batch_single_msg.restype = ctypes.c_int
        L.fd_ed25519_verify_batch_single_msg.argtypes = [_u8p, ctypes.c_ulong, _u8p, _u8p, ctypes.c_void_p, ctypes.c_uint8]
        L.fd_ed25519_strerror.restype = ctypes.c_char_p
        L.fd_ed25519_strerror.argtypes = [ctypes.c_int]
        L.fdgpu_ed25519_ctx_new.restype = ctypes.c_void_p
        L.fdgpu_ed25519_ctx_new.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_int]
        L.fdgpu_ed25519_ctx_delete.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_verify_txns_device.restype = ctypes.c_int
        L.fdgpu_ed25519_verify_txns_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                                                      ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.fdgpu_ed25519_verify_txns_host.restype = ctypes.c_int
        L.fdgpu_ed25519_verify_txns_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                                    ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
        L.fdgpu_txn_parse_device.restype = ctypes.c_int
        L.fdgpu_txn_parse_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                             ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
        L.fdgpu_ed25519_verify_raw_device.restype = ctypes.c_int
        L.fdgpu_ed25519_verify_raw_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                                                      ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                                                      ctypes.c_void_p, ctypes.c_void_p]
        L.fdgpu_ed25519_verify_raw_host.restype = ctypes.c_int
        L.fdgpu_ed25519_verify_raw_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                                    ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                                                    ctypes.c_void_p]
        L.fdgpu_ed25519_verify_many_host.restype = ctypes.c_int
        L.fdgpu_ed25519_verify_many_host.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_ulong, ctypes.c_void_p]
        L.fdgpu_sha512_batch_device.restype = ctypes.c_int
        L.fdgpu_sha512_batch_device.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
        L.fdgpu_sha512_batch_host.restype = ctypes.c_int
        L.fdgpu_sha512_batch_host.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p]
        L.fdgpu_ed25519_submit.restype = ctypes.c_int
        L.fdgpu_ed25519_submit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ushort, ctypes.c_ubyte,
                                           ctypes.c_ushort, ctypes.c_ushort, ctypes.c_ubyte, ctypes.c_ulong]
        L.fdgpu_ed25519_flush.restype = ctypes.c_int
        L.fdgpu_ed25519_flush.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_poll.restype = ctypes.c_ulong
        L.fdgpu_ed25519_poll.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int]
        L.fdgpu_ed25519_submit_raw.restype = ctypes.c_int
        L.fdgpu_ed25519_submit_raw.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ushort, ctypes.c_ulong]
        L.fdgpu_ed25519_poll_raw.restype = ctypes.c_ulong
        L.fdgpu_ed25519_poll_raw.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int]
        L.fdgpu_ed25519_set_dedup.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_ulong]
        L.fdgpu_ed25519_set_record_fp_off.restype = ctypes.c_int
        L.fdgpu_ed25519_set_record_fp_off.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.fdgpu_ed25519_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.fdgpu_ed25519_set_cu_exclusive.restype = ctypes.c_int
        L.fdgpu_ed25519_set_cu_exclusive.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.fdgpu_ed25519_set_lat_share.restype = ctypes.c_int
        L.fdgpu_ed25519_set_lat_share.argtypes = [ctypes.c_void_p, ctypes.c_uint]
        L.fdgpu_ed25519_front_batch.restype = ctypes.c_int
        L.fdgpu_ed25519_front_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulong),
                                                ctypes.POINTER(ctypes.c_ulong), ctypes.POINTER(ctypes.c_int)]
        L.fdgpu_ed25519_set_small_batch_max.restype = ctypes.c_ulong
        L.fdgpu_ed25519_set_small_batch_max.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
        L.fdgpu_ed25519_kernel_ms.restype = ctypes.c_float
        L.fdgpu_ed25519_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.fdgpu_ed25519_pipeline_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.fdgpu_ed25519_verify_txn_ptrs.restype = ctypes.c_int
        L.fdgpu_ed25519_verify_txn_ptrs.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_ulong, ctypes.c_void_p]
        L.fdgpu_ed25519_faulted.restype = ctypes.c_int
        L.fdgpu_ed25519_faulted.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_debug_fault.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_slow_count.restype = ctypes.c_ulong
        L.fdgpu_ed25519_slow_count.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_submit_raw_ref.restype = ctypes.c_int
        L.fdgpu_ed25519_submit_raw_ref.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ushort,
                                                   ctypes.c_ulong]
        L.fdgpu_ed25519_submit_raw_gather.restype = ctypes.c_int
        L.fdgpu_ed25519_submit_raw_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_ushort, ctypes.c_ushort, ctypes.c_ushort, ctypes.c_ulong]
        L.fdgpu_ed25519_submit_raw_gather_chk.restype = ctypes.c_int
        L.fdgpu_ed25519_submit_raw_gather_chk.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_ushort, ctypes.c_ushort,
                                                          ctypes.c_ushort, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_ulong]
        L.fdgpu_ed25519_gather.restype = ctypes.c_long
        L.fdgpu_ed25519_gather.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_gathered.restype = ctypes.c_ulong
        L.fdgpu_ed25519_gathered.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_gather_launched.restype = ctypes.c_ulong
        L.fdgpu_ed25519_gather_launched.argtypes = [ctypes.c_void_p]
        L.fdgpu_ed25519_gather_wait.restype = ctypes.c_int
        L.fdgpu_ed25519_gather_wait.argtypes = [ctypes.c_void_p]
        L.fdgpu_host_dev_ptr.restype = ctypes.c_void_p
        L.fdgpu_host_dev_ptr.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
        L.fdgpu_ed25519_dropin_init.restype = ctypes.c_int
        L.fdgpu_ed25519_dropin_init.argtypes = [ctypes.c_int, ctypes.c_int]
        L.fdgpu_debug_set_opts.argtypes = [ctypes.c_void_p]
        L.fdgpu_host_alloc.restype = ctypes.c_void_p
        L.fdgpu_host_alloc.argtypes = [ctypes.c_ulong]
        L.fdgpu_host_free.argtypes = [ctypes.c_void_p]
        L.fdgpu_last_error.restype = ctypes.c_char_p
        _lib = L
        return L


def last_error() -> str:
    return load_library().fdgpu_last_error().decode()


class DebugOpts(ctypes.Structure):
    """fdgpu_debug_opts_t: test / A/B choices for engine contexts created afterwards."""
    _fields_ = [("half", ctypes.c_int), ("half_force_slow", ctypes.c_uint), ("small_batch_max", ctypes.c_long),
                ("dsm_lanes", ctypes.c_int), ("nofold_max", ctypes.c_long), ("gather_no_writeback", ctypes.c_int),
                ("poll_prefetch", ctypes.c_int), ("gather_rpb", ctypes.c_int), ("gather_cu_spread", ctypes.c_int),
                ("cu_exclusive", ctypes.c_int), ("quad_sha", ctypes.c_int)]


def debug_set_opts(half: int = -1, half_force_slow: int = 0, small_batch_max: int = -1, dsm_lanes: int = 0,
                   nofold_max: int = -1, gather_no_writeback: int = 0, poll_prefetch: int = 0,
                   gather_rpb: int = 0, gather_cu_spread: int = 0, cu_exclusive: int = 0, quad_sha: int = 0) -> None:
    """fdgpu_debug_set_opts: the engine path of every context created from now on (tests only; the
    defaults restore the product's choices).  small_batch_max >= 2**63 means "always the latency path"."""
    o = DebugOpts(half=half, half_force_slow=half_force_slow,
                  small_batch_max=min(small_batch_max, 2**63 - 1), dsm_lanes=dsm_lanes, nofold_max=nofold_max,
                  gather_no_writeback=gather_no_writeback, poll_prefetch=poll_prefetch, gather_rpb=gather_rpb,
                  gather_cu_spread=gather_cu_spread, cu_exclusive=cu_exclusive, quad_sha=quad_sha)
    load_library().fdgpu_debug_set_opts(ctypes.byref(o))


def gather_pauses(reset: bool = True, n: int = 512) -> tuple[int, list]:
    """fdgpu_debug_gather_pauses: (how many, [(host ns of the issuing call, ns held on the GPU), ...])."""
    L = load_library()
    L.fdgpu_debug_gather_pauses.restype = ctypes.c_ulong
    L.fdgpu_debug_gather_pauses.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int]
    buf = np.zeros(2 * n, np.uint64)
    tot = int(L.fdgpu_debug_gather_pauses(buf.ctypes.data, n, 1 if reset else 0))
    m = min(tot, n)
    return tot, [(int(buf[2 * i]), int(buf[2 * i + 1])) for i in range(m)]


def debug_reset_opts() -> None:
    load_library().fdgpu_debug_set_opts(None)


def dropin_init(device: int = 0, semantics: int = SEMANTICS_AVX512) -> None:
    """fdgpu_ed25519_dropin_init: device and result-code semantics of the fd_ed25519_verify drop-ins."""
    rc = load_library().fdgpu_ed25519_dropin_init(device, semantics)
    if rc:
        raise RuntimeError(f"fdgpu_ed25519_dropin_init: {rc} {last_error()}")


def _buf(b: bytes):
    a = np.frombuffer(bytes(b) + b"\0", np.uint8)
    return a, a.ctypes.data_as(_u8p)


def fd_ed25519_verify(msg: bytes, sig: bytes, public_key: bytes) -> int:
    """Drop-in for fd_ed25519_verify (fd_ed25519.h:96-101) on the GPU."""
    L = load_library()
    m, mp = _buf(msg); s, sp = _buf(sig); p, pp = _buf(public_key)
    return L.fd_ed25519_verify(mp, len(msg), sp, pp, None)


def fd_ed25519_verify_batch_single_msg(msg: bytes, signatures: bytes, pubkeys: bytes, batch_sz: int) -> int:
    """Drop-in for fd_ed25519_verify_batch_single_msg (fd_ed25519.h:124-130) on the GPU."""
    L = load_library()
    m, mp = _buf(msg); s, sp = _buf(signatures); p, pp = _buf(pubkeys)
    return L.fd_ed25519_verify_batch_single_msg(mp, len(msg), sp, pp, None, batch_sz & 0xff)


def txn_parse_device(d_payload: int, d_raw: int, txn_cnt: int, d_img: int | None, d_fp: int,
                     stream: int | None = None, img_stride: int = TXN_IMG_STRIDE) -> None:
    """Batch fd_txn_parse on the GPU (fdgpu_txn_parse_device), device pointers."""
    rc = load_library().fdgpu_txn_parse_device(d_payload, d_raw, txn_cnt, d_img, img_stride, d_fp, stream)
    if rc:
        raise RuntimeError(f"fdgpu_txn_parse_device: {rc} {last_error()}")


def sha512_batch(msgs, device: int = 0) -> list[bytes]:
    """SHA-512 of each message on the GPU (fdgpu_sha512_batch_host)."""
    L = load_library()
    off = np.zeros(len(msgs), np.uint64)
    sz = np.zeros(len(msgs), np.uint32)
    pos = 0
    for i, m in enumerate(msgs):
        off[i], sz[i] = pos, len(m)
        pos += len(m)
    data = np.frombuffer(b"".join(bytes(m) for m in msgs) + b"\0", np.uint8)
    out = np.zeros((len(msgs), 64), np.uint8)
    rc = L.fdgpu_sha512_batch_host(device, data.ctypes.data, pos, off.ctypes.data, sz.ctypes.data, len(msgs),
                                   out.ctypes.data)
    if rc:
        raise RuntimeError(f"fdgpu_sha512_batch_host: {rc} {last_error()}")
    return [out[i].tobytes() for i in range(len(msgs))]


def raw_records(payload: np.ndarray, off: np.ndarray, sz: np.ndarray):
    """Host staging of a raw-payload batch: (RAW_DTYPE records, total signature lanes)."""
    raw = np.zeros(len(off), RAW_DTYPE)
    raw["payload_off"] = off
    raw["payload_sz"] = sz
    b0 = np.where(np.asarray(sz) > 0, payload[np.minimum(off, len(payload) - 1)], 0)
    lanes = np.where((b0 >= 1) & (b0 <= 16), b0, 0).astype(np.uint32)
    raw["sig_lanes"] = lanes
    raw["sig_base"] = np.concatenate([[0], np.cumsum(lanes)[:-1]]).astype(np.uint32) if len(off) else []
    return raw, int(lanes.sum())


def host_register(buf: np.ndarray) -> None:
    """fdgpu_host_register: page-lock and map a host array for the GPU (zero-copy intake); keep it alive."""
    L = load_library()
    if L.fdgpu_host_register(ctypes.c_void_p(buf.ctypes.data), ctypes.c_ulong(buf.nbytes)):
        raise RuntimeError("fdgpu_host_register failed: " + last_error())


def host_unregister(buf: np.ndarray) -> None:
    load_library().fdgpu_host_unregister(ctypes.c_void_p(buf.ctypes.data))


def fd_ed25519_strerror(err: int) -> str:
    return load_library().fd_ed25519_strerror(err).decode()


class Engine:
    """A verify engine bound to one GPU (fdgpu_ed25519_ctx_t)."""

    def __init__(self, device: int = 0, max_txn: int = 1 << 20, max_sig: int | None = None,
                 max_payload: int = 0, semantics: int = SEMANTICS_AVX512):
        L = load_library()
        self.L = L
        self.max_txn = max_txn
        self.max_sig = max_sig or max_txn
        self.max_payload = max_payload
        self.ctx = L.fdgpu_ed25519_ctx_new(device, max_txn, self.max_sig, max_payload, semantics)
        if not self.ctx:
            raise RuntimeError(f"fdgpu_ed25519_ctx_new failed: {last_error()}")

    def close(self):
        if self.ctx:
            self.L.fdgpu_ed25519_ctx_delete(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_small_batch_max(self, n: int) -> int:
        """Signatures per batch at or below which the latency path runs (0: never, 2**64-1: always)."""
        return int(self.L.fdgpu_ed25519_set_small_batch_max(self.ctx, ctypes.c_ulong(n)))

    def set_cu_exclusive(self, mode: int) -> None:
        """Latency-path workgroups alone on their CU (fdgpu_ed25519_set_cu_exclusive; 0 off)."""
        if self.L.fdgpu_ed25519_set_cu_exclusive(self.ctx, mode):
            raise RuntimeError(f"fdgpu_ed25519_set_cu_exclusive: {last_error()}")

    def set_lat_share(self, parts: int) -> None:
        """The exclusive walk within 1/parts of the CUs (fdgpu_ed25519_set_lat_share; 0 no limit)."""
        if self.L.fdgpu_ed25519_set_lat_share(self.ctx, parts):
            raise RuntimeError(f"fdgpu_ed25519_set_lat_share: {last_error()}")

    def front_batch(self) -> tuple[int, int, int] | None:
        """The oldest launched async batch: (txns, cursor, engine path), None if none is in flight."""
        t, c, p = ctypes.c_ulong(), ctypes.c_ulong(), ctypes.c_int()
        if not self.L.fdgpu_ed25519_front_batch(self.ctx, ctypes.byref(t), ctypes.byref(c), ctypes.byref(p)):
            return None
        return t.value, c.value, p.value

    def set_timing(self, on: bool = True):
        self.L.fdgpu_ed25519_set_timing(self.ctx, 1 if on else 0)

    def kernel_ms(self, idx: int) -> float:
        return float(self.L.fdgpu_ed25519_kernel_ms(self.ctx, idx))

    def verify_txns_host(self, payload: np.ndarray, desc: np.ndarray, want_sig_codes: bool = True):
        """Synchronous batch from host memory.  Returns (txn_codes, sig_codes)."""
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        nsig = int(desc["sig_cnt"].astype(np.int64).sum())
        txn_out = np.zeros(len(desc), np.int8)
        sig_out = np.zeros(max(nsig, 1), np.int8) if want_sig_codes else None
        rc = self.L.fdgpu_ed25519_verify_txns_host(self.ctx, payload.ctypes.data, payload.nbytes, desc.ctypes.data,
                                                   len(desc), txn_out.ctypes.data,
                                                   sig_out.ctypes.data if sig_out is not None else None)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_verify_txns_host: {rc} {last_error()}")
        return txn_out, (sig_out[:nsig] if sig_out is not None else None)

    def verify_txns_device(self, d_payload: int, d_desc: int, txn_cnt: int, sig_cnt: int,
                           d_txn_out: int, d_sig_out: int | None = None, stream: int | None = None):
        """Enqueue a batch already resident in HBM (raw device pointers)."""
        rc = self.L.fdgpu_ed25519_verify_txns_device(self.ctx, d_payload, d_desc, txn_cnt, sig_cnt, d_txn_out,
                                                     d_sig_out, stream)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_verify_txns_device: {rc} {last_error()}")

    def verify_many(self, msgs, sigs, pubs) -> np.ndarray:
        """fd_ed25519_verify codes of independent (msg, sig, pub) triples (fdgpu_ed25519_verify_many_host)."""
        n = len(msgs)
        keep = [np.frombuffer(bytes(x) + b"\0", np.uint8) for x in list(msgs) + list(sigs) + list(pubs)]
        ptrs = np.array([k.ctypes.data for k in keep], np.uint64)
        szs = np.array([len(m) for m in msgs], np.uint64)
        out = np.zeros(n, np.int8)
        rc = self.L.fdgpu_ed25519_verify_many_host(self.ctx, ptrs[:n].ctypes.data, szs.ctypes.data,
                                                   ptrs[n:2 * n].ctypes.data, ptrs[2 * n:].ctypes.data, n,
                                                   out.ctypes.data)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_verify_many_host: {rc} {last_error()}")
        return out

    def verify_txn_ptrs(self, payloads, desc: np.ndarray) -> np.ndarray:
        """Codes of pre-parsed transactions scattered in host memory (fdgpu_ed25519_verify_txn_ptrs):
        payloads[i] is transaction i's bytes, desc[i] its fd_txn_t offsets (payload_off/sig_base ignored)."""
        keep = [np.frombuffer(bytes(p) + b"\0", np.uint8) for p in payloads]
        ptrs = np.array([k.ctypes.data for k in keep], np.uint64)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        out = np.zeros(len(keep), np.int8)
        rc = self.L.fdgpu_ed25519_verify_txn_ptrs(self.ctx, ptrs.ctypes.data, desc.ctypes.data, len(keep),
                                                  out.ctypes.data)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_verify_txn_ptrs: {rc} {last_error()}")
        return out

    # -- raw payloads: device fd_txn_parse + verify ---------------------------
    def verify_raw_host(self, payload: np.ndarray, off: np.ndarray, sz: np.ndarray, want_img: bool = False):
        """Parse + verify raw transaction payloads (payload[off[t]:off[t]+sz[t]]).
        Returns (codes int8 -- FDGPU_ERR_PARSE or the batch verify code, footprints uint16,
        fd_txn_t images uint8[n, TXN_IMG_STRIDE] or None)."""
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        n = len(off)
        raw = np.zeros(n, RAW_DTYPE)
        raw["payload_off"] = off
        raw["payload_sz"] = sz
        codes = np.zeros(n, np.int8)
        fp = np.zeros(n, np.uint16)
        img = np.zeros((n, TXN_IMG_STRIDE), np.uint8) if want_img else None
        rc = self.L.fdgpu_ed25519_verify_raw_host(self.ctx, payload.ctypes.data, payload.nbytes, raw.ctypes.data, n,
                                                  codes.ctypes.data, img.ctypes.data if img is not None else None,
                                                  TXN_IMG_STRIDE, fp.ctypes.data)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_verify_raw_host: {rc} {last_error()}")
        return codes, fp, img

    def verify_raw_device(self, d_payload: int, d_raw: int, txn_cnt: int, sig_cnt: int, d_txn_out: int,
                          d_img: int | None = None, d_fp: int | None = None, stream: int | None = None):
        rc = self.L.fdgpu_ed25519_verify_raw_device(self.ctx, d_payload, d_raw, txn_cnt, sig_cnt, d_txn_out, d_img,
                                                    TXN_IMG_STRIDE, d_fp, stream)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_verify_raw_device: {rc} {last_error()}")

    # -- async pipeline ------------------------------------------------------
    def submit(self, payload: bytes, signature_off: int, acct_addr_off: int, message_off: int,
               sig_cnt: int, tag: int) -> int:
        b = np.frombuffer(payload, np.uint8)
        rc = self.L.fdgpu_ed25519_submit(self.ctx, b.ctypes.data, len(payload), signature_off, acct_addr_off,
                                         message_off, sig_cnt, tag)
        if rc <= -3:
            raise RuntimeError(f"fdgpu_ed25519_submit: {rc} {last_error()}")
        return rc

    def flush(self):
        rc = self.L.fdgpu_ed25519_flush(self.ctx)
        if rc:
            raise RuntimeError(f"fdgpu_ed25519_flush: {rc} {last_error()}")

    def submit_raw(self, payload: bytes, tag: int) -> int:
        b = np.frombuffer(payload, np.uint8) if len(payload) else np.zeros(1, np.uint8)
        rc = self.L.fdgpu_ed25519_submit_raw(self.ctx, b.ctypes.data, len(payload), tag)
        if rc <= -3:
            raise RuntimeError(f"fdgpu_ed25519_submit_raw: {rc} {last_error()}")
        return rc

    def set_dedup(self, enable: bool, seed: int = 0):
        """Raw batches also return the HA dedup tag (XXH64 of the first signature) computed on the GPU."""
        self.L.fdgpu_ed25519_set_dedup(self.ctx, 1 if enable else 0, seed)

    def poll_raw(self, max_n: int = 4096, blocking: bool = False, dedup: bool = False):
        """Completed raw submissions in order: (tags, codes, footprints, images[, dedup tags])."""
        tags = np.zeros(max_n, np.uint64)
        codes = np.zeros(max_n, np.int8)
        fp = np.zeros(max_n, np.uint16)
        img = np.zeros((max_n, TXN_IMG_STRIDE), np.uint8)
        dt = np.zeros(max_n, np.uint64)
        n = self.L.fdgpu_ed25519_poll_raw(self.ctx, tags.ctypes.data, codes.ctypes.data, img.ctypes.data,
                                          fp.ctypes.data, dt.ctypes.data, max_n, 1 if blocking else 0)
        if dedup:
            return tags[:n], codes[:n], fp[:n], img[:n], dt[:n]
        return tags[:n], codes[:n], fp[:n], img[:n]

    def faulted(self) -> bool:
        return bool(self.L.fdgpu_ed25519_faulted(self.ctx))

    def debug_fault(self):
        """Host-side test hook: the context behaves as after a failed batch."""
        self.L.fdgpu_ed25519_debug_fault(self.ctx)

    def slow_count(self) -> int:
        """Signatures of the last batch that took the full-length walk (half-size path; 0 when it is off)."""
        return int(self.L.fdgpu_ed25519_slow_count(self.ctx))

    def poll(self, max_n: int = 4096, blocking: bool = False):
        tags = np.zeros(max_n, np.uint64)
        codes = np.zeros(max_n, np.int8)
        n = self.L.fdgpu_ed25519_poll(self.ctx, tags.ctypes.data, codes.ctypes.data, max_n, 1 if blocking else 0)
        return tags[:n], codes[:n]
