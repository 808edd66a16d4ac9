"""TEST INFRASTRUCTURE ONLY -- ctypes bindings of the CPU oracle.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  It loads

* ``oracle/liboracle.so``  -- the from-scratch C restatement of the
  reference verify path (fd_ed25519_oracle.c), always available;
* ``oracle/_ref/libfdref_{avx512,portable}.so`` -- the reference's own
  verify sources compiled in place by ``oracle/Makefile ref`` (only
  where /root/reference existed at build time; the built .so travels to
  the GPU box, the sources do not);
* ``oracle/_ref/libfdref_stem.so`` -- the reference's stem run loop with
  the GPU tile's callbacks, a test harness.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SEM_AVX512 = 0
SEM_REF = 1

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i8p = ctypes.POINTER(ctypes.c_int8)


def build(ref: bool | None = None) -> None:
    """Compile liboracle.so (and the reference build when its sources exist)."""
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    if ref is None:
        ref = os.path.isdir("/root/reference/src/ballet/ed25519")
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


class Oracle:
    """The C restatement (oracle/fd_ed25519_oracle.c)."""

    def __init__(self, path: str | None = None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build(ref=False)
        self.lib = L = ctypes.CDLL(path)
        L.oracle_ed25519_verify.restype = ctypes.c_int
        L.oracle_ed25519_verify.argtypes = [_u8p, ctypes.c_size_t, _u8p, _u8p, ctypes.c_int]
        L.oracle_ed25519_verify_batch_single_msg.restype = ctypes.c_int
        L.oracle_ed25519_verify_batch_single_msg.argtypes = [_u8p, ctypes.c_size_t, _u8p, _u8p, ctypes.c_uint8, ctypes.c_int]
        L.oracle_verify_txns.restype = None
        L.oracle_verify_txns.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_size_t, _i8p, _i8p, ctypes.c_int, ctypes.c_int]
        L.oracle_sha512.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        L.oracle_scalar_reduce.argtypes = [_u8p, _u8p]
        L.oracle_scalar_validate.argtypes = [_u8p]
        L.oracle_point_decode.argtypes = [_u8p, _u8p, _u8p, ctypes.c_int]
        L.oracle_ed25519_public_from_private.argtypes = [_u8p, _u8p]
        L.oracle_ed25519_sign.argtypes = [_u8p, _u8p, ctypes.c_size_t, _u8p, _u8p]
        L.oracle_dsm_encode.argtypes = [_u8p, _u8p, _u8p, _u8p]
        L.oracle_txn_parse.restype = ctypes.c_uint32
        L.oracle_txn_parse.argtypes = [_u8p, ctypes.c_uint32, _u8p]
        L.oracle_txn_parse_batch.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, _u8p,
                                             ctypes.c_uint64, ctypes.c_void_p]

    @staticmethod
    def _b(x: bytes) -> np.ndarray:
        return np.frombuffer(bytes(x) + b"\0", dtype=np.uint8)

    def verify(self, msg: bytes, sig: bytes, pub: bytes, sem: int = SEM_AVX512) -> int:
        m = self._b(msg)
        return self.lib.oracle_ed25519_verify(_ptr(m), len(msg), _ptr(self._b(sig)), _ptr(self._b(pub)), sem)

    def verify_batch_single_msg(self, msg: bytes, sigs: bytes, pubs: bytes, n: int, sem: int = SEM_AVX512) -> int:
        return self.lib.oracle_ed25519_verify_batch_single_msg(
            _ptr(self._b(msg)), len(msg), _ptr(self._b(sigs)), _ptr(self._b(pubs)), n, sem)

    def verify_txns(self, payload: np.ndarray, desc: np.ndarray, sig_cnt_total: int,
                    sem: int = SEM_AVX512, threads: int = 1):
        txn_out = np.zeros(len(desc), dtype=np.int8)
        sig_out = np.zeros(max(sig_cnt_total, 1), dtype=np.int8)
        self.lib.oracle_verify_txns(_ptr(payload), desc.ctypes.data, len(desc), _ptr(txn_out, _i8p),
                                    _ptr(sig_out, _i8p), sem, threads)
        return txn_out, sig_out[:sig_cnt_total]

    def sha512(self, data: bytes) -> bytes:
        out = np.zeros(64, np.uint8)
        self.lib.oracle_sha512(_ptr(self._b(data)), len(data), _ptr(out))
        return out.tobytes()

    def scalar_reduce(self, x: bytes) -> bytes:
        out = np.zeros(32, np.uint8)
        self.lib.oracle_scalar_reduce(_ptr(out), _ptr(self._b(x)))
        return out.tobytes()

    def scalar_validate(self, s: bytes) -> bool:
        return bool(self.lib.oracle_scalar_validate(_ptr(self._b(s))))

    def point_decode(self, enc: bytes, sem: int = SEM_AVX512):
        x = np.zeros(32, np.uint8); y = np.zeros(32, np.uint8)
        rc = self.lib.oracle_point_decode(_ptr(x), _ptr(y), _ptr(self._b(enc)), sem)
        return rc, x.tobytes(), y.tobytes()

    def public_from_private(self, prv: bytes) -> bytes:
        out = np.zeros(32, np.uint8)
        self.lib.oracle_ed25519_public_from_private(_ptr(out), _ptr(self._b(prv)))
        return out.tobytes()

    def sign(self, msg: bytes, pub: bytes, prv: bytes) -> bytes:
        out = np.zeros(64, np.uint8)
        self.lib.oracle_ed25519_sign(_ptr(out), _ptr(self._b(msg)), len(msg), _ptr(self._b(pub)), _ptr(self._b(prv)))
        return out.tobytes()

    def txn_parse(self, payload: bytes):
        """fd_txn_parse restated: (footprint, fd_txn_t image bytes) -- footprint 0 = rejected."""
        out = np.zeros(1024, np.uint8)
        fp = self.lib.oracle_txn_parse(_ptr(self._b(payload)), len(payload), _ptr(out))
        return fp, out[:fp].tobytes()

    def txn_parse_batch(self, arena: np.ndarray, off: np.ndarray, sz: np.ndarray, stride: int = 864):
        return _parse_batch(self.lib.oracle_txn_parse_batch, arena, off, sz, stride)

    def dsm_encode(self, k: bytes, A: bytes, S: bytes):
        out = np.zeros(32, np.uint8)
        rc = self.lib.oracle_dsm_encode(_ptr(out), _ptr(self._b(k)), _ptr(self._b(A)), _ptr(self._b(S)))
        return rc, out.tobytes()


def _parse_batch(fn, arena, off, sz, stride):
    arena = np.ascontiguousarray(arena, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    sz = np.ascontiguousarray(sz, np.uint16)
    n = len(off)
    out = np.zeros((n, stride), np.uint8)
    fp = np.zeros(n, np.uint16)
    fn(_ptr(arena), off.ctypes.data, sz.ctypes.data, n, _ptr(out), stride, fp.ctypes.data)
    return fp, out


class RefTxn:
    """The reference's fd_txn_parse compiled from its own source (oracle/_ref/libfdref_txn.so)."""

    def __init__(self):
        path = os.path.join(HERE, "_ref", "libfdref_txn.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = L = ctypes.CDLL(path)
        L.ref_txn_parse.restype = ctypes.c_ulong
        L.ref_txn_parse.argtypes = [_u8p, ctypes.c_ulong, _u8p]
        L.ref_txn_parse_batch.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong, _u8p,
                                          ctypes.c_ulong, ctypes.c_void_p]

    def txn_parse(self, payload: bytes):
        out = np.zeros(1024, np.uint8)
        fp = self.lib.ref_txn_parse(_ptr(Oracle._b(payload)), len(payload), _ptr(out))
        return fp, out[:fp].tobytes()

    def txn_parse_batch(self, arena, off, sz, stride: int = 864):
        return _parse_batch(self.lib.ref_txn_parse_batch, arena, off, sz, stride)


class RefTile:
    """The reference verify tile's per-frag decision (oracle/_ref/libfdref_tile.so: fd_txn_verify, the
    tcache macros, fd_hash, fd_txn_parse and the AVX-512 verify compiled in place; after_frag's bundle
    bookkeeping restated in ref_tile_harness.c)."""

    REC_STRIDE = 1232 + 1024

    def __init__(self):
        path = os.path.join(HERE, "_ref", "libfdref_tile.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        if not cpu_has_avx512_ifma():
            raise RuntimeError("host CPU lacks AVX-512 IFMA; cannot run the AVX-512 reference build")
        self.lib = L = ctypes.CDLL(path)
        L.ref_tile_run.restype = ctypes.c_int
        L.ref_tile_run.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong] + \
            [ctypes.c_void_p] * 3 + [ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]

    def run(self, frags, depth: int, seed: int):
        """frags: [(payload bytes, bundle_id)].  Returns (results, metrics[5], {i: record bytes}, tags)."""
        n = len(frags)
        sz = np.array([len(p) for p, _ in frags], np.uint16)
        off = np.concatenate([[0], np.cumsum(sz.astype(np.int64))[:-1]]).astype(np.uint32) if n else np.zeros(0, np.uint32)
        arena = np.frombuffer(b"".join(bytes(p) for p, _ in frags) + bytes(64), np.uint8).copy()
        bid = np.array([b for _, b in frags], np.uint64)
        res = np.zeros(n, np.int32)
        rec_sz = np.zeros(n, np.uint64)
        rec = np.zeros((n, self.REC_STRIDE), np.uint8)
        tag = np.zeros(n, np.uint64)
        metrics = np.zeros(5, np.uint64)
        rc = self.lib.ref_tile_run(arena.ctypes.data, off.ctypes.data, sz.ctypes.data, bid.ctypes.data, n, depth, seed,
                                   res.ctypes.data, rec_sz.ctypes.data, rec.ctypes.data, self.REC_STRIDE,
                                   tag.ctypes.data, metrics.ctypes.data)
        if rc:
            raise RuntimeError(f"ref_tile_run: {rc}")
        recs = {i: rec[i, : int(rec_sz[i])].tobytes() for i in range(n) if res[i] == 0}
        return [int(x) for x in res], [int(x) for x in metrics], recs, [int(x) for x in tag]


    def run_kinds(self, frags, rr_idx: int, rr_cnt: int, depth: int, seed: int):
        """The full frag path of verify:rr_idx of rr_cnt (before_frag, during_frag, after_frag) over a mixed
        stream: frags = [(in_kind, sig, seq, frag bytes)] -- an fd_txn_m_t record for QUIC / bundle / send
        frags, an fd_gossip_update_message_t for gossip frags.  Returns (results with -2 = skipped by
        before_frag, metrics[5], {i: record bytes}, tags)."""
        n = len(frags)
        L = self.lib
        if not hasattr(self, "_kinds"):
            L.ref_tile_run_kinds.restype = ctypes.c_int
            L.ref_tile_run_kinds.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_ulong] * 5 + [ctypes.c_void_p] * 3 + \
                [ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
            self._kinds = True
        sz = np.array([len(f) for _, _, _, f in frags], np.uint16)
        off = np.zeros(n, np.uint32)
        pos, parts = 0, []
        for i, (_, _, _, f) in enumerate(frags):          # 64-B aligned, as chunks of a dcache
            off[i] = pos
            pad = (-len(f)) % 64
            parts.append(bytes(f) + bytes(pad))
            pos += len(f) + pad
        arena = np.frombuffer(b"".join(parts) + bytes(64), np.uint8).copy()
        kind = np.array([k for k, _, _, _ in frags], np.uint64)
        sig = np.array([g for _, g, _, _ in frags], np.uint64)
        seq = np.array([q for _, _, q, _ in frags], np.uint64)
        res = np.zeros(n, np.int32)
        rec_sz = np.zeros(n, np.uint64)
        rec = np.zeros((n, self.REC_STRIDE), np.uint8)
        tag = np.zeros(n, np.uint64)
        metrics = np.zeros(5, np.uint64)
        rc = L.ref_tile_run_kinds(arena.ctypes.data, off.ctypes.data, sz.ctypes.data, kind.ctypes.data,
                                  seq.ctypes.data, sig.ctypes.data, n, rr_idx, rr_cnt, depth, seed, res.ctypes.data,
                                  rec_sz.ctypes.data, rec.ctypes.data, self.REC_STRIDE, tag.ctypes.data,
                                  metrics.ctypes.data)
        if rc:
            raise RuntimeError(f"ref_tile_run_kinds: {rc}")
        recs = {i: rec[i, : int(rec_sz[i])].tobytes() for i in range(n) if res[i] == 0}
        return [int(x) for x in res], [int(x) for x in metrics], recs, [int(x) for x in tag]


class _StemCfg(ctypes.Structure):
    _fields_ = [("payload", ctypes.c_void_p), ("off", ctypes.c_void_p), ("sz", ctypes.c_void_p),
                ("n_payload", ctypes.c_ulong), ("n_frags", ctypes.c_ulong), ("in_depth", ctypes.c_ulong),
                ("out_depth", ctypes.c_ulong), ("batch_txn", ctypes.c_ulong), ("tcache_depth", ctypes.c_ulong),
                ("seed", ctypes.c_ulong), ("rate_fps", ctypes.c_ulong), ("consumer_pause_every", ctypes.c_ulong),
                ("consumer_pause_ns", ctypes.c_ulong), ("max_inflight", ctypes.c_ulong), ("device", ctypes.c_int),
                ("nctx", ctypes.c_int), ("zero_copy", ctypes.c_int), ("_pad", ctypes.c_int),
                ("tr_seq", ctypes.c_void_p), ("tr_res", ctypes.c_void_p), ("tr_tag", ctypes.c_void_p),
                ("tr_cap", ctypes.c_ulong), ("c_seq_in", ctypes.c_void_p), ("c_hash", ctypes.c_void_p),
                ("c_sz", ctypes.c_void_p), ("c_cap", ctypes.c_ulong), ("out", ctypes.c_ulong * 16),
                ("tile_metrics", ctypes.c_ulong * 5)]


class RefStem:
    """INTEGRATION.md section 2's tile patch over the reference's own stem run loop (oracle/_ref/libfdref_stem.so:
    src/disco/stem/fd_stem.c #included in place with the GPU tile's callbacks, reference tango objects and
    metrics, a producer thread and a reliable downstream consumer; ref_stem_harness.c).  Needs a GPU."""

    OUT_KEYS = ("verdicts", "consumed", "returned", "stem_overruns", "filtered", "taken", "published", "bursts",
                "link_consumed", "link_filtered", "link_overrun_polling_frags", "link_overrun_reading_frags",
                "backpressure_count", "traced", "err")

    def __init__(self):
        path = os.path.join(HERE, "_ref", "libfdref_stem.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = ctypes.CDLL(path)
        self.lib.ref_stem_run.restype = ctypes.c_int
        self.lib.ref_stem_run.argtypes = [ctypes.POINTER(_StemCfg)]

    def run(self, payloads, n_frags: int, *, in_depth: int = 1 << 16, out_depth: int = 256, batch_txn: int = 1024,
            tcache_depth: int = 1 << 16, seed: int = 0x5EED, rate_fps: int = 0, consumer_pause_every: int = 0,
            consumer_pause_ns: int = 0, max_inflight: int = 1, device: int = 0, nctx: int = 1, zero_copy: bool = False):
        """The producer publishes frag s = payloads[s % n]; returns (stats dict, the tile's verdicts
        (seq, result, tag) in order, what the consumer received: (record xxh64, size) per published frag)."""
        sz = np.array([len(p) for p in payloads], np.uint16)
        off = np.zeros(len(payloads), np.uint32)
        off[1:] = np.cumsum(sz[:-1].astype(np.int64))
        arena = np.frombuffer(b"".join(payloads) + bytes(64), np.uint8).copy()
        tr_seq = np.zeros(n_frags, np.uint64); tr_res = np.zeros(n_frags, np.int32); tr_tag = np.zeros(n_frags, np.uint64)
        c_hash = np.zeros(n_frags, np.uint64); c_sz = np.zeros(n_frags, np.uint64); c_seq = np.zeros(n_frags, np.uint64)
        c = _StemCfg(payload=arena.ctypes.data, off=off.ctypes.data, sz=sz.ctypes.data, n_payload=len(payloads),
                     n_frags=n_frags, in_depth=in_depth, out_depth=out_depth, batch_txn=batch_txn,
                     tcache_depth=tcache_depth, seed=seed, rate_fps=rate_fps, consumer_pause_every=consumer_pause_every,
                     consumer_pause_ns=consumer_pause_ns, max_inflight=max_inflight, device=device, nctx=nctx,
                     zero_copy=1 if zero_copy else 0, tr_seq=tr_seq.ctypes.data, tr_res=tr_res.ctypes.data,
                     tr_tag=tr_tag.ctypes.data, tr_cap=n_frags, c_seq_in=c_seq.ctypes.data, c_hash=c_hash.ctypes.data,
                     c_sz=c_sz.ctypes.data, c_cap=n_frags)
        rc = self.lib.ref_stem_run(ctypes.byref(c))
        st = {k: int(c.out[i]) for i, k in enumerate(self.OUT_KEYS)}
        st["rc"] = rc
        st["tile_metrics"] = [int(x) for x in c.tile_metrics]
        n = min(st["traced"], n_frags)
        m = min(st["consumed"], n_frags) if st["consumed"] < (1 << 63) else 0
        return st, (tr_seq[:n], tr_res[:n], tr_tag[:n]), (c_hash[:m], c_sz[:m])


class RefMcache:
    """A tango mcache written and read by the reference's own inline code (oracle/_ref/libfdref_mcache.so:
    fd_mcache_publish / fd_mcache_publish_avx / FD_MCACHE_WAIT compiled in place; fd_mcache_new's line
    initialisation restated).  The ring is an FD_MCACHE_ALIGN-aligned fd_frag_meta_t array inside a
    page-aligned numpy buffer (at byte offset `off`, like the lines of an fd_mcache region, which start
    past its header), so tests can hand `lines_addr` to fdgpu_mcache_wrap."""

    META_DTYPE = np.dtype([("seq", "<u8"), ("sig", "<u8"), ("chunk", "<u4"), ("sz", "<u2"), ("ctl", "<u2"),
                           ("tsorig", "<u4"), ("tspub", "<u4")])

    def __init__(self, depth: int, seq0: int = 0, off: int = 256):
        path = os.path.join(HERE, "_ref", "libfdref_mcache.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = L = ctypes.CDLL(path)
        ul, vp = ctypes.c_ulong, ctypes.c_void_p
        for n in ("ref_frag_meta_sz", "ref_mcache_align"):
            getattr(L, n).restype = ul
        L.ref_mcache_line_idx.restype = ul
        L.ref_mcache_line_idx.argtypes = [ul, ul]
        L.ref_mcache_init_lines.argtypes = [vp, ul, ul]
        L.ref_mcache_publish.argtypes = [vp] + [ul] * 8 + [ctypes.c_int]
        L.ref_mcache_wait.argtypes = [vp, ul, ul, vp, ctypes.POINTER(ul)]
        assert L.ref_frag_meta_sz() == self.META_DTYPE.itemsize == 32
        assert off % L.ref_mcache_align() == 0
        self.depth = depth
        nbytes = off + depth * 32
        self._raw = np.zeros(nbytes + 8192, np.uint8)
        base = (-self._raw.ctypes.data) % 4096
        self.buf = self._raw[base: base + ((nbytes + 4095) // 4096) * 4096]
        self.lines_addr = self.buf.ctypes.data + off
        self.lines = self.buf[off: off + depth * 32].view(self.META_DTYPE)
        L.ref_mcache_init_lines(self.lines_addr, depth, seq0)

    def line_idx(self, seq: int) -> int:
        return int(self.lib.ref_mcache_line_idx(seq, self.depth))

    def publish(self, seq, sig, chunk, sz, ctl=0, tsorig=0, tspub=0, avx=False):
        self.lib.ref_mcache_publish(self.lines_addr, self.depth, seq, sig, chunk, sz, ctl, tsorig, tspub, 1 if avx else 0)

    def wait(self, seq):
        """FD_MCACHE_WAIT once: (rc, meta record or None, seq_found); rc 0 ready, 1 not yet, -1 overrun."""
        out = np.zeros(1, self.META_DTYPE)
        found = ctypes.c_ulong(0)
        rc = self.lib.ref_mcache_wait(self.lines_addr, self.depth, seq, out.ctypes.data, ctypes.byref(found))
        return rc, (out[0] if rc == 0 else None), int(found.value)


def cpu_has_avx512_ifma() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split(":", 1)[1].split())
                    return {"avx512f", "avx512ifma", "avx512vl", "avx512bw", "avx512dq"} <= fl
    except OSError:
        pass
    return False


class Reference:
    """The reference's verify path, compiled from its own sources (oracle/_ref)."""

    def __init__(self, variant: str = "avx512"):
        path = os.path.join(HERE, "_ref", f"libfdref_{variant}.so")
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        if variant == "avx512" and not cpu_has_avx512_ifma():
            raise RuntimeError("host CPU lacks AVX-512 IFMA; cannot run the AVX-512 reference build")
        self.variant = variant
        self.lib = L = ctypes.CDLL(path)
        L.ref_verify.restype = ctypes.c_int
        L.ref_verify.argtypes = [_u8p, ctypes.c_ulong, _u8p, _u8p]
        L.ref_verify_batch.restype = ctypes.c_int
        L.ref_verify_batch.argtypes = [_u8p, ctypes.c_ulong, _u8p, _u8p, ctypes.c_uint8]
        L.ref_sign.argtypes = [_u8p, _u8p, ctypes.c_ulong, _u8p, _u8p]
        L.ref_public_from_private.argtypes = [_u8p, _u8p]
        L.ref_sha512.argtypes = [_u8p, ctypes.c_ulong, _u8p]
        L.ref_verify_txns.argtypes = [_u8p, ctypes.c_void_p, ctypes.c_ulong, _i8p, _i8p, ctypes.c_int]

    _b = staticmethod(Oracle._b)

    def verify(self, msg: bytes, sig: bytes, pub: bytes) -> int:
        return self.lib.ref_verify(_ptr(self._b(msg)), len(msg), _ptr(self._b(sig)), _ptr(self._b(pub)))

    def verify_batch_single_msg(self, msg: bytes, sigs: bytes, pubs: bytes, n: int) -> int:
        return self.lib.ref_verify_batch(_ptr(self._b(msg)), len(msg), _ptr(self._b(sigs)), _ptr(self._b(pubs)), n)

    def sign(self, msg: bytes, pub: bytes, prv: bytes) -> bytes:
        out = np.zeros(64, np.uint8)
        self.lib.ref_sign(_ptr(out), _ptr(self._b(msg)), len(msg), _ptr(self._b(pub)), _ptr(self._b(prv)))
        return out.tobytes()

    def public_from_private(self, prv: bytes) -> bytes:
        out = np.zeros(32, np.uint8)
        self.lib.ref_public_from_private(_ptr(out), _ptr(self._b(prv)))
        return out.tobytes()

    def sha512(self, data: bytes) -> bytes:
        out = np.zeros(64, np.uint8)
        self.lib.ref_sha512(_ptr(self._b(data)), len(data), _ptr(out))
        return out.tobytes()

    def verify_txns(self, payload: np.ndarray, desc: np.ndarray, sig_cnt_total: int, threads: int = 1,
                    want_sig_codes: bool = True):
        """(txn codes, per-signature codes or None).  want_sig_codes=False verifies every signature once
        (only the batch call, as fd_txn_verify does): the form the CPU baseline times."""
        txn_out = np.zeros(len(desc), dtype=np.int8)
        sig_out = np.zeros(max(sig_cnt_total, 1), dtype=np.int8) if want_sig_codes else None
        self.lib.ref_verify_txns(_ptr(payload), desc.ctypes.data, len(desc), _ptr(txn_out, _i8p),
                                 _ptr(sig_out, _i8p) if sig_out is not None else None, threads)
        return txn_out, (sig_out[:sig_cnt_total] if sig_out is not None else None)
