"""ctypes mirror of include/fd_verify_gpu.h (libfdgpu_vtile.so): the GPU
verify tile's frag callbacks, its tcache / mcache / dcache pieces, and
the streaming benchmark.  No CPU fallback: the tile needs the engine and
a GPU; the tango pieces (tcache, mcache, dedup tag) are host-only."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .engine import PKG_DIR, load_library as load_engine

LIB_PATH = os.environ.get("FDGPU_VTILE_LIB") or os.path.join(PKG_DIR, "libfdgpu_vtile.so")   # env: A/B builds
TXNM_HDR_SZ = 80
CHUNK_SZ = 64
PUBLISH, PARSE_FAIL, VERIFY_FAIL, DEDUP_FAIL, BUNDLE_PEER_FAIL, OVERRUN, GPU_FAULT = range(7)
IN_QUIC, IN_BUNDLE, IN_GOSSIP, IN_SEND = range(4)        # fd_verify_tile.c:7-10

GOSSIP_TAG_VOTE = 3                                      # fd_gossip_types.h:26
GOSSIP_VOTE_TXN_SZ_OFF, GOSSIP_VOTE_TXN_OFF = 64, 72   # fd_gossip_update_message_t vote.txn_sz / vote.txn, x86-64
GOSSIP_MSG_SZ = 1297     # FD_GOSSIP_UPDATE_SZ_VOTE = 49 + sizeof(fd_gossip_vote_t), the frame the gossip tile publishes
                         # (src/flamenco/gossip/fd_gossip_private.h:80, crds/fd_crds.c:938)
LAT_BUCKETS = 40

EXPORTS = ("fdgpu_dedup_tag", "fdgpu_xxh64", "fdgpu_link_set_trace", "fdgpu_link_trace", "fdgpu_link_anomalies", "fdgpu_link_anomaly_results", "fdgpu_tcache_new", "fdgpu_tcache_delete", "fdgpu_tcache_query", "fdgpu_tcache_insert",
           "fdgpu_mcache_new", "fdgpu_mcache_delete", "fdgpu_mcache_publish", "fdgpu_mcache_poll",
           "fdgpu_mcache_query", "fdgpu_mcache_wrap", "fdgpu_mcache_depth", "fdgpu_mcache_lines",
           "fdgpu_dcache_compact_next", "fdgpu_vtile_new", "fdgpu_vtile_delete", "fdgpu_vtile_out_dcache",
           "fdgpu_vtile_during_frag", "fdgpu_vtile_flush", "fdgpu_vtile_housekeep", "fdgpu_vtile_pipeline_state", "fdgpu_vtile_after_frags", "fdgpu_vtile_pending",
           "fdgpu_vtile_metrics", "fdgpu_vtile_set_in_link", "fdgpu_vtile_set_in_links", "fdgpu_vtile_oldest_pending_seq", "fdgpu_vtile_overruns",
           "fdgpu_vtile_faulted", "fdgpu_vtile_recover", "fdgpu_vtile_debug_fault", "fdgpu_vtile_gpu_metrics",
           "fdgpu_vtile_new_opts", "fdgpu_vtile_copy", "fdgpu_vtile_copy_state", "fdgpu_vtile_during_frag_overrun",
           "fdgpu_vtile_set_round_robin", "fdgpu_vtile_before_frag", "fdgpu_vtile_set_in",
           "fdgpu_vtile_during_frag_chunk",
           "fdgpu_link_new", "fdgpu_link_join", "fdgpu_link_delete", "fdgpu_link_joined", "fdgpu_link_cfg",
           "fdgpu_link_run", "fdgpu_link_tiles_of", "fdgpu_link_mcache", "fdgpu_link_dcache", "fdgpu_link_result",
           "fdgpu_stream_run", "fdgpu_stream_bench", "fdgpu_vsvc_new", "fdgpu_vsvc_join", "fdgpu_vsvc_add_region",
           "fdgpu_vsvc_start", "fdgpu_vsvc_ready", "fdgpu_vsvc_poll", "fdgpu_vsvc_run", "fdgpu_vsvc_stop",
           "fdgpu_vsvc_pending", "fdgpu_vsvc_stats", "fdgpu_vsvc_delete", "fdgpu_vtile_new_svc",
           "fdgpu_vtile_set_svc_region", "fdgpu_gpu_numa_node_sysfs", "fdgpu_link_svc_stats", "fdgpu_link_run_tile",
           "fdgpu_vtile_debug_fail_launch", "fdgpu_vsvc_debug_serve", "fdgpu_link_placement")

TXNM_DTYPE = np.dtype([("reference_slot", "<u8"), ("payload_sz", "<u2"), ("txn_t_sz", "<u2"), ("source_ipv4", "<u4"),
                       ("source_tpu", "u1"), ("_pad0", "u1", (7,)), ("bundle_id", "<u8"), ("bundle_txn_cnt", "<u8"),
                       ("commission", "u1"), ("commission_pubkey", "u1", (32,)), ("_pad1", "u1", (7,))])
assert TXNM_DTYPE.itemsize == TXNM_HDR_SZ


class FragMeta(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_ulong), ("sig", ctypes.c_ulong), ("chunk", ctypes.c_uint), ("sz", ctypes.c_uint),
                ("tsorig", ctypes.c_ulong), ("tspub", ctypes.c_ulong)]


class Done(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_ulong), ("tsorig", ctypes.c_ulong), ("chunk", ctypes.c_ulong), ("sz", ctypes.c_ulong),
                ("tag", ctypes.c_ulong), ("result", ctypes.c_int), ("code", ctypes.c_int), ("in_idx", ctypes.c_ulong),
                ("ctx", ctypes.c_uint), ("batch_txns", ctypes.c_uint), ("batch_pos", ctypes.c_uint), ("path", ctypes.c_int)]


class GpuMetrics(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_ulong), ("batch_txns", ctypes.c_ulong), ("inflight", ctypes.c_ulong),
                ("inflight_max", ctypes.c_ulong), ("pending", ctypes.c_ulong), ("overruns", ctypes.c_ulong),
                ("gpu_fault_frags", ctypes.c_ulong), ("faults", ctypes.c_ulong),
                ("lat_hist", ctypes.c_ulong * LAT_BUCKETS), ("wait_ns", ctypes.c_ulong),
                ("poll_ns", ctypes.c_ulong), ("after_ns", ctypes.c_ulong),
                ("launch_ns", ctypes.c_ulong), ("copies", ctypes.c_ulong), ("copy_lat_n", ctypes.c_ulong),
                ("copy_lat_ns_sum", ctypes.c_ulong), ("copy_lat_ns_max", ctypes.c_ulong),
                ("gather_gpu", ctypes.c_ulong * 8), ("phase", ctypes.c_ulong * 9), ("copy_backlog", ctypes.c_ulong),
                ("launcher", ctypes.c_ulong * 6), ("host_copy", ctypes.c_ulong * 4)]

    def as_dict(self) -> dict:
        return {k: (list(getattr(self, k)) if k in ("lat_hist", "gather_gpu", "phase", "launcher", "host_copy")
                    else int(getattr(self, k)))
                for k, _ in self._fields_}


class VTileOpts(ctypes.Structure):
    """fdgpu_vtile_opts_t (0 = default everywhere)."""
    _fields_ = [("nctx", ctypes.c_int), ("host_dedup_tag", ctypes.c_int), ("small_max", ctypes.c_ulong),
                ("min_batch", ctypes.c_ulong), ("max_wait_ns", ctypes.c_ulong), ("copy_wait_ns", ctypes.c_ulong),
                ("copy_min", ctypes.c_ulong), ("gather_cus", ctypes.c_uint), ("max_uncopied", ctypes.c_ulong),
                ("cu_split", ctypes.c_int), ("cu_exclusive", ctypes.c_int), ("launcher", ctypes.c_int),
                ("launcher_core", ctypes.c_int), ("copy_threads", ctypes.c_int), ("copy_cores", ctypes.c_int * 8),
                ("lat_share", ctypes.c_int)]


class StreamCfg(ctypes.Structure):
    _fields_ = [("n_frags", ctypes.c_ulong), ("batch_txn", ctypes.c_ulong), ("max_inflight", ctypes.c_ulong),
                ("rate_fps", ctypes.c_double), ("tiles", ctypes.c_int), ("gpus", ctypes.c_int),
                ("zero_copy", ctypes.c_int), ("reliable", ctypes.c_int), ("producers", ctypes.c_int),
                ("nctx", ctypes.c_int), ("prof", ctypes.c_int), ("out_mult", ctypes.c_ulong),
                ("copy_wait_ns", ctypes.c_ulong), ("copy_min", ctypes.c_ulong), ("gather_cus", ctypes.c_uint),
                ("max_uncopied", ctypes.c_ulong), ("pf_dist", ctypes.c_int), ("cu_split", ctypes.c_int),
                ("cu_exclusive", ctypes.c_int), ("no_huge_pages", ctypes.c_int), ("launcher", ctypes.c_int),
                ("copy_threads", ctypes.c_int), ("min_batch", ctypes.c_ulong), ("small_max", ctypes.c_ulong),
                ("hk_ns", ctypes.c_ulong), ("lat_share", ctypes.c_int), ("svc", ctypes.c_int),
                ("trace_cap", ctypes.c_ulong), ("prod_node", ctypes.c_int * 16)]


class VsvcCfg(ctypes.Structure):
    """fdgpu_vsvc_cfg_t (0 = default everywhere but clients / out_dcache_bytes / batch_txn)."""
    _fields_ = [("clients", ctypes.c_int), ("out_dcache_bytes", ctypes.c_ulong), ("batch_txn", ctypes.c_ulong),
                ("max_inflight", ctypes.c_ulong), ("semantics", ctypes.c_int), ("nctx", ctypes.c_int),
                ("small_max", ctypes.c_ulong), ("min_batch", ctypes.c_ulong), ("max_wait_ns", ctypes.c_ulong),
                ("copy_wait_ns", ctypes.c_ulong), ("copy_min", ctypes.c_ulong), ("gather_cus", ctypes.c_uint),
                ("cu_split", ctypes.c_int), ("cu_exclusive", ctypes.c_int), ("lat_share", ctypes.c_int),
                ("launcher", ctypes.c_int), ("launcher_core", ctypes.c_int),
                ("debug_hooks", ctypes.c_int)]


class VsvcStats(ctypes.Structure):
    _fields_ = [("gm", GpuMetrics), ("taken", ctypes.c_ulong), ("completed", ctypes.c_ulong),
                ("fault_completions", ctypes.c_ulong), ("busy_polls", ctypes.c_ulong), ("polls", ctypes.c_ulong),
                ("faults", ctypes.c_ulong), ("recovered", ctypes.c_ulong), ("mixed_batches", ctypes.c_ulong),
                ("loop_ns", ctypes.c_ulong),
                ("busy_ns", ctypes.c_ulong)]

    def as_dict(self) -> dict:
        d = {k: int(getattr(self, k)) for k, _ in self._fields_ if k != "gm"}
        d["gm"] = self.gm.as_dict()
        return d


class StreamStats(ctypes.Structure):
    _fields_ = [("seconds", ctypes.c_double), ("frags", ctypes.c_ulong), ("sigs", ctypes.c_ulong),
                ("published", ctypes.c_ulong), ("frags_per_s", ctypes.c_double), ("sigs_per_s", ctypes.c_double),
                ("lat_p50_us", ctypes.c_double), ("lat_p99_us", ctypes.c_double), ("lat_max_us", ctypes.c_double),
                ("metrics", ctypes.c_ulong * 5), ("overruns", ctypes.c_ulong), ("tile_ns", ctypes.c_ulong * 4),
                ("verdicts", ctypes.c_ulong), ("lost", ctypes.c_ulong), ("batches", ctypes.c_ulong),
                ("batch_txns", ctypes.c_ulong), ("inflight_max", ctypes.c_ulong),
                ("gpu_lat_hist", ctypes.c_ulong * LAT_BUCKETS), ("tiles", ctypes.c_int), ("gpus", ctypes.c_int),
                ("gpu_wait_ns", ctypes.c_ulong), ("poll_ns", ctypes.c_ulong), ("after_ns", ctypes.c_ulong),
                ("launch_ns", ctypes.c_ulong), ("tile_idle_ns", ctypes.c_ulong), ("prod_seconds", ctypes.c_double),
                ("prod_wait_ns", ctypes.c_ulong), ("prof_ns", ctypes.c_ulong * 8), ("copies", ctypes.c_ulong),
                ("copy_lat_n", ctypes.c_ulong), ("copy_lat_ns_sum", ctypes.c_ulong), ("copy_lat_ns_max", ctypes.c_ulong),
                ("gather_gpu", ctypes.c_ulong * 8), ("phase", ctypes.c_ulong * 9), ("copy_backlog", ctypes.c_ulong),
                ("tile_cpu_ns", ctypes.c_ulong), ("tile_wall_ns", ctypes.c_ulong), ("tile_nivcsw", ctypes.c_ulong),
                ("tile_cpu_share_min", ctypes.c_double), ("tile_cpu", ctypes.c_long * 8),
                ("prod_cpu_ns", ctypes.c_ulong), ("prod_wall_ns", ctypes.c_ulong), ("prod_nivcsw", ctypes.c_ulong),
                ("launcher", ctypes.c_ulong * 6), ("host_copy", ctypes.c_ulong * 4), ("prod_cpu", ctypes.c_long * 4),
                ("tiles_gpu_open", ctypes.c_ulong)]

    def as_dict(self) -> dict:
        out = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            out[k] = list(v) if k in ("metrics", "tile_ns", "gpu_lat_hist", "prof_ns", "gather_gpu", "phase", "tile_cpu",
                                      "launcher", "host_copy", "prod_cpu") else v
        return out


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        load_engine()
        L = ctypes.CDLL(LIB_PATH)
        vp, ul = ctypes.c_void_p, ctypes.c_ulong
        L.fdgpu_dedup_tag.restype = ul
        L.fdgpu_dedup_tag.argtypes = [ul, vp]
        L.fdgpu_tcache_new.restype = vp
        L.fdgpu_tcache_new.argtypes = [ul]
        L.fdgpu_tcache_delete.argtypes = [vp]
        L.fdgpu_tcache_query.argtypes = [vp, ul]
        L.fdgpu_tcache_insert.argtypes = [vp, ul]
        L.fdgpu_mcache_new.restype = vp
        L.fdgpu_mcache_new.argtypes = [ul, ul]
        L.fdgpu_mcache_delete.argtypes = [vp]
        L.fdgpu_mcache_publish.argtypes = [vp, ul, ul, ctypes.c_uint, ctypes.c_uint, ul, ul]
        L.fdgpu_mcache_poll.argtypes = [vp, ul, ctypes.POINTER(FragMeta)]
        L.fdgpu_mcache_query.argtypes = [vp, ul, ctypes.POINTER(FragMeta), ctypes.POINTER(ctypes.c_ulong)]
        L.fdgpu_mcache_wrap.restype = vp
        L.fdgpu_mcache_wrap.argtypes = [vp, ul]
        L.fdgpu_mcache_depth.restype = ul
        L.fdgpu_mcache_depth.argtypes = [vp]
        L.fdgpu_mcache_lines.restype = vp
        L.fdgpu_mcache_lines.argtypes = [vp]
        L.fdgpu_dcache_compact_next.restype = ul
        L.fdgpu_dcache_compact_next.argtypes = [ul, ul, ul, ul]
        L.fdgpu_vtile_new.restype = vp
        L.fdgpu_vtile_new.argtypes = [ctypes.c_int, ul, ul, ul, ul, ctypes.c_int]
        L.fdgpu_vtile_new_opts.restype = vp
        L.fdgpu_vtile_new_opts.argtypes = [ctypes.c_int, ul, ul, ul, ul, ctypes.c_int, ctypes.POINTER(VTileOpts)]
        L.fdgpu_vtile_copy.restype = ctypes.c_int
        L.fdgpu_vtile_copy.argtypes = [vp, ctypes.c_int]
        L.fdgpu_vtile_copy_state.restype = ul
        L.fdgpu_vtile_copy_state.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_ulong)]
        L.fdgpu_vtile_during_frag_overrun.argtypes = [vp]
        L.fdgpu_vtile_set_round_robin.argtypes = [vp, ul, ul]
        L.fdgpu_vtile_before_frag.argtypes = [vp, ul, ul, ul]
        L.fdgpu_vtile_set_in.argtypes = [vp, ul, ctypes.c_int, vp, ul, ul]
        L.fdgpu_vtile_during_frag_chunk.argtypes = [vp, ul, ul, ul, ul, ul, ul, ul]
        L.fdgpu_vtile_delete.argtypes = [vp]
        L.fdgpu_vtile_out_dcache.restype = vp
        L.fdgpu_vtile_out_dcache.argtypes = [vp]
        L.fdgpu_vtile_during_frag.argtypes = [vp, ul, vp, ul, ul, ul]
        L.fdgpu_vtile_flush.argtypes = [vp]
        L.fdgpu_vtile_housekeep.argtypes = [vp, ul]
        L.fdgpu_vtile_housekeep.restype = ctypes.c_int
        L.fdgpu_vtile_after_frags.restype = ul
        L.fdgpu_vtile_after_frags.argtypes = [vp, ctypes.POINTER(Done), ul, ctypes.c_int]
        L.fdgpu_vtile_pending.restype = ul
        L.fdgpu_vtile_pending.argtypes = [vp]
        L.fdgpu_vtile_metrics.argtypes = [vp, ctypes.POINTER(ctypes.c_ulong)]
        L.fdgpu_vtile_set_in_link.argtypes = [vp, vp]
        L.fdgpu_vtile_set_in_links.argtypes = [vp, vp, ctypes.c_int]
        L.fdgpu_vtile_oldest_pending_seq.restype = ul
        L.fdgpu_vtile_oldest_pending_seq.argtypes = [vp, ctypes.POINTER(ctypes.c_ulong)]
        L.fdgpu_vtile_overruns.restype = ul
        L.fdgpu_vtile_overruns.argtypes = [vp]
        L.fdgpu_vtile_faulted.argtypes = [vp]
        L.fdgpu_vtile_recover.argtypes = [vp]
        L.fdgpu_vtile_debug_fault.argtypes = [vp, ctypes.c_int]
        L.fdgpu_vtile_gpu_metrics.argtypes = [vp, ctypes.POINTER(GpuMetrics)]
        L.fdgpu_link_new.restype = vp
        L.fdgpu_link_new.argtypes = [ctypes.c_char_p, ctypes.POINTER(StreamCfg), vp, vp, vp, ul, ul]
        L.fdgpu_link_join.restype = vp
        L.fdgpu_link_join.argtypes = [ctypes.c_char_p, ctypes.c_double]
        L.fdgpu_link_delete.argtypes = [vp]
        L.fdgpu_link_joined.restype = ul
        L.fdgpu_link_joined.argtypes = [vp]
        L.fdgpu_link_cfg.argtypes = [vp, ctypes.POINTER(StreamCfg)]
        L.fdgpu_link_run.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.fdgpu_link_tiles_of.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.fdgpu_link_mcache.restype = vp
        L.fdgpu_link_mcache.argtypes = [vp]
        L.fdgpu_link_dcache.restype = vp
        L.fdgpu_link_dcache.argtypes = [vp]
        L.fdgpu_link_result.argtypes = [vp, ctypes.c_double, ctypes.POINTER(StreamStats)]
        L.fdgpu_xxh64.restype = ul
        L.fdgpu_xxh64.argtypes = [ul, vp, ul]
        L.fdgpu_link_set_trace.restype = ctypes.c_int
        L.fdgpu_link_set_trace.argtypes = [vp, ul]
        L.fdgpu_link_trace.restype = ul
        L.fdgpu_link_trace.argtypes = [vp, ctypes.c_int, vp, ul]
        L.fdgpu_link_anomalies.restype = ul
        L.fdgpu_link_anomalies.argtypes = [vp, ctypes.c_int, vp, ul]
        L.fdgpu_link_anomaly_results.restype = ul
        L.fdgpu_link_anomaly_results.argtypes = [vp, ctypes.c_int, vp]
        L.fdgpu_stream_run.argtypes = [ctypes.c_int, ctypes.POINTER(StreamCfg), vp, vp, vp, ul, ul,
                                       ctypes.POINTER(StreamStats)]
        L.fdgpu_stream_bench.argtypes = [ctypes.c_int, vp, vp, vp, ul, ul, ctypes.c_int, ul, ul, ul, ctypes.c_double,
                                         ctypes.c_int, ctypes.POINTER(StreamStats)]
        L.fdgpu_vsvc_new.restype = vp
        L.fdgpu_vsvc_new.argtypes = [ctypes.c_char_p, ctypes.POINTER(VsvcCfg)]
        L.fdgpu_vsvc_join.restype = vp
        L.fdgpu_vsvc_join.argtypes = [ctypes.c_char_p, ctypes.c_double]
        L.fdgpu_vsvc_add_region.argtypes = [vp, ctypes.c_int, vp, ul]
        L.fdgpu_vsvc_start.argtypes = [vp, ctypes.c_int]
        L.fdgpu_vsvc_ready.argtypes = [vp]
        L.fdgpu_vsvc_poll.argtypes = [vp]
        L.fdgpu_vsvc_run.argtypes = [vp]
        L.fdgpu_vsvc_stop.argtypes = [vp]
        L.fdgpu_vsvc_pending.restype = ul
        L.fdgpu_vsvc_pending.argtypes = [vp]
        L.fdgpu_vsvc_stats.argtypes = [vp, ctypes.POINTER(VsvcStats)]
        L.fdgpu_vsvc_delete.argtypes = [vp]
        L.fdgpu_vsvc_debug_serve.restype = ul
        L.fdgpu_vsvc_debug_serve.argtypes = [vp, vp, ul, ul]
        L.fdgpu_vtile_new_svc.restype = vp
        L.fdgpu_vtile_new_svc.argtypes = [vp, ctypes.c_int, ul, ul, ctypes.POINTER(VTileOpts)]
        L.fdgpu_vtile_set_svc_region.argtypes = [vp, ctypes.c_int, vp, ul]
        L.fdgpu_vtile_debug_fail_launch.argtypes = [vp, ctypes.c_int]
        L.fdgpu_gpu_numa_node_sysfs.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.fdgpu_link_svc_stats.argtypes = [vp, ctypes.POINTER(VsvcStats), ctypes.POINTER(ctypes.c_int)]
        L.fdgpu_link_placement.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_ulong), ctypes.POINTER(ctypes.c_ulong)]
        _lib = L
    return _lib


TRACE_DTYPE = np.dtype([("seq", "<u8"), ("tag", "<u8"), ("rec_hash", "<u8"), ("result", "<i4"), ("rec_sz", "<u4"),
                        ("in_idx", "<u8")])
ANOM_DTYPE = np.dtype([("seq", "<u8"), ("in_idx", "<u8"), ("payload_idx", "<u8"), ("tag", "<u8"), ("result", "<i4"),
                       ("code", "<i4"), ("ctx", "<u4"), ("batch_txns", "<u4"), ("batch_pos", "<u4"), ("path", "<i4")])


def xxh64(seed: int, data: bytes) -> int:
    b = np.frombuffer(bytes(data) + b"\0", np.uint8)
    return int(load().fdgpu_xxh64(seed, b.ctypes.data, len(data)))


def dedup_tag(seed: int, sig: bytes) -> int:
    b = np.frombuffer(bytes(sig[:64]).ljust(64, b"\0"), np.uint8)
    return int(load().fdgpu_dedup_tag(seed, b.ctypes.data))


class TCache:
    def __init__(self, depth: int):
        self.L = load()
        self.p = self.L.fdgpu_tcache_new(depth)

    def query(self, tag: int) -> bool:
        return bool(self.L.fdgpu_tcache_query(self.p, tag))

    def insert(self, tag: int) -> bool:
        return bool(self.L.fdgpu_tcache_insert(self.p, tag))

    def __del__(self):
        if getattr(self, "p", None):
            self.L.fdgpu_tcache_delete(self.p)
            self.p = None


def gossip_vote_msg(txn: bytes, tag: int = GOSSIP_TAG_VOTE, origin: bytes = bytes(32)) -> bytes:
    """An fd_gossip_update_message_t (src/flamenco/gossip/fd_gossip_types.h:182-205, x86-64 layout) carrying
    txn as its vote (tag VOTE) -- or, for another tag, whatever the union holds."""
    b = bytearray(max(GOSSIP_MSG_SZ, GOSSIP_VOTE_TXN_OFF + len(txn)))   # a vote txn past 1225 bytes runs past the frame
    b[0] = tag
    b[1:33] = origin[:32].ljust(32, b"\0")
    b[GOSSIP_VOTE_TXN_SZ_OFF:GOSSIP_VOTE_TXN_SZ_OFF + 8] = len(txn).to_bytes(8, "little")
    b[GOSSIP_VOTE_TXN_OFF:GOSSIP_VOTE_TXN_OFF + len(txn)] = txn
    return bytes(b)


def frag_bytes(payload: bytes, bundle_id: int = 0) -> bytes:
    h = np.zeros(1, TXNM_DTYPE)
    h["payload_sz"] = len(payload)
    h["bundle_id"] = bundle_id
    return h.tobytes() + bytes(payload)


class VTile:
    """One GPU verify tile (fdgpu_vtile_t)."""

    def __init__(self, device: int = 0, batch_txn: int = 1024, tcache_depth: int = 1 << 16, seed: int = 0x5eed,
                 out_dcache_bytes: int | None = None, semantics: int = 0, service: "Service | None" = None,
                 client: int = 0, **opts):
        """opts: fdgpu_vtile_opts_t fields (nctx, host_dedup_tag, small_max, min_batch, max_wait_ns,
        copy_wait_ns, copy_min); 0 / absent = default.  service: a tile served by that verify service as
        `client` (fdgpu_vtile_new_svc: no GPU call in this tile)."""
        self.L = load()
        out_dcache_bytes = out_dcache_bytes or (6 * batch_txn + 64) * 2304
        o = VTileOpts(**opts)
        self.service = service
        if service is not None:
            self.p = self.L.fdgpu_vtile_new_svc(service.p, client, tcache_depth, seed, ctypes.byref(o))
            if self.p:
                service._tiles.add(self)
        else:
            self.p = self.L.fdgpu_vtile_new_opts(device, batch_txn, tcache_depth, seed, out_dcache_bytes, semantics,
                                                 ctypes.byref(o))
        if not self.p:
            raise RuntimeError("fdgpu_vtile_new failed: " + load_engine().fdgpu_last_error().decode())
        self.seed = seed
        self.dcache = self.L.fdgpu_vtile_out_dcache(self.p)

    def during_frag(self, frag: bytes, seq: int, tsorig: int = 0, in_idx: int = 0) -> int:
        """fdgpu_vtile_during_frag of a frag from in link in_idx (its kind: set_in)."""
        b = np.frombuffer(frag, np.uint8)
        return self.L.fdgpu_vtile_during_frag(self.p, in_idx, b.ctypes.data, len(frag), seq, tsorig)

    def during_frag_at(self, addr: int, sz: int, seq: int, tsorig: int = 0, in_idx: int = 0) -> int:
        """during_frag on a frag already in memory at addr (zero-copy intake: inside a registered in dcache)."""
        return self.L.fdgpu_vtile_during_frag(self.p, in_idx, addr, sz, seq, tsorig)

    def during_frag_chunk(self, in_idx: int, seq: int, sig: int, chunk: int, sz: int, ctl: int = 0,
                          tsorig: int = 0) -> int:
        """fdgpu_vtile_during_frag_chunk: the stem's during_frag (in_idx, seq, sig, chunk, sz, ctl)."""
        return self.L.fdgpu_vtile_during_frag_chunk(self.p, in_idx, seq, sig, chunk, sz, ctl, tsorig)

    def set_in(self, in_idx: int, in_kind: int, mem: int = 0, chunk0: int = 0, wmark: int = 0) -> int:
        """fdgpu_vtile_set_in: in link in_idx's kind and data region (chunk c at mem + 64 c)."""
        return int(self.L.fdgpu_vtile_set_in(self.p, in_idx, in_kind, mem or None, chunk0, wmark))

    def set_round_robin(self, idx: int, cnt: int):
        self.L.fdgpu_vtile_set_round_robin(self.p, idx, cnt)

    def before_frag(self, in_idx: int, seq: int, sig: int) -> bool:
        """fdgpu_vtile_before_frag: True = this tile skips the frag (fd_verify_tile.c:36-59)."""
        return bool(self.L.fdgpu_vtile_before_frag(self.p, in_idx, seq, sig))

    def oldest_pending(self) -> tuple[int, int]:
        """(seq, in_idx) of the oldest frag not yet returned by after_frags (~0 both: none)."""
        li = ctypes.c_ulong(0)
        s = self.L.fdgpu_vtile_oldest_pending_seq(self.p, ctypes.byref(li))
        return int(s), int(li.value)

    def during_frag_overrun(self) -> int:
        return int(self.L.fdgpu_vtile_during_frag_overrun(self.p))

    def set_in_links(self, mcaches) -> int:
        """fdgpu_vtile_set_in_links: zero-copy intake from len(mcaches) links (entries may be None)."""
        arr = (ctypes.c_void_p * len(mcaches))(*[m or None for m in mcaches])
        return int(self.L.fdgpu_vtile_set_in_links(self.p, arr, len(mcaches)))

    def set_in_link(self, mcache=None) -> int:
        """Switch to zero-copy intake (fdgpu_vtile_set_in_link); mcache: an in-link mcache handle or None."""
        return int(self.L.fdgpu_vtile_set_in_link(self.p, mcache))

    def overruns(self) -> int:
        return int(self.L.fdgpu_vtile_overruns(self.p))

    def copy(self, blocking: bool = False) -> int:
        """fdgpu_vtile_copy: start (and, blocking, wait for) the GPU copy of every frag taken so far."""
        return int(self.L.fdgpu_vtile_copy(self.p, 1 if blocking else 0))

    def copy_state(self, link: int = 0) -> tuple[int, int]:
        """(frags of `link` not yet known copied, 1 + seq of its last frag known copied)."""
        cn = ctypes.c_ulong(0)
        n = self.L.fdgpu_vtile_copy_state(self.p, link, ctypes.byref(cn))
        return int(n), int(cn.value)

    def flush(self):
        return self.L.fdgpu_vtile_flush(self.p)

    def housekeep(self, max_inflight: int = 1) -> int:
        """fdgpu_vtile_housekeep: adaptive batching (launch the filling batch when there is room)."""
        return int(self.L.fdgpu_vtile_housekeep(self.p, max_inflight))

    def after_frags(self, max_n: int = 4096, blocking: bool = False):
        out = (Done * max_n)()
        n = self.L.fdgpu_vtile_after_frags(self.p, out, max_n, 1 if blocking else 0)
        return [(d.seq, d.result, d.chunk, d.sz, d.tag, d.in_idx) for d in out[:n]]

    def pending(self) -> int:
        return int(self.L.fdgpu_vtile_pending(self.p))

    def metrics(self):
        m = (ctypes.c_ulong * 5)()
        self.L.fdgpu_vtile_metrics(self.p, m)
        return list(m)

    def gpu_metrics(self) -> dict:
        m = GpuMetrics()
        self.L.fdgpu_vtile_gpu_metrics(self.p, ctypes.byref(m))
        return m.as_dict()

    def faulted(self) -> int:
        return int(self.L.fdgpu_vtile_faulted(self.p))

    def recover(self) -> int:
        return int(self.L.fdgpu_vtile_recover(self.p))

    def debug_fault(self, k: int):
        self.L.fdgpu_vtile_debug_fault(self.p, k)

    def debug_fail_launch(self, k: int):
        """Test hook: the tile's launch thread fails every batch launch of engine context k from now on."""
        self.L.fdgpu_vtile_debug_fail_launch(self.p, k)

    def set_svc_region(self, rid: int, base: int, sz: int) -> int:
        return int(self.L.fdgpu_vtile_set_svc_region(self.p, rid, base, sz))

    def record(self, chunk: int, sz: int) -> bytes:
        return ctypes.string_at(self.dcache + chunk * CHUNK_SZ, sz)

    def close(self):
        if self.p:
            self.L.fdgpu_vtile_delete(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stream_bench(payload: np.ndarray, off: np.ndarray, sz: np.ndarray, n_frags: int, tiles: int = 4,
                 batch_txn: int = 4096, max_inflight: int = 1, mcache_depth: int = 1 << 16, rate_fps: float = 0.0,
                 device: int = 0, zero_copy: bool = False) -> dict:
    L = load()
    payload = np.ascontiguousarray(payload, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    sz = np.ascontiguousarray(sz, np.uint16)
    st = StreamStats()
    rc = L.fdgpu_stream_bench(device, payload.ctypes.data, off.ctypes.data, sz.ctypes.data, len(off), n_frags, tiles,
                              batch_txn, max_inflight, mcache_depth, rate_fps, 1 if zero_copy else 0, ctypes.byref(st))
    if rc:
        raise RuntimeError(f"fdgpu_stream_bench: {rc} " + load_engine().fdgpu_last_error().decode())
    return st.as_dict()


def gpu_numa_node(device: int, sysfs_root: str | None = None) -> int:
    """fdgpu_gpu_numa_node_sysfs: HIP device -> NUMA node from sysfs alone (no GPU call), -1 if unknown."""
    return int(load().fdgpu_gpu_numa_node_sysfs(sysfs_root.encode() if sysfs_root else None, device))


class Service:
    """A verify service segment (fdgpu_vsvc_t): create (the service's process) or join (a tile process)."""

    def __init__(self, path: str | None, *, create: bool, clients: int = 1, batch_txn: int = 8192,
                 out_dcache_bytes: int | None = None, timeout_s: float = 30.0, **cfg):
        self.L = load()
        if create:
            c = VsvcCfg(clients=clients, batch_txn=batch_txn,
                        out_dcache_bytes=out_dcache_bytes or (6 * batch_txn + 64) * 2304, **cfg)
            self.p = self.L.fdgpu_vsvc_new(path.encode() if path else None, ctypes.byref(c))
        else:
            self.p = self.L.fdgpu_vsvc_join(path.encode(), timeout_s)
        if not self.p:
            raise RuntimeError(f"fdgpu_vsvc_{'new' if create else 'join'}({path}) failed")
        import weakref
        self._tiles = weakref.WeakSet()      # served tiles of this process: closed before the segment is unmapped

    def add_region(self, rid: int, base: int, sz: int) -> int:
        return int(self.L.fdgpu_vsvc_add_region(self.p, rid, base, sz))

    def start(self, device: int = 0) -> int:
        return int(self.L.fdgpu_vsvc_start(self.p, device))

    def poll(self) -> int:
        return int(self.L.fdgpu_vsvc_poll(self.p))

    def pending(self) -> int:
        return int(self.L.fdgpu_vsvc_pending(self.p))

    def debug_serve(self, codes: np.ndarray, fp: int = 100) -> int:
        """CPU loopback (no GPU): complete every request taken so far with codes[request index % len(codes)]."""
        codes = np.ascontiguousarray(codes, np.int32)
        return int(self.L.fdgpu_vsvc_debug_serve(self.p, codes.ctypes.data, len(codes), fp))

    def stats(self) -> dict:
        st = VsvcStats()
        self.L.fdgpu_vsvc_stats(self.p, ctypes.byref(st))
        return st.as_dict()

    def close(self):
        if getattr(self, "p", None):
            for t in list(getattr(self, "_tiles", ())):
                t.close()
            self.L.fdgpu_vsvc_delete(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def tiles_of(tiles: int, gpus: int, proc: int) -> list[int]:
    """The verify tiles process `proc` runs (tile i drives GPU i % gpus)."""
    out = (ctypes.c_int * max(tiles, 1))()
    n = load().fdgpu_link_tiles_of(tiles, gpus, proc, out)
    return list(out[:n])


def _cfg(n_frags, tiles, gpus, batch_txn, max_inflight, rate_fps, zero_copy, reliable, producers=1, nctx=0, prof=0,
         out_mult=0, copy_wait_ns=0, copy_min=0, gather_cus=0, max_uncopied=0, pf_dist=0, no_huge_pages=0, cu_split=0, cu_exclusive=0,
         launcher=0, copy_threads=0, min_batch=0, small_max=0, hk_ns=0, lat_share=0, svc=0, trace_cap=0,
         prod_node=None) -> StreamCfg:
    """prod_node: per producer q, the NUMA node of its mcache, dcache part and thread (None / -1: unplaced)."""
    pn = (ctypes.c_int * 16)(*[(n + 1 if n is not None and n >= 0 else 0) for n in list(prod_node or [])[:16]])
    return StreamCfg(prod_node=pn, n_frags=n_frags, batch_txn=batch_txn, max_inflight=max_inflight, rate_fps=rate_fps, tiles=tiles,
                     gpus=gpus, zero_copy=1 if zero_copy else 0, reliable=1 if reliable else 0, producers=producers,
                     nctx=nctx, prof=prof, out_mult=out_mult, copy_wait_ns=copy_wait_ns, copy_min=copy_min,
                     gather_cus=gather_cus, max_uncopied=max_uncopied, pf_dist=pf_dist, no_huge_pages=no_huge_pages, cu_split=cu_split,
                     cu_exclusive=cu_exclusive, launcher=launcher, copy_threads=copy_threads, min_batch=min_batch,
                     small_max=small_max, hk_ns=hk_ns, lat_share=lat_share, svc=1 if svc else 0, trace_cap=trace_cap)


def stream_run(payload: np.ndarray, off: np.ndarray, sz: np.ndarray, n_frags: int, tiles: int = 4,
               batch_txn: int = 4096, max_inflight: int = 1, mcache_depth: int = 1 << 16, rate_fps: float = 0.0,
               device: int = 0, zero_copy: bool = True, reliable: bool = True, producers: int = 1, **tune) -> dict:
    """One process: `producers` producer links + `tiles` verify tiles on `device`, private memory (G = 1).
    tune: nctx, prof, out_mult, copy_wait_ns, copy_min (fdgpu_stream_cfg_t)."""
    L = load()
    payload = np.ascontiguousarray(payload, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    sz = np.ascontiguousarray(sz, np.uint16)
    cfg = _cfg(n_frags, tiles, 1, batch_txn, max_inflight, rate_fps, zero_copy, reliable, producers, **tune)
    st = StreamStats()
    rc = L.fdgpu_stream_run(device, ctypes.byref(cfg), payload.ctypes.data, off.ctypes.data, sz.ctypes.data, len(off),
                            mcache_depth, ctypes.byref(st))
    if rc:
        raise RuntimeError(f"fdgpu_stream_run: {rc} " + load_engine().fdgpu_last_error().decode())
    return st.as_dict()


class Link:
    """The configs[4] link shared by several processes (fdgpu_link_t): create (with the payloads) or join."""

    def __init__(self, path: str | None, *, create: bool, payload=None, off=None, sz=None, n_frags: int = 0,
                 tiles: int = 1, gpus: int = 1, batch_txn: int = 8192, max_inflight: int = 1, rate_fps: float = 0.0,
                 zero_copy: bool = True, reliable: bool = True, mcache_depth: int = 1 << 18, timeout_s: float = 300.0,
                 producers: int = 1, **tune):
        self.L = load()
        self.path = path
        if create:
            payload = np.ascontiguousarray(payload, np.uint8)
            off = np.ascontiguousarray(off, np.uint32)
            sz = np.ascontiguousarray(sz, np.uint16)
            cfg = _cfg(n_frags, tiles, gpus, batch_txn, max_inflight, rate_fps, zero_copy, reliable, producers, **tune)
            self.p = self.L.fdgpu_link_new(path.encode() if path else None, ctypes.byref(cfg), payload.ctypes.data,
                                           off.ctypes.data, sz.ctypes.data, len(off), mcache_depth)
        else:
            self.p = self.L.fdgpu_link_join(path.encode(), timeout_s)
        if not self.p:
            raise RuntimeError(f"fdgpu_link_{'new' if create else 'join'}({path}) failed")

    def cfg(self) -> dict:
        c = StreamCfg()
        self.L.fdgpu_link_cfg(self.p, ctypes.byref(c))
        return {k: (list(getattr(c, k)) if k == "prod_node" else getattr(c, k)) for k, _ in c._fields_}

    def joined(self) -> int:
        return int(self.L.fdgpu_link_joined(self.p))

    def mcache(self):
        return self.L.fdgpu_link_mcache(self.p)

    def dcache(self) -> int:
        return int(self.L.fdgpu_link_dcache(self.p))

    def run(self, proc: int, device: int, run_producer: bool) -> int:
        return int(self.L.fdgpu_link_run(self.p, proc, device, 1 if run_producer else 0))

    def set_trace(self, cap: int) -> None:
        """fdgpu_link_set_trace: record up to cap verdicts of each of this process's tiles (before run)."""
        if self.L.fdgpu_link_set_trace(self.p, cap):
            raise RuntimeError("fdgpu_link_set_trace failed")

    def trace(self, tile: int, cap: int) -> np.ndarray:
        out = np.zeros(cap, TRACE_DTYPE)
        n = int(self.L.fdgpu_link_trace(self.p, tile, out.ctypes.data, cap))
        return out[:n]

    def anomalies(self, tile: int) -> tuple[int, list[dict]]:
        """fdgpu_link_anomalies: (count, the first few) verdicts of `tile` neither published nor overrun."""
        out = np.zeros(8, ANOM_DTYPE)
        n = int(self.L.fdgpu_link_anomalies(self.p, tile, out.ctypes.data, 8))
        return n, [{k: int(e[k]) for k in ANOM_DTYPE.names} for e in out[:min(n, 8)]]

    def anomaly_results(self, tile: int) -> list[int]:
        """fdgpu_link_anomaly_results: `tile`'s anomalous verdicts by result code (index = PUBLISH .. GPU_FAULT)."""
        cnt = np.zeros(8, np.uint64)
        self.L.fdgpu_link_anomaly_results(self.p, tile, cnt.ctypes.data)
        return [int(x) for x in cnt]

    def placement(self) -> dict:
        """fdgpu_link_placement: per producer the NUMA node of its dcache part / mcache, and the link's bytes in
        2 MiB pages in this process's mapping."""
        dc, mc = (ctypes.c_int * 16)(), (ctypes.c_int * 16)()
        hb, mb = ctypes.c_ulong(0), ctypes.c_ulong(0)
        n = self.L.fdgpu_link_placement(self.p, dc, mc, ctypes.byref(hb), ctypes.byref(mb))
        return {"dcache_nodes": list(dc[:n]), "mcache_nodes": list(mc[:n]), "huge_mb": round(hb.value / 2**20, 1),
                "map_mb": round(mb.value / 2**20, 1)}

    def svc_stats(self) -> dict:
        """Served tiles (cfg svc): this process's verify service after run (fdgpu_link_svc_stats)."""
        st, cpu = VsvcStats(), ctypes.c_int(-1)
        self.L.fdgpu_link_svc_stats(self.p, ctypes.byref(st), ctypes.byref(cpu))
        return dict(st.as_dict(), cpu=int(cpu.value))

    def result(self, timeout_s: float = 120.0) -> dict:
        st = StreamStats()
        rc = self.L.fdgpu_link_result(self.p, timeout_s, ctypes.byref(st))
        if rc:
            raise RuntimeError(f"fdgpu_link_result: {rc}")
        return st.as_dict()

    def close(self):
        if getattr(self, "p", None):
            self.L.fdgpu_link_delete(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
