"""ctypes binding of libhdrf.so (include/hdrf.h) — the product path.

There is no CPU fallback: if the HIP library is missing or no GPU is present the calls
raise.  `build()` compiles the library in-tree for gfx950.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HDRF_LIB_PATH") or os.path.join(_HERE, "_build", "libhdrf.so")   # env: A/B builds

HDRF_ERRORS = {
    -1: "HDRF_E_INVAL", -2: "HDRF_E_HIP", -3: "HDRF_E_NOMEM", -4: "HDRF_E_CAPACITY",
    -5: "HDRF_E_NOTFOUND", -6: "HDRF_E_UNSUPPORTED", -7: "HDRF_E_DEVICE",
}

# every symbol include/hdrf.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "hdrf_default_cfg", "hdrf_open", "hdrf_close", "hdrf_last_error", "hdrf_digest_len",
    "hdrf_reduce_block", "hdrf_reduce_batch", "hdrf_batch_info", "hdrf_batch_offsets",
    "hdrf_batch_digests", "hdrf_batch_is_new", "hdrf_batch_placement", "hdrf_index_get",
    "hdrf_index_count", "hdrf_index_dump", "hdrf_allocator", "hdrf_recipe_get", "hdrf_block_length",
    "hdrf_container_read", "hdrf_dev_alloc", "hdrf_dev_free", "hdrf_memcpy_h2d", "hdrf_memcpy_d2h",
    "hdrf_synchronize", "hdrf_corpus_fill", "hdrf_corpus_fill_kind", "hdrf_stage_times", "hdrf_reset",
    "hdrf_gx_layout_get", "hdrf_gx_front", "hdrf_gx_front_launch", "hdrf_gx_front_wait", "hdrf_gx_owner", "hdrf_gx_decide", "hdrf_gx_flush",
    "hdrf_gx_place", "hdrf_gx_x3_counts", "hdrf_gx_commit", "hdrf_gx_stream", "hdrf_gx_alloc_io", "hdrf_gx_piece", "hdrf_gx_compress", "hdrf_get_stats", "hdrf_submit_batch", "hdrf_wait_batch",
    "hdrf_batch_nblocks", "hdrf_reconstruct", "hdrf_reconstruct_block", "hdrf_submit_host",
    "hdrf_host_alloc", "hdrf_host_free", "hdrf_stream_block", "hdrf_stream_block_host", "hdrf_lz4_file_decode",
    "hdrf_stream_file_decode", "hdrf_gzip_match_pass", "hdrf_gzip_parse", "hdrf_container_load",
    "hdrf_container_unload", "hdrf_index_load", "hdrf_allocator_load", "hdrf_recipe_load",
    "hdrf_drain_containers", "hdrf_ticket_take", "hdrf_ticket_cancel", "hdrf_reduce_block_ticketed",
    "hdrf_probe_stats", "hdrf_rx_begin", "hdrf_append_packet", "hdrf_submit_slot", "hdrf_submit_slots", "hdrf_rx_cancel",
    "hdrf_gx_read_locate", "hdrf_gx_read_fill", "hdrf_gx_flush_fn", "hdrf_gx_alloc_scan",
    "hdrf_set_lzop_mtime", "hdrf_gx_flush_fn_dev", "hdrf_gx_alloc_scan_dev", "hdrf_gx_place_launch",
    "hdrf_gx_place_wait", "hdrf_gx_sync", "hdrf_reset_async",
]

ALLOC_STATE_BYTES = 128     # HDRF_ALLOC_STATE_BYTES
PIPELINE_DEPTH = 5          # HDRF_PIPELINE_DEPTH: batches in flight


# per-stage timers of hdrf_stage_times (kernel names in parentheses)
STAGES = ["walk(lane_walk_kernel)", "stitch(repair/path/count/scan/copy/fallback)", "sha(sha_chunk_kernel)",
          "sha_tail(none: padding inside the sha kernel)", "index_claim(idx_claim_kernel)", "index_apply(idx_apply_kernel)",
          "index_slow_decide(idx_slow/decide)", "scan(tile/chunk_scan)", "flush(flush_kernel)",
          "place(place_kernel)", "compress(lz4_seg/lz4_pack)", "gmax(gmax_kernel)",
          # node-global contexts (hdrf_gx_*): the front's local aggregation, the back phases and the
          # gaps on the back stream the caller's exchanges fill (X1 includes the host's turn-around)
          "gx_local(scratch claim/apply/decide + gx_emit)", "gx_owner(own_claim..own_finish)",
          "gx_decide(gx_decide + x3want)", "gx_flush_fn(fn_info/fn_chain/fn_pack)", "gx_alloc_scan(gx_scan_kernel)",
          "gx_place_meta(place_kernel part 1)", "gx_commit(own_commit)", "gx_x1(X1 all-to-all + host)",
          "gx_x2(X2 all-to-all)", "gx_allgather(flush descriptors)", "gx_x3(X3 all-to-all + host)"]


class HdrfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{HDRF_ERRORS.get(code, code)}: {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [
        ("hasher", ctypes.c_int32), ("compressor", ctypes.c_int32), ("window", ctypes.c_int32),
        ("max_chunk", ctypes.c_int32), ("n_thread", ctypes.c_int32), ("min_mt_chunks", ctypes.c_int32),
        ("container_max", ctypes.c_uint32), ("device", ctypes.c_int32), ("max_block_bytes", ctypes.c_int64),
        ("max_batch_blocks", ctypes.c_int32), ("index_log2", ctypes.c_int32), ("arena_slots", ctypes.c_int64),
        ("segment_bytes", ctypes.c_int32), ("keep_recipes", ctypes.c_int32), ("timing", ctypes.c_int32),
        ("debug_tag_bits", ctypes.c_int32), ("n_ranks", ctypes.c_int32), ("rank", ctypes.c_int32),
        ("retain_containers", ctypes.c_int32),
    ]


class ContainerEvent(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint32), ("closed", ctypes.c_int32), ("file_off", ctypes.c_int64),
                ("nbytes", ctypes.c_int64), ("data_off", ctypes.c_int64)]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in ("blocks", "chunks", "logical_bytes", "new_bytes", "closed_containers",
                                             "closed_raw_bytes", "closed_file_bytes", "open_bytes", "recipe_bytes")]


class GxLayout(ctypes.Structure):
    _fields_ = [("cap", ctypes.c_int64), ("x1_words", ctypes.c_int32), ("x2_words", ctypes.c_int32),
                ("x3_words", ctypes.c_int32), ("depth", ctypes.c_int32), ("fn_bytes", ctypes.c_int64)]


class BlockResult(ctypes.Structure):
    _fields_ = [
        ("n_chunks", ctypes.c_int64), ("store_size", ctypes.c_int64), ("capacity", ctypes.c_int64),
        ("offsets", ctypes.POINTER(ctypes.c_uint32)), ("digests", ctypes.POINTER(ctypes.c_uint8)),
        ("is_new", ctypes.POINTER(ctypes.c_uint8)), ("container_id", ctypes.POINTER(ctypes.c_uint32)),
        ("container_pos", ctypes.POINTER(ctypes.c_uint32)),
    ]


def build(verbose=False):
    """Compile libhdrf.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    r = subprocess.run(["make", "-s", "-j8", "-C", _HERE], capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise RuntimeError("libhdrf build failed:\n" + (r.stdout or "") + (r.stderr or ""))
    return LIB_PATH


_lib = None
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p


def load():
    """Load libhdrf.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libhdrf.so not built at {LIB_PATH}: run hdrf_amd.lib.build() "
                           "(the HIP extension is required; there is no CPU path)")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "hdrf_default_cfg": (ctypes.c_int, [ctypes.POINTER(Config)]),
        "hdrf_open": (ctypes.c_int, [ctypes.POINTER(Config), ctypes.POINTER(_vp)]),
        "hdrf_close": (ctypes.c_int, [_vp]),
        "hdrf_last_error": (ctypes.c_char_p, [_vp]),
        "hdrf_digest_len": (ctypes.c_int, [_vp]),
        "hdrf_reduce_block": (ctypes.c_int, [_vp, ctypes.c_uint64, _u8p, ctypes.c_uint64, ctypes.POINTER(BlockResult)]),
        "hdrf_reduce_block_ticketed": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, _u8p, ctypes.c_uint64,
                                                      ctypes.POINTER(BlockResult)]),
        "hdrf_ticket_take": (ctypes.c_int, [_vp, _u64p]),
        "hdrf_rx_begin": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int32)]),
        "hdrf_append_packet": (ctypes.c_int, [_vp, ctypes.c_int32, _vp, ctypes.c_uint64]),
        "hdrf_submit_slot": (ctypes.c_int, [_vp, ctypes.c_int32]),
        "hdrf_submit_slots": (ctypes.c_int, [_vp, ctypes.c_int32, _vp]),
        "hdrf_rx_cancel": (ctypes.c_int, [_vp, ctypes.c_int32]),
        "hdrf_probe_stats": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                            ctypes.POINTER(ctypes.c_int64)]),
        "hdrf_ticket_cancel": (ctypes.c_int, [_vp, ctypes.c_uint64]),
        "hdrf_drain_containers": (ctypes.c_int64, [_vp, ctypes.POINTER(ContainerEvent), ctypes.c_int64, _u8p,
                                                   ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
        "hdrf_reduce_batch": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(_vp), _u64p, _u64p, _u64p]),
        "hdrf_submit_batch": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(_vp), _u64p, _u64p, _u64p]),
        "hdrf_wait_batch": (ctypes.c_int, [_vp]),
        "hdrf_submit_host": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(_vp), _u64p, _u64p]),
        "hdrf_host_alloc": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(_vp)]),
        "hdrf_host_free": (ctypes.c_int, [_vp, _vp]),
        "hdrf_lz4_file_decode": (ctypes.c_int64, [_vp, _u8p, ctypes.c_int64, _vp, ctypes.c_int64]),
        "hdrf_gzip_match_pass": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp]),
        "hdrf_gzip_parse": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, _vp, _vp]),
        "hdrf_stream_file_decode": (ctypes.c_int64, [_vp, ctypes.c_int32, _u8p, ctypes.c_int64, _vp, ctypes.c_int64]),
        "hdrf_set_lzop_mtime": (ctypes.c_int, [_vp, ctypes.c_uint32]),
        "hdrf_container_load": (ctypes.c_int, [_vp, ctypes.c_uint32, _u8p, ctypes.c_int64, ctypes.c_int32]),
        "hdrf_container_unload": (ctypes.c_int, [_vp, ctypes.c_uint32]),
        "hdrf_index_load": (ctypes.c_int, [_vp, _u8p, _u8p, ctypes.c_int64]),
        "hdrf_allocator_load": (ctypes.c_int, [_vp, _u8p, ctypes.POINTER(_vp), _i64p]),
        "hdrf_recipe_load": (ctypes.c_int, [_vp, ctypes.c_uint64, _u8p, ctypes.c_int64]),
        "hdrf_stream_block": (ctypes.c_int64, [_vp, ctypes.c_int32, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                               ctypes.c_uint64, _u64p, ctypes.c_int32, _u8p, ctypes.c_int64]),
        "hdrf_stream_block_host": (ctypes.c_int64, [_vp, ctypes.c_int32, ctypes.c_uint64, _u8p, ctypes.c_uint64,
                                                    _u64p, ctypes.c_int32, _u8p, ctypes.c_int64]),
        "hdrf_batch_nblocks": (ctypes.c_int, [_vp]),
        "hdrf_reconstruct": (ctypes.c_int64, [_vp, _u8p, ctypes.c_int64, _vp, ctypes.c_int64]),
        "hdrf_reconstruct_block": (ctypes.c_int64, [_vp, ctypes.c_uint64, _u8p, ctypes.c_int64]),
        "hdrf_gx_read_locate": (ctypes.c_int64, [_vp, _u8p, ctypes.c_int64, _vp]),
        "hdrf_gx_flush_fn": (ctypes.c_int64, [_vp, _vp, ctypes.c_int64]),
        "hdrf_gx_alloc_scan": (ctypes.c_int32, [_vp, _vp, _vp, _u8p, _u8p]),
        "hdrf_gx_read_fill": (ctypes.c_int64, [_vp, _vp, ctypes.c_int64, _vp, ctypes.c_int64]),
        "hdrf_batch_info": (ctypes.c_int, [_vp, ctypes.c_int32, _i64p, _i64p]),
        "hdrf_batch_offsets": (ctypes.c_int, [_vp, ctypes.c_int32, _u32p, ctypes.c_int64]),
        "hdrf_batch_digests": (ctypes.c_int, [_vp, ctypes.c_int32, _u8p, ctypes.c_int64]),
        "hdrf_batch_is_new": (ctypes.c_int, [_vp, ctypes.c_int32, _u8p, ctypes.c_int64]),
        "hdrf_batch_placement": (ctypes.c_int, [_vp, ctypes.c_int32, _u32p, _u32p, ctypes.c_int64]),
        "hdrf_index_get": (ctypes.c_int, [_vp, _u8p, _u8p]),
        "hdrf_index_count": (ctypes.c_int64, [_vp]),
        "hdrf_index_dump": (ctypes.c_int64, [_vp, _u8p, _u8p, ctypes.c_int64]),
        "hdrf_allocator": (ctypes.c_int, [_vp, _u8p]),
        "hdrf_recipe_get": (ctypes.c_int64, [_vp, ctypes.c_uint64, _u8p, ctypes.c_int64]),
        "hdrf_block_length": (ctypes.c_int64, [_vp, ctypes.c_uint64]),
        "hdrf_container_read": (ctypes.c_int64, [_vp, ctypes.c_uint32, _u8p, ctypes.c_int64,
                                                 ctypes.POINTER(ctypes.c_int32)]),
        "hdrf_dev_alloc": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.POINTER(_vp)]),
        "hdrf_dev_free": (ctypes.c_int, [_vp, _vp]),
        "hdrf_memcpy_h2d": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64]),
        "hdrf_memcpy_d2h": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64]),
        "hdrf_synchronize": (ctypes.c_int, [_vp]),
        "hdrf_corpus_fill": (ctypes.c_int, [_vp, _vp, _u32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_uint64]),
        "hdrf_corpus_fill_kind": (ctypes.c_int, [_vp, _vp, _u32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                 ctypes.c_uint64, ctypes.c_int32]),
        "hdrf_stage_times": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int32, ctypes.c_int32]),
        "hdrf_reset": (ctypes.c_int, [_vp]),
        "hdrf_reset_async": (ctypes.c_int, [_vp]),
        "hdrf_get_stats": (ctypes.c_int, [_vp, ctypes.POINTER(Stats)]),
        "hdrf_gx_layout_get": (ctypes.c_int, [_vp, ctypes.POINTER(GxLayout)]),
        "hdrf_gx_front_launch": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(_vp), _u64p, _u64p, _u64p,
                                                ctypes.c_uint32, _vp]),
        "hdrf_gx_front_wait": (ctypes.c_int, [_vp, _i64p]),
        "hdrf_gx_front": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(_vp), _u64p, _u64p, _u64p,
                                         ctypes.c_uint32, _vp, _i64p]),
        "hdrf_gx_owner": (ctypes.c_int, [_vp, _vp, _i64p, _vp]),
        "hdrf_gx_decide": (ctypes.c_int, [_vp, _vp]),
        "hdrf_gx_flush": (ctypes.c_int, [_vp, _u8p, _u8p]),
        "hdrf_gx_place": (ctypes.c_int, [_vp, _u8p, _vp, _i64p]),
        "hdrf_gx_x3_counts": (ctypes.c_int, [_vp, _i64p]),
        "hdrf_gx_commit": (ctypes.c_int, [_vp, _vp, _i64p]),
        "hdrf_gx_stream": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p)]),
        "hdrf_gx_alloc_io": (ctypes.c_int, [_vp, _u8p, _u8p]),
        "hdrf_gx_piece": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, _vp, ctypes.c_int32]),
        "hdrf_gx_compress": (ctypes.c_int, [_vp]),
        "hdrf_gx_flush_fn_dev": (ctypes.c_int, [_vp, _vp]),
        "hdrf_gx_alloc_scan_dev": (ctypes.c_int, [_vp, _vp]),
        "hdrf_gx_place_launch": (ctypes.c_int, [_vp, _u8p, _vp]),
        "hdrf_gx_place_wait": (ctypes.c_int, [_vp, _i64p]),
        "hdrf_gx_sync": (ctypes.c_int, [_vp]),
    }
    ab_build = bool(os.environ.get("HDRF_LIB_PATH"))
    for name, (res, args) in sig.items():
        if ab_build and not hasattr(L, name):
            continue                 # an older build under A/B (HDRF_LIB_PATH) lacks a newer entry point
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def default_config(**kw):
    cfg = Config()
    load().hdrf_default_cfg(ctypes.byref(cfg))
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise KeyError(k)
        setattr(cfg, k, v)
    return cfg


def _p(a, t=_u8p):
    return a.ctypes.data_as(t)


def _u8(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(data, dtype=np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8)


class Context:
    """One DataNode's reduction state on one GPU (index, containers, allocator, recipes)."""

    def __init__(self, cfg=None, **kw):
        self.L = load()
        self.cfg = cfg if cfg is not None else default_config(**kw)
        h = _vp()
        rc = self.L.hdrf_open(ctypes.byref(self.cfg), ctypes.byref(h))
        if rc != 0:
            raise HdrfError(rc, "hdrf_open failed")
        self._h = h
        self.H = self.L.hdrf_digest_len(h)
        self._pinned = {}

    def _ck(self, rc):
        if rc < 0:
            raise HdrfError(rc, self.L.hdrf_last_error(self._h).decode())
        return rc

    def close(self):
        if getattr(self, "_h", None):
            self.L.hdrf_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- write path ---------------------------------------------------------------------
    def reduce_block(self, data, block_id, ticket=None):
        """hdrf_reduce_block (or hdrf_reduce_block_ticketed with an arrival ticket from
        ticket_take(): waits for every earlier ticket; safe to call from any thread)."""
        a = _u8(data)
        buf = a if a.size else np.zeros(1, np.uint8)
        cap = a.size // (self.cfg.window + 2) + 2
        offs = np.zeros(cap, np.uint32)
        digs = np.zeros(cap * self.H, np.uint8)
        isnew = np.zeros(cap, np.uint8)
        cid = np.zeros(cap, np.uint32)
        pos = np.zeros(cap, np.uint32)
        r = BlockResult(0, 0, cap, _p(offs, _u32p), _p(digs), _p(isnew), _p(cid, _u32p), _p(pos, _u32p))
        if ticket is None:
            self._ck(self.L.hdrf_reduce_block(self._h, block_id, _p(buf), a.size, ctypes.byref(r)))
        else:
            self._ck(self.L.hdrf_reduce_block_ticketed(self._h, ticket, block_id, _p(buf), a.size, ctypes.byref(r)))
        n = r.n_chunks
        return {"offsets": offs[:n].copy(), "digests": digs[:n * self.H].reshape(n, self.H).copy(),
                "is_new": isnew[:n].copy(), "container_id": cid[:n].copy(), "container_pos": pos[:n].copy(),
                "store_size": r.store_size}

    def rx_begin(self, block_id):
        r = ctypes.c_int32()
        self._ck(self.L.hdrf_rx_begin(self._h, block_id, ctypes.byref(r)))
        return r.value

    def append_packet(self, rx, ptr, nbytes):
        """Host address + length of one received packet (copied before the call returns)."""
        self._ck(self.L.hdrf_append_packet(self._h, rx, ptr, nbytes))

    def submit_slot(self, rx):
        self._ck(self.L.hdrf_submit_slot(self._h, rx))

    def submit_slots(self, rxs):
        """Received blocks (receive buffers in arrival order) submitted as one batch."""
        a = (ctypes.c_int32 * len(rxs))(*rxs)
        self._ck(self.L.hdrf_submit_slots(self._h, len(rxs), a))

    def rx_cancel(self, rx):
        self._ck(self.L.hdrf_rx_cancel(self._h, rx))

    def probe_stats(self):
        """(probe_sum, probe_max, chunks) of the last completed batch."""
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._ck(self.L.hdrf_probe_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def ticket_take(self):
        t = ctypes.c_uint64()
        self._ck(self.L.hdrf_ticket_take(self._h, ctypes.byref(t)))
        return t.value

    def ticket_cancel(self, ticket):
        self._ck(self.L.hdrf_ticket_cancel(self._h, ticket))

    def drain_containers(self, buf_bytes=64 << 20, max_events=4096):
        """hdrf_drain_containers until nothing is pending: [(id, closed, file_off, bytes)] in order."""
        out = []
        ev = (ContainerEvent * max_events)()
        need = ctypes.c_int64()
        cap = buf_bytes
        while True:
            buf = np.zeros(max(cap, 1), np.uint8)
            n = self.L.hdrf_drain_containers(self._h, ev, max_events, _p(buf), cap, ctypes.byref(need))
            if n == -4 and need.value > cap:                 # HDRF_E_CAPACITY: the next event alone
                cap = int(need.value)
                continue
            self._ck(n)
            if n == 0:
                return out
            for e in ev[:n]:
                out.append((e.id, e.closed, e.file_off, buf[e.data_off:e.data_off + e.nbytes].tobytes()))

    def drain_into(self, ptr, cap, max_events=4096):
        """hdrf_drain_containers into caller memory (e.g. pinned) until nothing is pending; the
        bytes stay there (the bench's DataNode shape): returns (events, bytes) handed out."""
        ev = (ContainerEvent * max_events)()
        need = ctypes.c_int64()
        nev = nbytes = 0
        while True:
            n = self._ck(self.L.hdrf_drain_containers(self._h, ev, max_events, ctypes.cast(ptr, _u8p), cap,
                                                      ctypes.byref(need)))
            if n == 0:
                return nev, nbytes
            nev += n
            nbytes += sum(e.nbytes for e in ev[:n])

    def reduce_batch(self, dev_ptrs, lens, readable, block_ids):
        n = len(dev_ptrs)
        ptrs = (_vp * n)(*dev_ptrs)
        ln = np.ascontiguousarray(lens, np.uint64)
        rd = np.ascontiguousarray(readable, np.uint64)
        ids = np.ascontiguousarray(block_ids, np.uint64)
        self._ck(self.L.hdrf_reduce_batch(self._h, n, ptrs, _p(ln, _u64p), _p(rd, _u64p), _p(ids, _u64p)))

    def submit_batch(self, dev_ptrs, lens, readable, block_ids):
        """Enqueue a batch (PIPELINE_DEPTH in flight at most); complete it with wait_batch() in order."""
        n = len(dev_ptrs)
        ptrs = (_vp * n)(*dev_ptrs)
        ln = np.ascontiguousarray(lens, np.uint64)
        rd = np.ascontiguousarray(readable, np.uint64)
        ids = np.ascontiguousarray(block_ids, np.uint64)
        self._ck(self.L.hdrf_submit_batch(self._h, n, ptrs, _p(ln, _u64p), _p(rd, _u64p), _p(ids, _u64p)))

    def submit_host(self, host_ptrs, lens, block_ids):
        """Enqueue a batch of HOST-resident blocks (addresses; pinned memory from host_alloc()
        overlaps the copies with the batches in flight).  The buffers must stay intact until the
        batch is completed with wait_batch()."""
        n = len(host_ptrs)
        ptrs = (_vp * n)(*host_ptrs)
        ln = np.ascontiguousarray(lens, np.uint64)
        ids = np.ascontiguousarray(block_ids, np.uint64)
        self._ck(self.L.hdrf_submit_host(self._h, n, ptrs, _p(ln, _u64p), _p(ids, _u64p)))

    def host_alloc(self, nbytes):
        """Pinned host buffer as a numpy uint8 array view (free with host_free(array))."""
        p = _vp()
        self._ck(self.L.hdrf_host_alloc(self._h, nbytes, ctypes.byref(p)))
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(p.value)
        a = np.frombuffer(buf, np.uint8, count=nbytes)
        self._pinned[a.ctypes.data] = p.value
        return a

    def host_free(self, a):
        p = self._pinned.pop(a.ctypes.data)
        self._ck(self.L.hdrf_host_free(self._h, p))

    def wait_batch(self):
        self._ck(self.L.hdrf_wait_batch(self._h))

    def lz4_file_decode(self, file, raw_cap):
        """Decode a Hadoop Lz4Codec file on the GPU -> raw bytes."""
        f = _u8(file)
        dev = self.dev_alloc(raw_cap + 64)
        try:
            n = self._ck(self.L.hdrf_lz4_file_decode(self._h, _p(f if f.size else np.zeros(1, np.uint8)), f.size,
                                                     dev, raw_cap))
            return self.d2h(dev, n).tobytes() if n else b""
        finally:
            self.dev_free(dev)

    def stream_file_decode(self, codec, file, raw_cap):
        """Decode a stream-mode block file (codec 0 SnappyCodec, 4 Lz4Codec, 5 GzipCodec) on the GPU -> raw bytes."""
        f = _u8(file)
        dev = self.dev_alloc(raw_cap + 64)
        try:
            n = self._ck(self.L.hdrf_stream_file_decode(self._h, codec, _p(f if f.size else np.zeros(1, np.uint8)),
                                                        f.size, dev, raw_cap))
            return self.d2h(dev, n).tobytes() if n else b""
        finally:
            self.dev_free(dev)

    def container_load(self, cid, file, lz4):
        f = _u8(file)
        self._ck(self.L.hdrf_container_load(self._h, cid, _p(f if f.size else np.zeros(1, np.uint8)), f.size,
                                            1 if lz4 else 0))

    def container_unload(self, cid):
        self._ck(self.L.hdrf_container_unload(self._h, cid))

    # ---- restore (index persistence) --------------------------------------------------------
    def index_load(self, keys, vals):
        k = np.ascontiguousarray(keys, np.uint8).reshape(-1)
        v = np.ascontiguousarray(vals, np.uint8).reshape(-1)
        n = v.size // 11
        self._ck(self.L.hdrf_index_load(self._h, _p(k if k.size else np.zeros(1, np.uint8)),
                                        _p(v if v.size else np.zeros(1, np.uint8)), n))

    def allocator_load(self, alloc24, open_files):
        """open_files[t]: bytes of storer range t's open container file, or None."""
        a = np.frombuffer(bytes(alloc24), np.uint8).copy()
        bufs = [np.frombuffer(f, np.uint8).copy() if f else np.zeros(1, np.uint8) for f in open_files]
        ptrs = (_vp * len(bufs))(*[b.ctypes.data for b in bufs])
        lens = np.array([len(f) if f is not None else -1 for f in open_files], np.int64)
        self._ck(self.L.hdrf_allocator_load(self._h, _p(a), ptrs, _p(lens, _i64p)))

    def recipe_load(self, block_id, recipe):
        r = np.frombuffer(bytes(recipe), np.uint8).copy()
        self._ck(self.L.hdrf_recipe_load(self._h, block_id, _p(r), r.size))

    def stream_block(self, codec, block_id, dev, nbytes, readable, writes):
        """Stream-mode scheme (compressor 4 = Lz4Codec, 0 = SnappyCodec): the file the reference
        writes for a block received as write()s of the given sizes -> bytes."""
        w = np.ascontiguousarray(writes, np.uint64)
        wp = _p(w if w.size else np.zeros(1, np.uint64), _u64p)
        cap = 16 + nbytes + nbytes // 6 + 48 * (len(w) + nbytes // 218422 + 2)
        out = np.zeros(cap, np.uint8)
        n = self._ck(self.L.hdrf_stream_block(self._h, codec, block_id, dev, nbytes, readable, wp, len(w), _p(out),
                                              cap))
        return out[:n].tobytes()

    def set_lzop_mtime(self, mtime):
        self._ck(self.L.hdrf_set_lzop_mtime(self._h, mtime))

    def stream_block_host(self, codec, block_id, data, writes):
        """hdrf_stream_block for host bytes (staged H2D by the library)."""
        d = _u8(data)
        w = np.ascontiguousarray(writes, np.uint64)
        wp = _p(w if w.size else np.zeros(1, np.uint64), _u64p)
        cap = 16 + d.size + d.size // 6 + 48 * (len(w) + d.size // 218422 + 2)
        out = np.zeros(cap, np.uint8)
        n = self._ck(self.L.hdrf_stream_block_host(self._h, codec, block_id, _p(d if d.size else np.zeros(1, np.uint8)),
                                                   d.size, wp, len(w), _p(out), cap))
        return out[:n].tobytes()

    def last_nblocks(self):
        """Blocks of the batch hdrf_batch_* currently report."""
        return self._ck(self.L.hdrf_batch_nblocks(self._h))

    def batch_info(self, b):
        n, s = ctypes.c_int64(), ctypes.c_int64()
        self._ck(self.L.hdrf_batch_info(self._h, b, ctypes.byref(n), ctypes.byref(s)))
        return n.value, s.value

    def batch_result(self, b):
        n, ss = self.batch_info(b)
        offs = np.zeros(max(n, 1), np.uint32)
        digs = np.zeros(max(n, 1) * self.H, np.uint8)
        isnew = np.zeros(max(n, 1), np.uint8)
        cid = np.zeros(max(n, 1), np.uint32)
        pos = np.zeros(max(n, 1), np.uint32)
        self._ck(self.L.hdrf_batch_offsets(self._h, b, _p(offs, _u32p), n))
        self._ck(self.L.hdrf_batch_digests(self._h, b, _p(digs), n * self.H))
        self._ck(self.L.hdrf_batch_is_new(self._h, b, _p(isnew), n))
        self._ck(self.L.hdrf_batch_placement(self._h, b, _p(cid, _u32p), _p(pos, _u32p), n))
        return {"offsets": offs[:n], "digests": digs[:n * self.H].reshape(n, self.H), "is_new": isnew[:n],
                "container_id": cid[:n], "container_pos": pos[:n], "store_size": ss}

    # ---- Redis / chunkDir views ---------------------------------------------------------
    def index_get(self, digest):
        d = np.frombuffer(bytes(digest), np.uint8).copy()
        out = np.zeros(11, np.uint8)
        return out.tobytes() if self._ck(self.L.hdrf_index_get(self._h, _p(d), _p(out))) else None

    def index_count(self):
        return self._ck(self.L.hdrf_index_count(self._h))

    def index_dump(self):
        cnt = self.index_count()
        keys = np.zeros(max(cnt, 1) * self.H, np.uint8)
        vals = np.zeros(max(cnt, 1) * 11, np.uint8)
        n = self._ck(self.L.hdrf_index_dump(self._h, _p(keys), _p(vals), cnt))
        return keys[:n * self.H].reshape(n, self.H), vals[:n * 11].reshape(n, 11)

    def allocator(self):
        out = np.zeros(24, np.uint8)
        return out.tobytes() if self._ck(self.L.hdrf_allocator(self._h, _p(out))) else None

    def recipe(self, block_id):
        n = self.L.hdrf_recipe_get(self._h, block_id, None, 0)
        if n == 0:
            return None
        if n != -4:
            self._ck(n)
        need = 4 + self.H * (2 + int(self.cfg.max_block_bytes) // (self.cfg.window + 2))
        out = np.zeros(need, np.uint8)
        m = self._ck(self.L.hdrf_recipe_get(self._h, block_id, _p(out), need))
        return out[:m].tobytes()

    def reconstruct_block(self, block_id):
        """DataConstructor(blkID, recipe).data: the block rebuilt from the index + containers."""
        n = self.block_length(block_id)
        out = np.zeros(max(n, 1), np.uint8)
        m = self._ck(self.L.hdrf_reconstruct_block(self._h, block_id, _p(out), n))
        return out[:m]

    def reconstruct(self, recipe, dev_out, cap):
        r = np.frombuffer(bytes(recipe), np.uint8).copy()
        return self._ck(self.L.hdrf_reconstruct(self._h, _p(r), r.size, dev_out, cap))

    def block_length(self, block_id):
        return self._ck(self.L.hdrf_block_length(self._h, block_id))

    def container(self, cid):
        closed = ctypes.c_int32(0)
        n = self.L.hdrf_container_read(self._h, cid, None, 0, ctypes.byref(closed))
        if n == -5:
            return None, False
        self._ck(n)
        out = np.zeros(max(n, 1), np.uint8)
        m = self._ck(self.L.hdrf_container_read(self._h, cid, _p(out), n, ctypes.byref(closed)))
        return out[:m].tobytes(), bool(closed.value)

    # ---- device memory / corpus / timing ------------------------------------------------
    def dev_alloc(self, nbytes):
        p = _vp()
        self._ck(self.L.hdrf_dev_alloc(self._h, nbytes, ctypes.byref(p)))
        return p.value

    def dev_free(self, p):
        self._ck(self.L.hdrf_dev_free(self._h, p))

    def h2d(self, dev, data):
        a = _u8(data)
        self._ck(self.L.hdrf_memcpy_h2d(self._h, dev, a.ctypes.data, a.size))

    def d2h(self, dev, nbytes):
        out = np.zeros(nbytes, np.uint8)
        self._ck(self.L.hdrf_memcpy_d2h(self._h, out.ctypes.data, dev, nbytes))
        return out

    def gzip_match_pass(self, dev, nbytes, parse=False):
        """Compressor 5 stage 1 (hdrf_gzip_match_pass): per-position chain-128 and chain-32
        longest_match answers, (len << 16) | dist, for the nbytes device bytes at dev.  With
        parse=True also stage 2 (hdrf_gzip_parse): returns (m128, m32, symbols, blocks)."""
        if nbytes == 0 and not parse:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint32)
        nb = nbytes // 16383 + 2
        bufs = [self.dev_alloc(4 * nbytes + 64) for _ in range(4)] + [self.dev_alloc(40 * nb + 64)]
        try:
            self._ck(self.L.hdrf_gzip_match_pass(self._h, dev, nbytes, bufs[0], bufs[1], bufs[2]))
            m128 = self.d2h(bufs[1], 4 * nbytes).view(np.uint32).copy()
            m32 = self.d2h(bufs[2], 4 * nbytes).view(np.uint32).copy()
            if not parse:
                return m128, m32
            self._ck(self.L.hdrf_gzip_parse(self._h, dev, nbytes, bufs[1], bufs[2], bufs[3], bufs[4], bufs[0]))
            ns, nblk = (int(x) for x in self.d2h(bufs[0], 16).view(np.int64))
            syms = self.d2h(bufs[3], 4 * ns).view(np.uint32).copy()
            blks = self.d2h(bufs[4], 40 * nblk).view(np.int64).reshape(nblk, 5).copy()
            return m128, m32, syms, blks
        finally:
            for b in bufs:
                self.dev_free(b)

    def corpus_fill(self, dev, roots, nblocks, segs_per_block, seg_bytes, seed, mixed=False):
        r = np.ascontiguousarray(roots, np.uint32)
        self._ck(self.L.hdrf_corpus_fill_kind(self._h, dev, _p(r, _u32p), nblocks, segs_per_block, seg_bytes, seed,
                                              1 if mixed else 0))

    def synchronize(self):
        self._ck(self.L.hdrf_synchronize(self._h))

    def stage_times(self, reset=False):
        out = (ctypes.c_double * len(STAGES))()
        self._ck(self.L.hdrf_stage_times(self._h, out, len(STAGES), 1 if reset else 0))
        return list(out)

    def reset(self):
        self._ck(self.L.hdrf_reset(self._h))

    def reset_async(self):
        """A fresh DataNode from the next submit on, without draining the batches in flight."""
        self._ck(self.L.hdrf_reset_async(self._h))

    def stats(self):
        st = Stats()
        self._ck(self.L.hdrf_get_stats(self._h, ctypes.byref(st)))
        return {f: getattr(st, f) for f, _ in Stats._fields_}

    # ---- node-global index phases (include/hdrf.h; orchestrated by hdrf_amd/node.py) -----
    def gx_layout(self):
        lay = GxLayout()
        self._ck(self.L.hdrf_gx_layout_get(self._h, ctypes.byref(lay)))
        return lay

    def gx_front(self, dev_ptrs, lens, readable, block_ids, gbase, x1_send):
        n = len(dev_ptrs)
        ptrs = (_vp * n)(*dev_ptrs)
        ln = np.ascontiguousarray(lens, np.uint64)
        rd = np.ascontiguousarray(readable, np.uint64)
        ids = np.ascontiguousarray(block_ids, np.uint64)
        cnt = np.zeros(self.cfg.n_ranks, np.int64)
        self._ck(self.L.hdrf_gx_front(self._h, n, ptrs, _p(ln, _u64p), _p(rd, _u64p), _p(ids, _u64p), gbase,
                                      x1_send, _p(cnt, _i64p)))
        return cnt

    def gx_front_launch(self, dev_ptrs, lens, readable, block_ids, gbase, x1_send):
        """Launch the front half of a node-global batch without waiting (overlaps the previous
        batch's back phases); gx_front_wait() returns its X1 send counts."""
        n = len(dev_ptrs)
        self._gx_keep = (_vp * n)(*dev_ptrs)
        ln = np.ascontiguousarray(lens, np.uint64)
        rd = np.ascontiguousarray(readable, np.uint64)
        ids = np.ascontiguousarray(block_ids, np.uint64)
        self._ck(self.L.hdrf_gx_front_launch(self._h, n, self._gx_keep, _p(ln, _u64p), _p(rd, _u64p), _p(ids, _u64p),
                                             gbase, x1_send))

    def gx_front_wait(self):
        cnt = np.zeros(self.cfg.n_ranks, np.int64)
        self._ck(self.L.hdrf_gx_front_wait(self._h, _p(cnt, _i64p)))
        return cnt

    def gx_owner(self, x1_recv, recv_counts, x2_send):
        rc = np.ascontiguousarray(recv_counts, np.int64)
        self._ck(self.L.hdrf_gx_owner(self._h, x1_recv, _p(rc, _i64p), x2_send))

    def gx_stream(self):
        """hipStream_t (as an int) the back phases run on: RCCL exchanges enqueued on it need no host sync."""
        s = ctypes.c_void_p()
        self._ck(self.L.hdrf_gx_stream(self._h, ctypes.byref(s)))
        return int(s.value or 0)

    def gx_decide(self, x2_recv):
        self._ck(self.L.hdrf_gx_decide(self._h, x2_recv))

    def gx_flush(self, alloc_in=None, want_out=True):
        out = np.zeros(ALLOC_STATE_BYTES, np.uint8)
        a = None if alloc_in is None else np.ascontiguousarray(alloc_in, np.uint8)
        self._ck(self.L.hdrf_gx_flush(self._h, None if a is None else _p(a), _p(out) if want_out else None))
        return out if want_out else None

    def gx_flush_fn(self):
        """This rank's flush function (int64 descriptor) for the allocator scan."""
        cap = 1 << 16
        while True:
            d = np.zeros(cap, np.int64)
            n = self.L.hdrf_gx_flush_fn(self._h, d.ctypes.data, cap)
            if n <= -1000:
                cap = int(-n - 1000)
                continue
            return d[:self._ck(n)]

    def gx_alloc_scan(self, descs):
        """Every rank's descriptor (rank order) -> (this rank's allocator in, the node's after the batch)."""
        lens = np.array([len(d) for d in descs], np.int64)
        cat = np.ascontiguousarray(np.concatenate(descs), np.int64)
        ain = np.zeros(ALLOC_STATE_BYTES, np.uint8)
        afin = np.zeros(ALLOC_STATE_BYTES, np.uint8)
        self._ck(self.L.hdrf_gx_alloc_scan(self._h, cat.ctypes.data, lens.ctypes.data, _p(ain), _p(afin)))
        return ain, afin

    def gx_place(self, alloc_final, x3_send):
        cnt = np.zeros(self.cfg.n_ranks, np.int64)
        af = None if alloc_final is None else _p(np.ascontiguousarray(alloc_final, np.uint8))
        self._ck(self.L.hdrf_gx_place(self._h, af, x3_send, _p(cnt, _i64p)))
        return cnt

    def gx_place_launch(self, alloc_final, x3_send):
        """Placement + X3 records + read-back enqueued (the arena copy on its own stream); alloc_final
        None after gx_alloc_scan_dev.  gx_place_wait() returns the X3 send counts."""
        self._gx_af = None if alloc_final is None else np.ascontiguousarray(alloc_final, np.uint8)
        self._ck(self.L.hdrf_gx_place_launch(self._h, None if self._gx_af is None else _p(self._gx_af), x3_send))

    def gx_place_wait(self):
        cnt = np.zeros(self.cfg.n_ranks, np.int64)
        self._ck(self.L.hdrf_gx_place_wait(self._h, _p(cnt, _i64p)))
        return cnt

    def gx_flush_fn_dev(self, dev_desc):
        """This rank's flush function packed on the device into dev_desc (layout.fn_bytes)."""
        self._ck(self.L.hdrf_gx_flush_fn_dev(self._h, dev_desc))

    def gx_alloc_scan_dev(self, dev_descs):
        """Compose every rank's descriptor (G x fn_bytes on the device, rank order) on the device."""
        self._ck(self.L.hdrf_gx_alloc_scan_dev(self._h, dev_descs))

    def gx_sync(self):
        """Complete the node-global batches in flight; raises a commit's device error."""
        self._ck(self.L.hdrf_gx_sync(self._h))

    def gx_read_locate(self, digests):
        """Node-global read, step 1: locations {cid, start, stop, placing rank + 1} of the recipe
        digests this rank owns (uint32 [n, 4], zero rows for the others) and how many it owns."""
        d = np.frombuffer(bytes(digests), np.uint8).copy()
        n = d.size // self.H
        loc = np.zeros((max(n, 1), 4), np.uint32)
        m = self._ck(self.L.hdrf_gx_read_locate(self._h, _p(d) if d.size else None, n, loc.ctypes.data))
        return loc[:n], m

    def gx_read_fill(self, loc, dev_out, cap):
        """Node-global read, step 3: write the chunks this rank placed at their block offsets."""
        loc = np.ascontiguousarray(loc, np.uint32)
        return self._ck(self.L.hdrf_gx_read_fill(self._h, loc.ctypes.data if loc.size else None, loc.shape[0],
                                                 dev_out, cap))

    def gx_alloc_io(self):
        """This rank's allocator state before and after its flush walk (128 B each)."""
        a = np.zeros(ALLOC_STATE_BYTES, np.uint8)
        b = np.zeros(ALLOC_STATE_BYTES, np.uint8)
        self._ck(self.L.hdrf_gx_alloc_io(self._h, _p(a), _p(b)))
        return a, b

    def gx_piece(self, cid, off, n, dev_ptr, write):
        self._ck(self.L.hdrf_gx_piece(self._h, cid, off, n, dev_ptr, 1 if write else 0))

    def gx_compress(self):
        return self._ck(self.L.hdrf_gx_compress(self._h))

    def gx_x3_counts(self):
        """X3 receive counts implied by this owner's decisions (after gx_place)."""
        cnt = np.zeros(self.cfg.n_ranks, np.int64)
        self._ck(self.L.hdrf_gx_x3_counts(self._h, _p(cnt, _i64p)))
        return cnt

    def gx_commit(self, x3_recv, recv_counts):
        rc = np.ascontiguousarray(recv_counts, np.int64)
        self._ck(self.L.hdrf_gx_commit(self._h, x3_recv, _p(rc, _i64p)))
