"""ctypes wrapper around the CPU oracle (oracle/hdrf_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package (hdrf_amd/).
Pinning status: see oracle/hdrf_oracle.h and DESIGN.md §Oracle.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libhdrf_oracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i64p = ctypes.POINTER(ctypes.c_int64)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.hdrf_oracle_chunk.argtypes = [_u8p, ctypes.c_int64, _u32p, ctypes.c_int64]
        L.hdrf_oracle_chunk.restype = ctypes.c_int64
        L.hdrf_oracle_sha1.argtypes = [_u8p, ctypes.c_uint64, _u8p]
        L.hdrf_oracle_sha224.argtypes = [_u8p, ctypes.c_uint64, _u8p]
        L.hdrf_oracle_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        L.hdrf_oracle_new.restype = ctypes.c_void_p
        L.hdrf_oracle_free.argtypes = [ctypes.c_void_p]
        L.hdrf_oracle_set_store_only.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.hdrf_oracle_reduce.argtypes = [ctypes.c_void_p, _u8p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int64, _u32p, _u8p, _u8p, _u8p, _i64p]
        L.hdrf_oracle_reduce.restype = ctypes.c_int64
        L.hdrf_oracle_index_get.argtypes = [ctypes.c_void_p, _u8p, _u8p]
        L.hdrf_oracle_index_get.restype = ctypes.c_int
        L.hdrf_oracle_index_count.argtypes = [ctypes.c_void_p]
        L.hdrf_oracle_index_count.restype = ctypes.c_int64
        L.hdrf_oracle_index_dump.argtypes = [ctypes.c_void_p, _u8p, _u8p, ctypes.c_int64]
        L.hdrf_oracle_index_dump.restype = ctypes.c_int64
        L.hdrf_oracle_allocator.argtypes = [ctypes.c_void_p, _u8p]
        L.hdrf_oracle_allocator.restype = ctypes.c_int
        L.hdrf_oracle_recipe.argtypes = [ctypes.c_void_p, ctypes.c_int64, _u8p, ctypes.c_int64]
        L.hdrf_oracle_recipe.restype = ctypes.c_int64
        L.hdrf_oracle_container.argtypes = [ctypes.c_void_p, ctypes.c_uint32, _u8p, ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_int)]
        L.hdrf_oracle_container.restype = ctypes.c_int64
        L.hdrf_oracle_mix64.argtypes = [ctypes.c_uint64]
        L.hdrf_oracle_mix64.restype = ctypes.c_uint64
        L.hdrf_oracle_corpus_roots.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64,
                                               ctypes.c_int64, _u32p]
        L.hdrf_oracle_corpus_fill.argtypes = [ctypes.c_uint64, _u32p, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, _u8p]
        L.hdrf_oracle_java_random_bytes.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, _u8p]
        for name in ("hdrf_oracle_lz4_bound", "hdrf_oracle_hadoop_lz4_bound"):
            getattr(L, name).argtypes = [ctypes.c_int64]
            getattr(L, name).restype = ctypes.c_int64
        for name in ("hdrf_oracle_lz4_compress", "hdrf_oracle_hadoop_lz4_frame"):
            getattr(L, name).argtypes = [_u8p, ctypes.c_int64, _u8p]
            getattr(L, name).restype = ctypes.c_int64
        L.hdrf_oracle_lz4_compress_modern.argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_int]
        L.hdrf_oracle_lz4_compress_modern.restype = ctypes.c_int64
        L.hdrf_oracle_reduce_many.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                              ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        L.hdrf_oracle_reduce_many.restype = ctypes.c_int64
        L.hdrf_oracle_reduce_many_out.argtypes = L.hdrf_oracle_reduce_many.argtypes + [ctypes.c_void_p,
                                                                                        ctypes.POINTER(ctypes.c_int64)]
        L.hdrf_oracle_reduce_many_out.restype = ctypes.c_int64
        L.hdrf_oracle_reduce_ref_shape.argtypes = L.hdrf_oracle_reduce_many.argtypes
        L.hdrf_oracle_reduce_ref_shape.restype = ctypes.c_int64
        L.hdrf_oracle_hadoop_lz4_stream_bound.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.hdrf_oracle_hadoop_lz4_stream_bound.restype = ctypes.c_int64
        L.hdrf_oracle_hadoop_lz4_stream.argtypes = [_u8p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, _u8p]
        L.hdrf_oracle_hadoop_lz4_stream.restype = ctypes.c_int64
        for name in ("hdrf_oracle_lz4_decompress", "hdrf_oracle_hadoop_lz4_unframe"):
            getattr(L, name).argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_int64]
            getattr(L, name).restype = ctypes.c_int64
        L.hdrf_oracle_snappy_bound.argtypes = [ctypes.c_int64]
        L.hdrf_oracle_snappy_bound.restype = ctypes.c_int64
        L.hdrf_oracle_snappy_compress.argtypes = [_u8p, ctypes.c_int64, _u8p]
        L.hdrf_oracle_snappy_compress.restype = ctypes.c_int64
        L.hdrf_oracle_snappy_decompress.argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_int64]
        L.hdrf_oracle_snappy_decompress.restype = ctypes.c_int64
        L.hdrf_oracle_hadoop_stream_bound.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
        L.hdrf_oracle_hadoop_stream_bound.restype = ctypes.c_int64
        L.hdrf_oracle_hadoop_stream.argtypes = [ctypes.c_int, _u8p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64,
                                                _u8p]
        L.hdrf_oracle_hadoop_stream.restype = ctypes.c_int64
        L.hdrf_oracle_hadoop_unframe.argtypes = [ctypes.c_int, _u8p, ctypes.c_int64, _u8p, ctypes.c_int64]
        L.hdrf_oracle_hadoop_unframe.restype = ctypes.c_int64
        L.hdrf_oracle_gzip_bound.argtypes = [ctypes.c_int64]
        L.hdrf_oracle_gzip_bound.restype = ctypes.c_int64
        L.hdrf_oracle_gzip_compress.argtypes = [_u8p, ctypes.c_int64, _u8p]
        L.hdrf_oracle_gzip_compress.restype = ctypes.c_int64
        L.hdrf_oracle_gzip_trace.argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_void_p]
        L.hdrf_oracle_gzip_trace.restype = ctypes.c_int64
        L.hdrf_oracle_gzip_symbols.argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p]
        L.hdrf_oracle_gzip_symbols.restype = ctypes.c_int64
        L.hdrf_oracle_lzo1x_1_compress.argtypes = [_u8p, ctypes.c_int64, _u8p]
        L.hdrf_oracle_lzo1x_1_compress.restype = ctypes.c_int64
        L.hdrf_oracle_lzo1x_decompress.argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_int64]
        L.hdrf_oracle_lzo1x_decompress.restype = ctypes.c_int64
        L.hdrf_oracle_lzop_header.argtypes = [ctypes.c_uint32, _u8p]
        L.hdrf_oracle_lzop_header.restype = ctypes.c_int64
        L.hdrf_oracle_lzop_stream_bound.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.hdrf_oracle_lzop_stream_bound.restype = ctypes.c_int64
        L.hdrf_oracle_lzop_stream.argtypes = [_u8p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.c_uint32,
                                              _u8p]
        L.hdrf_oracle_lzop_stream.restype = ctypes.c_int64
        L.hdrf_oracle_lzop_decode.argtypes = [_u8p, ctypes.c_int64, _u8p, ctypes.c_int64]
        L.hdrf_oracle_lzop_decode.restype = ctypes.c_int64
        L.hdrf_oracle_crc32.argtypes = [_u8p, ctypes.c_int64]
        L.hdrf_oracle_crc32.restype = ctypes.c_uint32
        _lib = L
    return _lib


def _p(a, t=_u8p):
    return a.ctypes.data_as(t)


def _as_u8(data):
    a = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
        else np.ascontiguousarray(data, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, dtype=np.uint8)[:0]
    return a


def chunk(data):
    """DataDeduplicator.chunking (DN/DataDeduplicator.java:264-307) -> uint32 end offsets."""
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    cap = a.size // 700 + 2
    out = np.zeros(cap, dtype=np.uint32)
    n = lib().hdrf_oracle_chunk(_p(buf), a.size, _p(out, _u32p), cap)
    assert n > 0
    return out[:n].copy()


def sha1(data):
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(20, np.uint8)
    lib().hdrf_oracle_sha1(_p(buf), a.size, _p(out))
    return out.tobytes()


def sha224(data):
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(28, np.uint8)
    lib().hdrf_oracle_sha224(_p(buf), a.size, _p(out))
    return out.tobytes()


def mix64(z):
    return lib().hdrf_oracle_mix64(z & 0xFFFFFFFFFFFFFFFF)


def corpus_roots(seed, dup_ppm, nblocks, segs_per_block):
    roots = np.zeros(nblocks * segs_per_block, np.uint32)
    lib().hdrf_oracle_corpus_roots(seed, dup_ppm, nblocks, segs_per_block, _p(roots, _u32p))
    return roots


def corpus_block(seed, roots, block, segs_per_block, seg_bytes):
    out = np.empty(segs_per_block * seg_bytes, np.uint8)
    lib().hdrf_oracle_corpus_fill(seed, _p(roots, _u32p), block, segs_per_block, seg_bytes, _p(out))
    return out


def java_random_bytes(seed, buffer_len, total):
    out = np.empty(max(total, 1), np.uint8)
    lib().hdrf_oracle_java_random_bytes(seed, buffer_len, total, _p(out))
    return out[:total]


def lz4_block(data):
    """lz4 r123 LZ4_compress (hadoop-common 3.1.0 native Lz4Compressor) -> block bytes."""
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(lib().hdrf_oracle_lz4_bound(a.size), np.uint8)
    n = lib().hdrf_oracle_lz4_compress(_p(buf), a.size, _p(out))
    return out[:n].tobytes()


def lz4_block_modern(data, rules=7):
    """The same parse under liblz4 >= 1.9's rules (hdrf_oracle.c lz4_compress_rules; tests only):
    compared byte for byte with pyarrow's bundled liblz4 to pin the shared encoder."""
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(lib().hdrf_oracle_lz4_bound(a.size), np.uint8)
    n = lib().hdrf_oracle_lz4_compress_modern(_p(buf), a.size, _p(out), rules)
    return out[:n].tobytes()


def lz4_block_decode(data, size):
    a = _as_u8(data)
    out = np.zeros(max(size, 1), np.uint8)
    n = lib().hdrf_oracle_lz4_decompress(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), size)
    return None if n < 0 else out[:n].tobytes()


def hadoop_lz4(data):
    """Lz4Codec BlockCompressorStream: write(data); close() -> file bytes (DN/DataDeduplicator.java:770-779)."""
    a = _as_u8(data)
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(lib().hdrf_oracle_hadoop_lz4_bound(a.size), np.uint8)
    n = lib().hdrf_oracle_hadoop_lz4_frame(_p(buf), a.size, _p(out))
    return out[:n].tobytes()


def hadoop_lz4_stream(data, writes):
    """Stream mode (compressor 4): Lz4Codec output stream, one write() per packet of the given
    sizes, then close() -> file bytes (DN/BlockReceiver.java:846-855,887-894,1238-1256)."""
    a = _as_u8(data)
    w = np.ascontiguousarray(writes, np.int64)
    assert int(w.sum()) == a.size
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(lib().hdrf_oracle_hadoop_lz4_stream_bound(a.size, w.size), np.uint8)
    n = lib().hdrf_oracle_hadoop_lz4_stream(_p(buf), w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), w.size,
                                            _p(out))
    return out[:n].tobytes()


def lzo1x_1(data):
    """LZO 2.10 lzo1x_1_compress (x86-64 build) -> compressed bytes."""
    a = _as_u8(data)
    buf = np.concatenate([a, np.zeros(16, np.uint8)])
    out = np.zeros(a.size + a.size // 16 + 64 + 3 + 16, np.uint8)
    n = lib().hdrf_oracle_lzo1x_1_compress(_p(buf), a.size, _p(out))
    return out[:n].copy()


def lzo1x_decode(data, size):
    a = _as_u8(data)
    out = np.zeros(max(size, 1), np.uint8)
    n = lib().hdrf_oracle_lzo1x_decompress(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), size)
    if n < 0:
        raise ValueError("malformed LZO1X stream")
    return out[:n].copy()


def lzop_stream(data, writes, mtime=0):
    """hadoop-lzo LzopCodec output stream of one block: writes (sizes) then close()."""
    a = _as_u8(data)
    w = np.ascontiguousarray(writes, np.int64)
    buf = np.concatenate([a, np.zeros(16, np.uint8)])
    out = np.zeros(lib().hdrf_oracle_lzop_stream_bound(a.size, w.size), np.uint8)
    n = lib().hdrf_oracle_lzop_stream(_p(buf), w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), w.size, mtime, _p(out))
    return out[:n].copy()


def lzop_decode(data, cap):
    a = _as_u8(data)
    out = np.zeros(max(cap, 1), np.uint8)
    n = lib().hdrf_oracle_lzop_decode(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), cap)
    if n < 0:
        raise ValueError("malformed LZOP file")
    return out[:n].copy()


def hadoop_lz4_decode(data, cap):
    a = _as_u8(data)
    out = np.zeros(max(cap, 1), np.uint8)
    n = lib().hdrf_oracle_hadoop_lz4_unframe(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), cap)
    return None if n < 0 else out[:n].tobytes()


class _OracleOut(ctypes.Structure):
    _fields_ = [("cap", ctypes.c_int64), ("offsets", ctypes.c_void_p), ("digests", ctypes.c_void_p),
                ("is_new", ctypes.c_void_p), ("values", ctypes.c_void_p)]


class Oracle:
    """Stateful restatement of DataDeduplicator + Redis + chunkDir (one DataNode)."""

    def __init__(self, hasher=0, compressor=1, max_size=1 << 25, store_only=False):
        """store_only: container lengths instead of bytes and no recipes (storeSize, dedup decisions,
        index values and the allocator unchanged): the whole-corpus dedup-ratio check."""
        self.H = 20 if hasher == 0 else 28
        self.hasher = hasher
        self._h = lib().hdrf_oracle_new(hasher, compressor, max_size)
        assert self._h
        if store_only:
            lib().hdrf_oracle_set_store_only(self._h, 1)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().hdrf_oracle_free(h)
            self._h = None

    def reduce_many(self, blocks, block_ids, nthreads):
        """Threaded CPU baseline: chunk+hash on nthreads workers ahead of the ordered index/store
        part; same state as reduce() called in order.  Returns per-block storeSize."""
        arrs = [_as_u8(b) for b in blocks]
        n = len(arrs)
        keep = [a if a.size else np.zeros(1, np.uint8) for a in arrs]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in keep])
        sizes = np.array([a.size for a in arrs], np.int64)
        ids = np.ascontiguousarray(block_ids, np.int64)
        ss = np.zeros(max(n, 1), np.int64)
        p64 = ctypes.POINTER(ctypes.c_int64)
        rc = lib().hdrf_oracle_reduce_many(self._h, ptrs, sizes.ctypes.data_as(p64), ids.ctypes.data_as(p64), n,
                                           int(nthreads), ss.ctypes.data_as(p64))
        if rc < 0:
            raise RuntimeError(f"hdrf_oracle_reduce_many: {rc}")
        return ss[:n]

    def reduce_many_full(self, blocks, block_ids, nthreads):
        """reduce_many with every block's full result (offsets, digests, is_new, values,
        store_size), as reduce() called on each block in order would return them."""
        arrs = [_as_u8(b) for b in blocks]
        n = len(arrs)
        keep = [a if a.size else np.zeros(1, np.uint8) for a in arrs]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in keep])
        sizes = np.array([a.size for a in arrs], np.int64)
        ids = np.ascontiguousarray(block_ids, np.int64)
        ss = np.zeros(max(n, 1), np.int64)
        cnt = np.zeros(max(n, 1), np.int64)
        res = []
        outs = (_OracleOut * max(n, 1))()
        for i, a in enumerate(arrs):
            cap = a.size // 700 + 2
            r = {"offsets": np.zeros(cap, np.uint32), "digests": np.zeros(cap * self.H, np.uint8),
                 "is_new": np.zeros(cap, np.uint8), "values": np.zeros(cap * 11, np.uint8)}
            outs[i].cap = cap
            outs[i].offsets = r["offsets"].ctypes.data
            outs[i].digests = r["digests"].ctypes.data
            outs[i].is_new = r["is_new"].ctypes.data
            outs[i].values = r["values"].ctypes.data
            res.append(r)
        p64 = ctypes.POINTER(ctypes.c_int64)
        rc = lib().hdrf_oracle_reduce_many_out(self._h, ptrs, sizes.ctypes.data_as(p64), ids.ctypes.data_as(p64), n,
                                               int(nthreads), ss.ctypes.data_as(p64), ctypes.cast(outs, ctypes.c_void_p),
                                               cnt.ctypes.data_as(p64))
        if rc < 0:
            raise RuntimeError(f"hdrf_oracle_reduce_many_out: {rc}")
        for i, r in enumerate(res):
            k = int(cnt[i])
            r["offsets"] = r["offsets"][:k]
            r["digests"] = r["digests"][:k * self.H].reshape(k, self.H)
            r["is_new"] = r["is_new"][:k]
            r["values"] = r["values"][:k * 11].reshape(k, 11)
            r["store_size"] = int(ss[i])
        return res

    def reduce_ref_shape(self, blocks, block_ids, nhash=3):
        """The reference's concurrency shape, blocks serialised: per block 1 chunking thread, nhash
        hasher threads over chunk ranges, then the ordered part.  Returns per-block storeSize."""
        arrs = [_as_u8(b) for b in blocks]
        n = len(arrs)
        keep = [a if a.size else np.zeros(1, np.uint8) for a in arrs]
        ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in keep])
        sizes = np.array([a.size for a in arrs], np.int64)
        ids = np.ascontiguousarray(block_ids, np.int64)
        ss = np.zeros(max(n, 1), np.int64)
        p64 = ctypes.POINTER(ctypes.c_int64)
        rc = lib().hdrf_oracle_reduce_ref_shape(self._h, ptrs, sizes.ctypes.data_as(p64), ids.ctypes.data_as(p64),
                                                n, int(nhash), ss.ctypes.data_as(p64))
        if rc < 0:
            raise RuntimeError(f"hdrf_oracle_reduce_ref_shape: {rc}")
        return ss[:n]

    def reduce(self, data, block_id):
        a = _as_u8(data)
        buf = a if a.size else np.zeros(1, np.uint8)
        cap = a.size // 700 + 2
        offs = np.zeros(cap, np.uint32)
        digs = np.zeros(cap * self.H, np.uint8)
        isnew = np.zeros(cap, np.uint8)
        vals = np.zeros(cap * 11, np.uint8)
        ss = ctypes.c_int64(0)
        n = lib().hdrf_oracle_reduce(self._h, _p(buf), a.size, block_id, cap, _p(offs, _u32p),
                                     _p(digs), _p(isnew), _p(vals), ctypes.byref(ss))
        assert n > 0, n
        return {
            "offsets": offs[:n].copy(),
            "digests": digs[:n * self.H].reshape(n, self.H).copy(),
            "is_new": isnew[:n].copy(),
            "values": vals[:n * 11].reshape(n, 11).copy(),
            "store_size": ss.value,
        }

    def index_get(self, digest):
        d = np.frombuffer(bytes(digest), np.uint8).copy()
        out = np.zeros(11, np.uint8)
        return out.tobytes() if lib().hdrf_oracle_index_get(self._h, _p(d), _p(out)) else None

    def index_dump(self):
        cnt = lib().hdrf_oracle_index_count(self._h)
        keys = np.zeros(max(cnt, 1) * self.H, np.uint8)
        vals = np.zeros(max(cnt, 1) * 11, np.uint8)
        n = lib().hdrf_oracle_index_dump(self._h, _p(keys), _p(vals), cnt)
        assert n == cnt
        return keys[:n * self.H].reshape(n, self.H), vals[:n * 11].reshape(n, 11)

    def allocator(self):
        out = np.zeros(24, np.uint8)
        return out.tobytes() if lib().hdrf_oracle_allocator(self._h, _p(out)) else None

    def recipe(self, block_id):
        n = lib().hdrf_oracle_recipe(self._h, block_id, None, 0)
        if n == 0:
            return None
        out = np.zeros(-n, np.uint8)
        m = lib().hdrf_oracle_recipe(self._h, block_id, _p(out), -n)
        return out[:m].tobytes()

    def container(self, cid):
        closed = ctypes.c_int(0)
        n = lib().hdrf_oracle_container(self._h, cid, None, 0, ctypes.byref(closed))
        if n == -1:
            return None, False
        need = -(n + 2) if n < 0 else 0
        out = np.zeros(max(need, 1), np.uint8)
        m = lib().hdrf_oracle_container(self._h, cid, _p(out), need, ctypes.byref(closed))
        return out[:m].tobytes(), bool(closed.value)


def snappy_raw(data):
    """snappy::RawCompress (google/snappy level 1) -> raw snappy bytes (oracle restatement)."""
    a = _as_u8(data)
    out = np.zeros(lib().hdrf_oracle_snappy_bound(a.size) + 8, np.uint8)
    n = lib().hdrf_oracle_snappy_compress(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out))
    return out[:n].tobytes()


def snappy_raw_decode(data, cap):
    a = _as_u8(data)
    out = np.zeros(max(cap, 1), np.uint8)
    n = lib().hdrf_oracle_snappy_decompress(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), cap)
    return None if n < 0 else out[:n].tobytes()


def hadoop_stream(codec, data, writes):
    """Stream mode through a Hadoop codec output stream (codec 0 SnappyCodec, 4 Lz4Codec): one
    write() per packet of the given sizes, then close() -> file bytes
    (DN/BlockReceiver.java:826-873,887-894,1238-1256)."""
    a = _as_u8(data)
    w = np.ascontiguousarray(writes, np.int64)
    assert int(w.sum()) == a.size
    buf = a if a.size else np.zeros(1, np.uint8)
    out = np.zeros(lib().hdrf_oracle_hadoop_stream_bound(codec, a.size, w.size), np.uint8)
    n = lib().hdrf_oracle_hadoop_stream(codec, _p(buf), w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), w.size,
                                        _p(out))
    if n < 0:
        raise ValueError("unsupported stream codec %d" % codec)
    return out[:n].tobytes()


def gzip_stream(data):
    """Stream mode compressor 5 (Hadoop GzipCodec, native zlib level 6): the block file
    (DN/BlockReceiver.java:858-873); any packet-write pattern gives the same bytes."""
    a = _as_u8(data)
    out = np.zeros(lib().hdrf_oracle_gzip_bound(a.size), np.uint8)
    n = lib().hdrf_oracle_gzip_compress(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out))
    if n < 0:
        raise MemoryError("gzip oracle state")
    return out[:n].tobytes()


def gzip_trace(data):
    """The longest_match calls of gzip_stream(data) as an int64 array of rows (strstart,
    prev_length, returned length, match_start): the checker of the GPU match pass."""
    a = _as_u8(data)
    out = np.zeros(lib().hdrf_oracle_gzip_bound(a.size), np.uint8)
    cap = max(a.size, 1)
    tr = np.zeros((cap, 4), np.int64)
    nt = ctypes.c_int64(0)
    n = lib().hdrf_oracle_gzip_trace(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), tr.ctypes.data,
                                     cap, ctypes.byref(nt))
    if n < 0:
        raise MemoryError("gzip oracle state")
    return out[:n].tobytes(), tr[:nt.value]


def gzip_symbols(data):
    """The lazy parse of gzip_stream(data): (file, symbols u32 (dist << 8) | lc, blocks int64 rows
    (symbol end, block_start, strstart, window base, last))."""
    a = _as_u8(data)
    out = np.zeros(lib().hdrf_oracle_gzip_bound(a.size), np.uint8)
    syms = np.zeros(a.size + 1, np.uint32)
    blks = np.zeros((a.size // 16383 + 2, 5), np.int64)
    ns, nb = ctypes.c_int64(0), ctypes.c_int64(0)
    n = lib().hdrf_oracle_gzip_symbols(_p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), syms.ctypes.data,
                                       ctypes.byref(ns), blks.ctypes.data, ctypes.byref(nb))
    if n < 0:
        raise MemoryError("gzip oracle state")
    return out[:n].tobytes(), syms[:ns.value], blks[:nb.value]


def hadoop_stream_decode(codec, data, cap):
    a = _as_u8(data)
    out = np.zeros(max(cap, 1), np.uint8)
    n = lib().hdrf_oracle_hadoop_unframe(codec, _p(a if a.size else np.zeros(1, np.uint8)), a.size, _p(out), cap)
    return None if n < 0 else out[:n].tobytes()
