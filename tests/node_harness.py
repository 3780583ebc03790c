"""Node-global (multi-GPU) test harness: G ranks' contexts driven phase by phase, in one
process (loopback exchange: torch copies between the ranks' record buffers) or one rank per
process (hdrf_amd.node.NodeRank over torch.distributed), and the merge of the ranks' views
into the single-node view the oracle produces for the global block sequence."""
import numpy as np
import torch

from hdrf_amd.lib import Context
from helpers import make_block


def open_ranks(G, device=0, **cfg):
    return [Context(device=device, n_ranks=G, rank=r, **cfg) for r in range(G)]


class Loopback:
    """All G ranks in this process: the X1/X2/X3 all-to-alls become region copies."""

    def __init__(self, ctxs):
        self.ctxs = ctxs
        self.G = len(ctxs)
        lay = ctxs[0].gx_layout()
        self.cap, self.w = int(lay.cap), (int(lay.x1_words), int(lay.x2_words), int(lay.x3_words))
        dev = torch.device("cuda", int(ctxs[0].cfg.device))
        n = self.G * self.cap

        def mk(w):
            return [torch.zeros(n * w, dtype=torch.int32, device=dev) for _ in range(self.G)]
        self.x1s, self.x1r = mk(self.w[0]), mk(self.w[0])
        self.x2s, self.x2r = mk(self.w[1]), mk(self.w[1])
        self.x3s, self.x3r = mk(self.w[2]), mk(self.w[2])
        self.alloc = None
        from hdrf_amd.node import ContainerPieces
        self.pieces = ContainerPieces(int(ctxs[0].cfg.n_thread))
        self.dev = dev

    def _compress(self):
        """Compressor 2 (NodeRank._compress in one process): the closers gather the head pieces,
        then every rank compresses what it closed."""
        if int(self.ctxs[0].cfg.compressor) != 2:
            return
        io = [c.gx_alloc_io() for c in self.ctxs]
        held = []                                # a write is enqueued: keep its source until gx_compress
        for q, s, cid, a, b in self.pieces.batch([x[0] for x in io], [x[1] for x in io]):
            buf = torch.empty(b - a, dtype=torch.uint8, device=self.dev)
            torch.cuda.synchronize()
            self.ctxs[q].gx_piece(cid, a, b - a, buf.data_ptr(), write=False)
            self.ctxs[s].gx_piece(cid, a, b - a, buf.data_ptr(), write=True)
            held.append(buf)
            self.moved = getattr(self, "moved", 0) + (b - a)
        for c in self.ctxs:
            c.gx_compress()
        del held

    def _a2a(self, send, recv, counts, w):
        """counts[s][d] records from rank s to rank d; returns recv counts [d][s]."""
        cap, G = self.cap, self.G
        torch.cuda.synchronize()                 # the phases only enqueue on the contexts' streams
        for s in range(G):
            for d in range(G):
                n = int(counts[s][d]) * w
                if n:
                    recv[d][s * cap * w:s * cap * w + n].copy_(send[s][d * cap * w:d * cap * w + n])
        torch.cuda.synchronize()
        return [[int(counts[s][d]) for s in range(G)] for d in range(G)]

    def batch(self, per_rank):
        """per_rank[r] = (dev_ptrs, lens, readable, block_ids) of rank r's blocks, rank-major."""
        G, ctxs = self.G, self.ctxs
        gb = np.cumsum([0] + [len(p[0]) for p in per_rank])
        c1 = [ctxs[r].gx_front(*per_rank[r], int(gb[r]), self.x1s[r].data_ptr()) for r in range(G)]
        r1 = self._a2a(self.x1s, self.x1r, c1, self.w[0])
        for d in range(G):
            ctxs[d].gx_owner(self.x1r[d].data_ptr(), r1[d], self.x2s[d].data_ptr())
        self._a2a(self.x2s, self.x2r, r1, self.w[1])
        for r in range(G):
            ctxs[r].gx_decide(self.x2r[r].data_ptr())
        a = self.alloc
        for r in range(G):
            a = ctxs[r].gx_flush(a)
        self.alloc = a
        c3 = [ctxs[r].gx_place(a, self.x3s[r].data_ptr()) for r in range(G)]
        self._compress()
        r3 = self._a2a(self.x3s, self.x3r, c3, self.w[2])
        for d in range(G):
            ctxs[d].gx_commit(self.x3r[d].data_ptr(), r3[d])


    def batches_pipelined(self, per_rank_batches, done=None, scan="device", gens=()):
        """per_rank_batches[j][r] = rank r's share of global batch j, run as NodeRank.reduce_batches
        does: the fronts of `depth` batches launched ahead (each rank's slot reused only after its
        previous batch's back phases), the oldest batch's back phases meanwhile.  scan="device":
        the packed flush descriptors all-gathered (region copies here) and composed on the device
        (hdrf_gx_flush_fn_dev / hdrf_gx_alloc_scan_dev), placement launched and waited separately;
        scan="host": the host descriptors and hdrf_gx_alloc_scan (the A/B form).  gens: the global
        batches that start a fresh DataNode (hdrf_reset_async on every rank before their fronts)."""
        G, ctxs = self.G, self.ctxs
        gens = set(gens)
        n = len(per_rank_batches)
        lay = ctxs[0].gx_layout()
        D, fnb = int(lay.depth), int(lay.fn_bytes)
        x1b = [self.x1s] + [[torch.zeros_like(t) for t in self.x1s] for _ in range(D - 1)]
        fn_send = [torch.zeros(fnb, dtype=torch.uint8, device=self.dev) for _ in range(G)]
        fn_recv = [torch.zeros(G * fnb, dtype=torch.uint8, device=self.dev) for _ in range(G)]
        launched = 0

        def launch():
            nonlocal launched
            per = per_rank_batches[launched]
            gb = np.cumsum([0] + [len(p[0]) for p in per])
            if launched in gens:
                for c in ctxs:
                    c.reset_async()
            for r in range(G):
                ctxs[r].gx_front_launch(*per[r], int(gb[r]), x1b[launched % D][r].data_ptr())
            launched += 1

        while launched < min(D, n):
            launch()
        c1 = [ctxs[r].gx_front_wait() for r in range(G)]
        for j in range(n):
            if j in gens:
                self.alloc = None
                self.pieces.reset()
            send = x1b[j % D]
            r1 = self._a2a(send, self.x1r, c1, self.w[0])
            for d in range(G):
                ctxs[d].gx_owner(self.x1r[d].data_ptr(), r1[d], self.x2s[d].data_ptr())
            self._a2a(self.x2s, self.x2r, r1, self.w[1])
            for r in range(G):
                ctxs[r].gx_decide(self.x2r[r].data_ptr())
            if scan == "device":
                for r in range(G):
                    ctxs[r].gx_flush_fn_dev(fn_send[r].data_ptr())
                torch.cuda.synchronize()                 # (the phases only enqueue on the contexts' streams)
                for d in range(G):
                    for r in range(G):
                        fn_recv[d][r * fnb:(r + 1) * fnb].copy_(fn_send[r])
                torch.cuda.synchronize()
                for r in range(G):
                    ctxs[r].gx_alloc_scan_dev(fn_recv[r].data_ptr())
                    ctxs[r].gx_flush(None, want_out=(r % 2 == 0))   # both the checked and the async form
                for r in range(G):
                    ctxs[r].gx_place_launch(None, self.x3s[r].data_ptr())
                if j + 1 < n:
                    c1n = [ctxs[r].gx_front_wait() for r in range(G)]
                c3 = [ctxs[r].gx_place_wait() for r in range(G)]
            else:
                descs = [ctxs[r].gx_flush_fn() for r in range(G)]
                fin = None
                for r in range(G):
                    a_in, a_fin = ctxs[r].gx_alloc_scan(descs)
                    assert fin is None or np.array_equal(fin, a_fin), "ranks disagree on the node allocator"
                    fin = a_fin
                    ctxs[r].gx_flush(a_in, want_out=(r % 2 == 0))
                a = self.alloc = fin
                c3 = [ctxs[r].gx_place(a, self.x3s[r].data_ptr()) for r in range(G)]
                if j + 1 < n:
                    c1n = [ctxs[r].gx_front_wait() for r in range(G)]
            self._compress()
            r3 = self._a2a(self.x3s, self.x3r, c3, self.w[2])
            for d in range(G):
                ctxs[d].gx_commit(self.x3r[d].data_ptr(), r3[d])
            if done is not None:
                done(j)
            if j + 1 < n:
                c1 = c1n
            if launched < n:
                launch()
        for c in ctxs:
            c.gx_sync()


def loopback_read(ctxs, reader, block_id):
    """The node read (hdrf_gx_read_locate / _fill on every rank, summed) in one process."""
    rec = ctxs[reader].recipe(block_id)
    size = int.from_bytes(rec[:4], "big")
    locs = [c.gx_read_locate(rec[4:])[0].astype(np.int64) for c in ctxs]
    loc = np.sum(locs, axis=0).astype(np.uint32)
    dev = torch.device("cuda", int(ctxs[0].cfg.device))
    total = torch.zeros(max(size, 1), dtype=torch.int32, device=dev)
    filled = 0
    for c in ctxs:
        part = torch.zeros(max(size, 1), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()                    # zero fill on torch's stream before the gather
        filled += c.gx_read_fill(loc, part.data_ptr(), size)
        torch.cuda.synchronize()
        total += part.to(torch.int32)
    assert filled == size, f"{filled} of {size} bytes placed"
    assert int(total.max()) <= 255
    return total[:size].to(torch.uint8).cpu().numpy()


def merged_index(ctxs):
    """Union of the ranks' index partitions, sorted by digest (the node's Redis)."""
    ks, vs = zip(*[c.index_dump() for c in ctxs])
    k = np.concatenate(ks)
    v = np.concatenate(vs)
    order = np.lexsort(k.T[::-1])
    return k[order], v[order]


def assemble_containers(pieces):
    """pieces: (cid, pos, bytes) of every new chunk on every rank -> {cid: container bytes}."""
    out = {}
    for cid, pos, data in pieces:
        buf = out.setdefault(cid, bytearray())
        end = pos + len(data)
        if len(buf) < end:
            buf.extend(b"\0" * (end - len(buf)))
        buf[pos:end] = data
    return {k: bytes(v) for k, v in out.items()}


def mixed_blocks(seed, nblk, size):
    """Blocks with cross-block duplicates (copies of earlier blocks' pieces), intra-block
    repeats and a few non-random kinds."""
    rng = np.random.default_rng(seed)
    pool = [make_block("random", seed * 100 + i, size) for i in range(4)]
    out = []
    for i in range(nblk):
        kind = i % 5
        if kind == 3:
            out.append(make_block("text", seed + i, size // 2))
            continue
        parts = []
        for _ in range(4):
            src = pool[int(rng.integers(len(pool)))] if (i and rng.random() < 0.5) else \
                make_block("random", seed * 1000 + i * 10 + len(parts), size)
            a = int(rng.integers(0, size // 2))
            parts.append(src[a:a + size // 4])
        blk = np.concatenate(parts)
        if kind == 4:
            blk = np.concatenate([blk[: size // 3], blk[: size // 3]])      # intra-block repeat
        out.append(blk)
        pool.append(blk)
    return out


def plan(nblocks_per_rank_per_batch):
    """Global sequence of (batch, rank, local index) in rank-major order."""
    seq = []
    for j, per in enumerate(nblocks_per_rank_per_batch):
        for r, n in enumerate(per):
            for i in range(n):
                seq.append((j, r, i))
    return seq
