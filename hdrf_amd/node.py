"""Node-global reduction over G GPUs: one fingerprint index partitioned by digest prefix.

Reference behaviour (BASELINE config 3): all DataNodes of one host share one
Redis (`JedisPool("localhost")`, DN/DataDeduplicator.java:119), one "blockID" allocator
(:165-172, :389), one chunkDir and one static FIFO (:124-158, :197-204), so the node is ONE
reduction over the global block sequence.  Here each GPU is a rank: it reduces its own shard
of every global batch and owns the index partition {digest : first digest word mod G == rank};
the three record exchanges of a batch are all-to-alls over RCCL (xGMI) — or gloo when the
ranks share a device in tests — and the container allocator is handed rank to rank.  The
result is byte-identical to one sequential run over the global order (rank-major within a
global batch), which is what tests/test_node.py checks against the oracle.

The phases themselves are C-ABI calls into libhdrf (include/hdrf.h, hdrf_gx_*); this module
only moves bytes between ranks.
"""
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from .lib import ALLOC_STATE_BYTES, HdrfError


class Exchange:
    """all-to-all of variable-length record regions laid out [G][cap][words] (int32 words)."""

    def __init__(self, G, rank, device, stream=None):
        self.G, self.rank, self.device = G, rank, device      # default process group, rank = GPU
        self.nccl = dist.get_backend() == "nccl"
        if self.nccl and (device is None or device.type != "cuda"):
            raise ValueError("the nccl (RCCL) exchange needs a GPU device")
        # RCCL: the record exchanges are enqueued on the library's back stream (hdrf_gx_stream), so
        # the phase that reads a receive buffer is ordered after the exchange on the device, with no
        # host synchronisation in between
        self.stream = stream if self.nccl else None
        # host-known metadata (X1 send counts, known once the front half was waited; flush-function
        # descriptors; allocator images) goes rank to rank over a gloo group on the CPU, so no
        # exchange makes the host wait on a device stream (an RCCL exchange of host values would
        # copy them to the GPU and back).  Collective: every rank builds its Exchange in order.
        self.meta = dist.new_group(backend="gloo") if self.nccl else None

    def counts(self, send_counts):
        """Every rank's send counts -> this rank's receive counts (int64[G]); host to host."""
        s = torch.as_tensor(np.asarray(send_counts, np.int64))
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.meta)
        return r.numpy()

    def records(self, send, recv, send_counts, recv_counts, cap, words):
        G = self.G
        if self.nccl:
            sv = [send[d * cap * words:(d * cap + int(send_counts[d])) * words] for d in range(G)]
            rv = [recv[s * cap * words:(s * cap + int(recv_counts[s])) * words] for s in range(G)]
            if self.stream is not None:
                with torch.cuda.stream(self.stream):   # ordered on the back stream: no host sync
                    dist.all_to_all(rv, sv)
                return
            dist.all_to_all(rv, sv)
            torch.cuda.current_stream(self.device).synchronize()
            return
        # (a CPU device is allowed here: the multi-process CPU tests drive this path directly)
        # gloo: stage through host memory, packed for all_to_all_single; the send buffer may still be
        # being written on the library's back stream (hdrf_gx_owner does not wait), so the device first
        if send.is_cuda:
            torch.cuda.synchronize(send.device)
        packed = torch.cat([send[d * cap * words:(d * cap + int(send_counts[d])) * words].cpu() for d in range(G)])
        out = torch.empty(int(np.sum(recv_counts)) * words, dtype=send.dtype)
        dist.all_to_all_single(out, packed, [int(c) * words for c in recv_counts],
                               [int(c) * words for c in send_counts])
        o = 0
        for s in range(G):
            n = int(recv_counts[s]) * words
            if n:
                recv[s * cap * words:s * cap * words + n].copy_(out[o:o + n])
            o += n
        if recv.is_cuda:
            torch.cuda.current_stream(recv.device).synchronize()

    def all_gather_i64(self, arr):
        """Every rank's int64 array (lengths may differ) -> list in rank order; host to host."""
        n = torch.tensor([len(arr)], dtype=torch.int64)
        ns = [torch.empty_like(n) for _ in range(self.G)]
        dist.all_gather(ns, n, group=self.meta)
        ns = [int(x[0]) for x in ns]
        t = torch.zeros(max(ns), dtype=torch.int64)
        t[:len(arr)] = torch.as_tensor(np.asarray(arr, np.int64))
        out = [torch.empty_like(t) for _ in range(self.G)]
        dist.all_gather(out, t, group=self.meta)
        return [o[:k].numpy() for o, k in zip(out, ns)]

    def chain_alloc(self, alloc_prev_batch, flush):
        """Rank r flushes after rank r-1 (rank 0 starts from the node's state); returns the node's
        allocator state after the last rank, known to every rank (host images, over the meta group)."""
        G, r = self.G, self.rank
        if r == 0:
            a_in = alloc_prev_batch
        else:
            t = torch.empty(ALLOC_STATE_BYTES, dtype=torch.uint8)
            dist.recv(t, src=r - 1, group=self.meta)
            a_in = t.numpy()
        a_out = flush(a_in)
        if r + 1 < G:
            dist.send(torch.as_tensor(a_out), dst=r + 1, group=self.meta)
        fin = torch.as_tensor(a_out).clone() if r == G - 1 else torch.empty(ALLOC_STATE_BYTES, dtype=torch.uint8)
        dist.broadcast(fin, src=G - 1, group=self.meta)
        return fin.numpy()


def alloc_fields(a):
    """AllocState (hdrf_amd/csrc/common.hpp) from its 128-B image: id, cur, pos, slot, exists per range."""
    w = np.frombuffer(np.ascontiguousarray(a, np.uint8).tobytes()[:88], np.uint32)
    return {"id": w[0:4], "cur": w[4:8], "slot": w[12:16], "exists": w[18:22]}


class ContainerPieces:
    """Which rank holds which bytes of each storer range's open node-global container
    (DN/DataDeduplicator.java:723-818 over the global block order): rank r continues the container
    rank r - 1 left open, so a container closed by rank s may hold head pieces written by earlier
    ranks (or batches).  Every rank runs the same plan from the all-gathered allocator states, so
    they agree on the transfers without further exchange."""

    def __init__(self, n_thread=3):
        self.n_thread = n_thread
        self.open = {}                       # range t -> (cid, [(rank, start, end), ...])

    def batch(self, ains, aouts):
        """ains / aouts[r]: rank r's allocator state before / after its flush walk (rank order).
        Returns the transfers (src rank, dst rank, cid, start, end) the closers need."""
        xfer = []
        for t in range(self.n_thread):
            for s, (ai, ao) in enumerate(zip(ains, aouts)):
                fi, fo = alloc_fields(ai), alloc_fields(ao)
                if (fi["id"][t], fi["cur"][t], fi["exists"][t]) == (fo["id"][t], fo["cur"][t], fo["exists"][t]):
                    continue                 # rank s placed nothing in range t
                c0 = int(fi["id"][t])
                x0 = int(fi["cur"][t]) if fi["exists"][t] else 0
                c1, x1 = int(fo["id"][t]), int(fo["cur"][t])
                cid, pieces = self.open.get(t, (c0, []))
                if cid != c0:
                    pieces = []
                if c1 == c0:
                    self.open[t] = (c0, pieces + [(s, x0, x1)])
                    continue
                for q, a, b in pieces:       # c0 closes on rank s: the heads the others hold
                    if q != s and b > a:
                        xfer.append((q, s, c0, a, b))
                self.open[t] = (c1, [(s, 0, x1)])
        return xfer

    def reset(self):
        self.open = {}


class NodeRank:
    """One GPU's share of a node-global reduction (ctx must be opened with n_ranks = G > 1)."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.G = int(ctx.cfg.n_ranks)
        self.rank = int(ctx.cfg.rank)
        if self.G < 2:
            raise ValueError("NodeRank needs a context opened with n_ranks > 1")
        self.device = torch.device("cuda", int(ctx.cfg.device))
        ext = None
        if dist.get_backend() == "nccl":
            ext = torch.cuda.ExternalStream(ctx.gx_stream(), device=self.device)
        self.xc = Exchange(self.G, self.rank, self.device, ext)
        lay = ctx.gx_layout()
        self.cap, self.w = int(lay.cap), (int(lay.x1_words), int(lay.x2_words), int(lay.x3_words))
        n = self.G * self.cap
        mk = lambda w: torch.empty(n * w, dtype=torch.int32, device=self.device)  # noqa: E731
        self.x1s, self.x1r = mk(self.w[0]), mk(self.w[0])
        self.x1s2 = mk(self.w[0])      # second X1 send buffer: the next batch's front fills it
        self.x2s, self.x2r = mk(self.w[1]), mk(self.w[1])
        self.x3s, self.x3r = mk(self.w[2]), mk(self.w[2])
        self.alloc = None          # node allocator after the last batch (None: initial state)
        self.pieces = ContainerPieces(int(ctx.cfg.n_thread))   # compressor 2: head-piece plan
        self.phase_ms = {}         # host wall time per back phase, summed over batches
        self.chain = os.environ.get("HDRF_NODE_CHAIN") == "1"   # A/B: the old rank-to-rank chain

    def reset(self):
        self.ctx.reset()
        self.alloc = None
        self.pieces.reset()

    def _compress(self):
        """Compressor 2: gather the head pieces of the containers this rank closes (the plan every
        rank derives from the all-gathered allocator states), then compress them."""
        ctx, r = self.ctx, self.rank
        ai, ao = ctx.gx_alloc_io()
        both = self.xc.all_gather_i64(np.concatenate([ai, ao]).astype(np.int64))
        ains = [b[:len(ai)].astype(np.uint8) for b in both]
        aouts = [b[len(ai):].astype(np.uint8) for b in both]
        xfer = self.pieces.batch(ains, aouts)
        ops, bufs = [], []
        dev = self.device if self.xc.nccl else torch.device("cpu")
        for q, s, cid, a, b in xfer:
            if r not in (q, s):
                continue
            buf = torch.empty(b - a, dtype=torch.uint8, device=self.device)
            if r == q:
                ctx.gx_piece(cid, a, b - a, buf.data_ptr(), write=False)
                ops.append(dist.P2POp(dist.isend, buf.to(dev), s))
            else:
                rb = torch.empty(b - a, dtype=torch.uint8, device=dev)
                ops.append(dist.P2POp(dist.irecv, rb, q))
                bufs.append((cid, a, b, rb))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        # one device synchronisation for every received piece (gloo: their H2D copies on torch's
        # stream); the writes are then enqueued on the back stream ahead of gx_compress, which keeps
        # the order and synchronises once, so the pieces stay referenced until it returned
        held = [(cid, a, b, rb.to(self.device)) for cid, a, b, rb in bufs]
        if held:
            torch.cuda.synchronize(self.device)
        try:
            for cid, a, b, t in held:
                ctx.gx_piece(cid, a, b - a, t.data_ptr(), write=True)
            n = ctx.gx_compress()        # synchronises the back stream on every return path
        finally:
            if held:                     # a raised call: the queued writes still read `held`
                ctx.synchronize()
            del held
        return n

    def reduce_batch(self, dev_ptrs, lens, readable, block_ids, gbase):
        """Reduce this rank's blocks of one global batch; gbase = its first batch position."""
        torch.cuda.current_stream(self.device).synchronize()
        c1 = self.ctx.gx_front(dev_ptrs, lens, readable, block_ids, gbase, self.x1s.data_ptr())
        self._back(c1, self.x1s)

    def _back(self, c1, x1s):
        """Exchanges and back phases of the batch whose front was waited (X1 counts c1)."""
        ctx, xc, cap, (w1, w2, w3) = self.ctx, self.xc, self.cap, self.w
        tm = self.phase_ms
        t0 = time.perf_counter()
        r1 = xc.counts(c1)
        xc.records(x1s, self.x1r, c1, r1, cap, w1)
        t1 = time.perf_counter()
        ctx.gx_owner(self.x1r.data_ptr(), r1, self.x2s.data_ptr())
        t2 = time.perf_counter()
        xc.records(self.x2s, self.x2r, r1, c1, cap, w2)           # responses retrace X1
        t3 = time.perf_counter()
        ctx.gx_decide(self.x2r.data_ptr())
        if self.chain:                                   # the rank-to-rank allocator chain
            self.alloc = xc.chain_alloc(self.alloc, ctx.gx_flush)
            ta = tb = time.perf_counter()
        else:
            # the allocator as an exclusive scan of the ranks' flush functions: one all-gather
            # instead of a rank-to-rank chain (hdrf_gx_flush_fn / hdrf_gx_alloc_scan)
            desc = ctx.gx_flush_fn()
            ta = time.perf_counter()
            descs = xc.all_gather_i64(desc)
            tb = time.perf_counter()
            a_in, self.alloc = ctx.gx_alloc_scan(descs)
            ctx.gx_flush(a_in, want_out=False)
        t4 = time.perf_counter()
        c3 = ctx.gx_place(self.alloc, self.x3s.data_ptr())
        if int(ctx.cfg.compressor) == 2:
            self._compress()
        t5 = time.perf_counter()
        r3 = ctx.gx_x3_counts()          # implied by this owner's decisions: no count exchange
        xc.records(self.x3s, self.x3r, c3, r3, cap, w3)
        t6 = time.perf_counter()
        ctx.gx_commit(self.x3r.data_ptr(), r3)
        t7 = time.perf_counter()
        for k, (a, b) in zip(("x1", "owner", "x2", "decide+flush_fn" if not self.chain else "decide+flush chain",
                              "fn all_gather", "scan+flush", "place", "x3", "commit"),
                             ((t0, t1), (t1, t2), (t2, t3), (t3, ta), (ta, tb), (tb, t4), (t4, t5), (t5, t6), (t6, t7))):
            tm[k] = tm.get(k, 0.0) + 1e3 * (b - a)
        tm["batches"] = tm.get("batches", 0) + 1

    def reduce_batches(self, batches, done=None):
        """Pipelined node-global reduction of a sequence of this rank's batches
        [(dev_ptrs, lens, readable, block_ids, gbase), ...]: the front half (chunking, SHA, local
        aggregation) of batch k+1 runs on the GPU while batch k is exchanged and stored.
        done(k) is called after batch k committed (its hdrf_batch_* views are valid then)."""
        ctx = self.ctx
        bufs = (self.x1s, self.x1s2)
        torch.cuda.current_stream(self.device).synchronize()
        if not batches:
            return
        ctx.gx_front_launch(*batches[0], bufs[0].data_ptr())
        c1 = ctx.gx_front_wait()
        for k in range(len(batches)):
            if k + 1 < len(batches):
                ctx.gx_front_launch(*batches[k + 1], bufs[(k + 1) % 2].data_ptr())
            self._back(c1, bufs[k % 2])
            if done is not None:
                done(k)
            if k + 1 < len(batches):
                c1 = ctx.gx_front_wait()

    def reconstruct_block(self, block_id, reader):
        """DataConstructor(blkID, recipe).data on the node (DN/DataConstructor.java:73-250,360-417):
        a collective of every rank; the reading rank (the one that reduced the block and keeps
        its recipe) gets the block as a numpy uint8 array, the others None.  The owners locate
        the digests (hdrf_gx_read_locate), the disjoint locations are summed, each rank gathers
        the chunks it placed (hdrf_gx_read_fill) and the disjoint partial blocks are summed on
        the reader."""
        ctx, dev = self.ctx, (self.device if self.xc.nccl else None)
        rec = np.frombuffer(ctx.recipe(block_id), np.uint8) if self.rank == reader else np.zeros(0, np.uint8)
        n = torch.tensor([rec.size], dtype=torch.int64, device=dev)
        dist.broadcast(n, src=reader)
        t = torch.zeros(int(n.item()), dtype=torch.uint8, device=dev)
        if self.rank == reader:
            t.copy_(torch.from_numpy(rec.copy()))
        dist.broadcast(t, src=reader)
        rec = t.cpu().numpy()
        size = int.from_bytes(rec[:4].tobytes(), "big")
        nd = (rec.size - 4) // ctx.H
        err = 0
        try:
            loc, _ = ctx.gx_read_locate(rec[4:].tobytes())
        except HdrfError:
            loc, err = np.zeros((nd, 4), np.uint32), 1
        # the disjoint rows summed, plus an error row: every rank fails together, none blocks
        lt = torch.as_tensor(np.vstack([loc.astype(np.int64), [[err, 0, 0, 0]]]), device=dev)
        dist.all_reduce(lt)
        lt = lt.cpu().numpy()
        if lt[-1, 0]:
            raise HdrfError(-5, f"node read of block {block_id}: a digest is missing from its owner's partition")
        loc = lt[:-1].astype(np.uint32)
        self.last_loc = loc
        part = torch.zeros(max(size, 1), dtype=torch.uint8, device=self.device)
        torch.cuda.synchronize(self.device)            # the zero fill (torch's stream) lands before the gather
        try:
            filled, err = ctx.gx_read_fill(loc, part.data_ptr(), size), 0
        except HdrfError:
            filled, err = 0, 1
        torch.cuda.synchronize(self.device)
        tot = torch.tensor([filled, err], dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        if int(tot[1].item()) or int(tot[0].item()) != size:
            raise HdrfError(-5, f"node read of block {block_id}: {int(tot[0].item())} of {size} bytes readable")
        buf = part if self.xc.nccl else part.cpu()
        dist.reduce(buf, dst=reader)
        return buf[:size].cpu().numpy() if self.rank == reader else None

    def batch_base(self, nblocks):
        """Rank-major batch positions: gbase of this rank given every rank's block count."""
        t = torch.tensor([nblocks], dtype=torch.int64, device=self.device if self.xc.nccl else None)
        allc = [torch.empty_like(t) for _ in range(self.G)]
        dist.all_gather(allc, t)
        counts = [int(x.item()) for x in allc]
        return sum(counts[:self.rank]), counts


def global_block(local, rank, G, B):
    """Global sequence number of rank's local block `local` when every global batch takes B
    blocks from each rank, rank-major (rank 0's B blocks, then rank 1's, ...)."""
    return (local // B) * G * B + rank * B + (local % B)
