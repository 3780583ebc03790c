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

    def all_gather_dev(self, send, recv):
        """Every rank's equal-size device buffer `send` -> `recv` (G x len, rank order).  RCCL: enqueued
        on the library's back stream (no host sync); gloo: staged through host memory."""
        if self.nccl:
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    dist.all_gather_into_tensor(recv, send)
                return
            dist.all_gather_into_tensor(recv, send)
            torch.cuda.current_stream(self.device).synchronize()
            return
        if send.is_cuda:
            torch.cuda.synchronize(send.device)
        parts = [torch.empty(send.numel(), dtype=send.dtype) for _ in range(self.G)]
        dist.all_gather(parts, send.cpu())
        recv.copy_(torch.cat(parts))
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
        self.depth = int(lay.depth)
        n = self.G * self.cap
        mk = lambda w: torch.empty(n * w, dtype=torch.int32, device=self.device)  # noqa: E731
        # one X1 send buffer per batch in the pipeline: the fronts of the next batches fill theirs
        self.x1sb = [mk(self.w[0]) for _ in range(self.depth)]
        self.x1s, self.x1r = self.x1sb[0], mk(self.w[0])
        self.x2s, self.x2r = mk(self.w[1]), mk(self.w[1])
        self.x3s, self.x3r = mk(self.w[2]), mk(self.w[2])
        # the packed flush descriptors (device allocator scan): this rank's and every rank's
        self.fn_send = torch.zeros(int(lay.fn_bytes), dtype=torch.uint8, device=self.device)
        self.fn_recv = torch.zeros(self.G * int(lay.fn_bytes), dtype=torch.uint8, device=self.device)
        self.alloc = None          # node allocator after the last batch (host scan / chain; None: initial state)
        self.pieces = ContainerPieces(int(ctx.cfg.n_thread))   # compressor 2: head-piece plan
        self.phase_ms = {}         # host wall time per back phase, summed over batches
        # A/B: the rank-to-rank allocator chain (HDRF_NODE_CHAIN=1) or the host-side scan over a gloo
        # all-gather of the descriptors (HDRF_NODE_SCAN=host); default: the device scan
        self.chain = os.environ.get("HDRF_NODE_CHAIN") == "1"
        self.host_scan = os.environ.get("HDRF_NODE_SCAN") == "host"

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

    def _tick(self, key, t0):
        t = time.perf_counter()
        self.phase_ms[key] = self.phase_ms.get(key, 0.0) + 1e3 * (t - t0)
        return t

    def _back_enqueue(self, c1, r1, x1s):
        """X1 .. placement of the oldest waited batch, enqueued on the back stream (the device scan:
        no host wait; the chain and host-scan A/B forms wait where they must)."""
        ctx, xc, cap, (w1, w2, w3) = self.ctx, self.xc, self.cap, self.w
        t = time.perf_counter()
        xc.records(x1s, self.x1r, c1, r1, cap, w1)
        ctx.gx_owner(self.x1r.data_ptr(), r1, self.x2s.data_ptr())
        xc.records(self.x2s, self.x2r, r1, c1, cap, w2)           # responses retrace X1
        ctx.gx_decide(self.x2r.data_ptr())
        if self.chain:                                   # the rank-to-rank allocator chain
            self.alloc = xc.chain_alloc(self.alloc, ctx.gx_flush)
            ctx.gx_place_launch(self.alloc, self.x3s.data_ptr())
        elif self.host_scan:                             # descriptors over gloo, scanned on every host
            descs = xc.all_gather_i64(ctx.gx_flush_fn())
            a_in, self.alloc = ctx.gx_alloc_scan(descs)
            ctx.gx_flush(a_in, want_out=False)
            ctx.gx_place_launch(self.alloc, self.x3s.data_ptr())
        else:                                            # descriptors all-gathered and scanned on the device
            ctx.gx_flush_fn_dev(self.fn_send.data_ptr())
            xc.all_gather_dev(self.fn_send, self.fn_recv)
            ctx.gx_alloc_scan_dev(self.fn_recv.data_ptr())
            ctx.gx_flush(None, want_out=False)
            ctx.gx_place_launch(None, self.x3s.data_ptr())
        self._tick("enqueue x1..place", t)

    def _back_finish(self, new_gen=False):
        """Wait for the placement's read-back, then X3 and the owners' commit (not waited for)."""
        ctx, xc, cap, w3 = self.ctx, self.xc, self.cap, self.w[2]
        if new_gen:
            self.pieces.reset()
        t = time.perf_counter()
        c3 = ctx.gx_place_wait()
        t = self._tick("place wait", t)
        if int(ctx.cfg.compressor) == 2:
            self._compress()
            t = self._tick("compress", t)
        r3 = ctx.gx_x3_counts()          # implied by this owner's decisions: no count exchange
        xc.records(self.x3s, self.x3r, c3, r3, cap, w3)
        ctx.gx_commit(self.x3r.data_ptr(), r3)
        self._tick("x3+commit", t)
        self.phase_ms["batches"] = self.phase_ms.get("batches", 0) + 1

    def reduce_batch(self, dev_ptrs, lens, readable, block_ids, gbase):
        """Reduce this rank's blocks of one global batch; gbase = its first batch position."""
        torch.cuda.current_stream(self.device).synchronize()
        c1 = self.ctx.gx_front(dev_ptrs, lens, readable, block_ids, gbase, self.x1s.data_ptr())
        self._back_enqueue(c1, self.xc.counts(c1), self.x1s)
        self._back_finish()
        self.ctx.gx_sync()

    def reduce_batches(self, batches, done=None, gens=()):
        """Pipelined node-global reduction of a sequence of this rank's batches
        [(dev_ptrs, lens, readable, block_ids, gbase), ...]: the fronts (chunking, SHA, local
        aggregation) of the next `depth` - 1 batches run on the GPU while the oldest is exchanged and
        stored.  done(k) is called after batch k's placement was waited for (its hdrf_batch_* views
        are valid then).  gens: the batches that start a fresh DataNode (every rank the same):
        hdrf_reset_async before their fronts, so the node's steps run back to back, the previous
        generation's last batches completing while the next one's fronts run (bench.py's primed
        steps, as at N = 1)."""
        ctx, xc, D = self.ctx, self.xc, self.depth
        gens = set(gens)
        torch.cuda.current_stream(self.device).synchronize()
        n = len(batches)
        if not n:
            return
        launched = 0

        def launch():
            nonlocal launched
            if launched in gens:
                ctx.reset_async()
            ctx.gx_front_launch(*batches[launched], self.x1sb[launched % D].data_ptr())
            launched += 1

        while launched < min(D, n):
            launch()
        t = time.perf_counter()
        c1 = ctx.gx_front_wait()
        r1 = xc.counts(c1)
        self._tick("front wait+counts", t)
        for k in range(n):
            if k in gens:
                self.alloc = None                        # (the chain / host-scan forms' node allocator)
            self._back_enqueue(c1, r1, self.x1sb[k % D])
            if k + 1 < n:                                # host work while the back stream runs
                t = time.perf_counter()
                c1 = ctx.gx_front_wait()
                r1 = xc.counts(c1)
                self._tick("front wait+counts", t)
            self._back_finish(k in gens)
            if done is not None:
                done(k)
            if launched < n:                             # batch k's slot: the device waits for its back
                launch()
        ctx.gx_sync()

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
