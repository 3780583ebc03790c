"""Independent pure-Python transliteration of HDRF's write path, for small inputs.

TEST INFRASTRUCTURE ONLY.  Used to cross-check the C oracle (oracle/hdrf_oracle.c),
which is the oracle the GPU path is compared with.  Written separately from the C
code (Java-style signed bytes, dict-based Redis, hashlib digests) so that a slip in
one restatement shows up as a mismatch.  Parity against the running Java reference
is UNPINNED (no JDK/Redis here).

`DN/` = hadoop-hdfs/src/main/java/org/apache/hadoop/hdfs/server/datanode/.
"""
import hashlib


def _sbyte(v):
    return v - 256 if v >= 128 else v


def chunking(data):
    """DataDeduplicator.chunking — DN/DataDeduplicator.java:264-307."""
    size = len(data)
    w = 700
    m_value = _sbyte(data[0]) if size else 0
    m_pos = w
    offsets = []
    c_length = 0
    m_length = 1000000
    for i in range(size):
        c_length += 1
        b = _sbyte(data[i])
        if b >= m_value:
            if i > m_pos:
                offsets.append(i + 1)
                m_pos = i + w + 1
                m_value = 0
                c_length = 0
                continue
            m_value = b
        if c_length > m_length:
            offsets.append(i + 1)
            m_pos = i + w + 1
            m_value = 0
            c_length = 0
    out = offsets[:-1] if offsets else []
    out.append(size)
    return out


def chunking_closed_form(data):
    """next(p) = min(first j >= p+701 with s[j] >= M(p), p+10^6) + 1 (SURVEY.md §7 hard part 1)."""
    size = len(data)
    s = [_sbyte(x) for x in data]
    bounds = []
    p = 0
    first = True
    while True:
        e = p + 700
        if e >= size:
            break
        m = max(s[p:e + 1])
        if not first:
            m = max(m, 0)
        lim = min(p + 1000000, size - 1)
        cut = None
        for j in range(p + 701, lim + 1):
            if s[j] >= m:
                cut = j + 1
                break
        if cut is None:
            if p + 1000000 <= size - 1:
                cut = p + 1000001
            else:
                break
        bounds.append(cut)
        p = cut
        first = False
    out = bounds[:-1] if bounds else []
    out.append(size)
    return out


class PyRef:
    """DataDeduplicator (DN/DataDeduplicator.java:108-217) against a dict 'Redis'."""

    def __init__(self, hasher=0, max_size=1 << 25):
        self.hasher = hasher
        self.max_size = max_size
        self.redis = {}          # bytes key -> bytes value
        self.files = {}          # container id -> bytearray
        self.closed = set()

    def _hash(self, b):
        return hashlib.sha1(b).digest() if self.hasher == 0 else hashlib.sha224(b).digest()

    @staticmethod
    def _get_meta(m):
        """chunkMeta.getMeta — DN/chunkMeta.java:62-77."""
        st, sp = m["start"], m["stop"]
        return bytes([m["nCopy"] & 0xFF, (m["id"] >> 16) & 0xFF, (m["id"] >> 8) & 0xFF, m["id"] & 0xFF,
                      (st >> 16) & 0xFF, (st >> 8) & 0xFF, st & 0xFF,
                      (sp >> 16) & 0xFF, (sp >> 8) & 0xFF, sp & 0xFF,
                      ((st >> 20) & 0xF0) | ((sp >> 24) & 0x0F)])

    def reduce(self, data, block_id):
        data = bytes(data)
        offs = chunking(data)
        alloc = self.redis.get(b"blockID")
        last = []
        for i in range(4):
            last.append(int.from_bytes(alloc[3 * i:3 * i + 3], "big") if alloc else i << 22)
        for i in range(4):
            last.append(int.from_bytes(alloc[3 * (i + 4):3 * (i + 4) + 3], "big") if alloc else 0)
        metas = []
        prev = 0
        for end in offs:
            h = self._hash(data[prev:end])
            v = self.redis.get(h)
            m = {"h": h, "bb": prev, "len": end - prev, "id": 0, "start": 0, "stop": 0}
            if v is None:                            # chunkMeta.process — DN/chunkMeta.java:35-60
                m.update(new=True, nCopy=1)
            else:
                st = ((v[10] & 0xF0) << 20) | (v[4] << 16) | (v[5] << 8) | v[6]
                sp = ((v[10] & 0x0F) << 24) | (v[7] << 16) | (v[8] << 8) | v[9]
                m.update(new=False, nCopy=v[0] + 1, id=(v[1] << 16) | (v[2] << 8) | v[3],
                         start=st, stop=sp, len=sp - st)
            metas.append(m)
            prev = end
        store_size = sum(m["len"] for m in metas if m["new"])
        n = len(metas)
        nthread = 1 if n < 25 else 3
        sets = []
        for t in range(nthread):                     # threadedStorer.run :702-836
            lo, hi = n * t // nthread, n * (t + 1) // nthread
            if store_size == 0:
                sets += [(m["h"], self._get_meta(m)) for m in metas[lo:hi]]
                continue
            cid = last[t]
            if cid in self.files:
                cur = len(self.files[cid])
            else:
                self.files[cid] = bytearray()
                cur = 0
            buf = 0
            for m in metas[lo:hi]:
                if m["new"]:
                    if cur + m["len"] > self.max_size:
                        self.closed.add(cid)
                        buf = 0
                        cur = 0
                        last[t] += 1
                        last[t + 4] = 0
                        cid = last[t]
                        self.files.setdefault(cid, bytearray())
                    self.files[cid] += data[m["bb"]:m["bb"] + m["len"]]
                    buf += m["len"]
                    m["id"], m["start"], m["stop"] = cid, cur, cur + m["len"]
                    cur += m["len"]
                sets.append((m["h"], self._get_meta(m)))
            last[t + 4] = buf
        for k, v in sets:
            self.redis[k] = v
        self.redis[b"blockID"] = b"".join(x.to_bytes(3, "big") for x in
                                          [y & 0xFFFFFF for y in last])
        recipe = len(data).to_bytes(4, "big") + b"".join(m["h"] for m in metas)
        self.redis[(block_id & 0xFFFFFFFF).to_bytes(4, "big")] = recipe
        return {"offsets": offs, "digests": [m["h"] for m in metas],
                "is_new": [int(m["new"]) for m in metas], "store_size": store_size}
