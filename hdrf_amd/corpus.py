"""Synthetic corpus spec (BASELINE config 2) — see DESIGN.md §Corpus.

A corpus is `nblocks` blocks of `segs_per_block` segments of `seg_bytes` bytes.  Segment
(b, s) is a duplicate with probability dup_ppm/1e6 (b > 0): it then repeats a uniformly
chosen segment of an EARLIER block, so the duplicate fraction is cross-block only (an
intra-block repeat would not deduplicate in HDRF, DN/DataDeduplicator.java:338-367).
`roots[b*spb+s]` is the fresh segment whose bytes (b, s) carries; the bytes themselves are
splitmix64 words generated on the device (hdrf_corpus_fill).
"""
import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def mix64(z):
    """splitmix64 finaliser, vectorised over uint64 arrays (wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        z = np.asarray(z, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def corpus_roots(seed, dup_ppm, nblocks, segs_per_block):
    g = np.arange(nblocks * segs_per_block, dtype=np.uint64)
    coin = mix64(np.uint64(seed) ^ np.uint64(0xD1B54A32D192ED03) ^ mix64(g))
    roots = g.astype(np.uint32)
    dup = (coin % np.uint64(1000000)) < np.uint64(dup_ppm)
    r1 = mix64(coin)
    ss = mix64(r1) % np.uint64(segs_per_block)
    spb = segs_per_block
    for b in range(1, nblocks):
        lo, hi = b * spb, (b + 1) * spb
        d = dup[lo:hi]
        if not d.any():
            continue
        sb = (r1[lo:hi] % np.uint64(b)).astype(np.int64)
        src = sb * spb + ss[lo:hi].astype(np.int64)
        roots[lo:hi] = np.where(d, roots[src], roots[lo:hi])
    return roots


_WORDS = None


def _text_words():
    """The 512 eight-byte 'text' slots of the mixed-entropy corpus (7 letters + space)."""
    global _WORDS
    if _WORDS is None:
        m = mix64(np.arange(512, dtype=np.uint64) ^ np.uint64(0x7E57))
        w = np.zeros(512, np.uint64)
        for j in range(7):
            letter = (m >> np.uint64(5 * j)) % np.uint64(26) + np.uint64(ord("a"))
            w |= letter << np.uint64(8 * j)
        _WORDS = w | (np.uint64(ord(" ")) << np.uint64(56))
    return _WORDS


def segment_kind(root):
    """Mixed-entropy corpus (config 4): 0 random, 1 text, 2 binary records."""
    return int(mix64(np.uint64(int(root)) ^ np.uint64(0x5BD1E995)) % np.uint64(3))


def corpus_block_host(seed, roots, block, segs_per_block, seg_bytes, mixed=False):
    """Host copy of one block (tests / CPU baseline input); same bytes as hdrf_corpus_fill(_kind)."""
    out = np.empty(segs_per_block * seg_bytes, dtype=np.uint8)
    nw = seg_bytes // 8
    wi = np.arange(nw, dtype=np.uint64)
    for s in range(segs_per_block):
        root = int(roots[block * segs_per_block + s])
        key = mix64(np.uint64(seed) ^ mix64(np.uint64(root + 1)))
        with np.errstate(over="ignore"):
            words = mix64(key + wi)
        if mixed:
            kind = segment_kind(root)
            if kind == 1:
                words = _text_words()[(words & np.uint64(511)).astype(np.int64)]
            elif kind == 2:
                a, b = words[0::2], words[1::2]
                idx = np.arange(nw // 2, dtype=np.uint64)
                words = words.copy()
                words[0::2] = idx | ((a % np.uint64(200)) << np.uint64(32))
                words[1::2] = b % np.uint64(4)
        out[s * seg_bytes:(s + 1) * seg_bytes] = words.view(np.uint8)
    return out
