// chunk.hip — exact content-defined chunking (HDRF window-max CDC) on gfx950.
//
// Reference: DataDeduplicator.chunking, DN/DataDeduplicator.java:264-307.  With s[] the
// block's signed bytes, w = 700 and maxlen = 1,000,000 the reference loop is the chain
//     next(p) = min(first j >= p+w+1 with s[j] >= M(p), p+maxlen) + 1
//     M(p)    = max(0, max s[p..p+w])       (the very first chunk has no 0 floor)
// iterated from p = 0 while the data lasts; the last detected cut is dropped and the
// block size appended (:300-304).
//
// GPU formulation:
//   1a. gmax        — one coalesced pass: the biased maximum of every 16-B granule (1 B each).
//   1b. lane walk   — each block is cut into speculative segments of seg_len bytes; one LANE
//                     walks the chain from each segment start as if a cut were there, one chunk
//                     per step from the granule maxima (window max = 42-44 maxima + two exact
//                     edge granules; search = first granule max >= M, then its first byte).
//                     Past its segment end it compares its cuts with the next lane's list (LDS):
//                     the first shared cut proves the chains equal from there on.
//   2.  repair      — boundaries whose chains did not meet within the lane's caps: the exact
//                     wave walker (walk_chain below) continues the chain until it meets ANY
//                     later segment's list (or gives up).
//   3.  stitch/copy — follow the path through synced / repaired boundaries, prefix-sum the pieces,
//                     compact them into offsets[].
//   4.  fallback    — blocks whose path ends at an unrepaired boundary (periodic data) are finished
//                     by the sequential exact walk from the last proven cut; every block then gets
//                     the reference's drop-last/append-size rule.
#include "launchers.hpp"

namespace hdrf {

// ---- byte helpers (the general path works on biased bytes, XOR 0x80, so signed order ==
// unsigned order; tiles themselves stay raw) -----------------------------------------------
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ us2 as_us2(uint32_t x) { return __builtin_bit_cast(us2, x); }

__device__ __forceinline__ uint32_t gmax16(uint4 v)
{
    // split bytes into even/odd u16 lanes and reduce with v_pk_max_u16
    us2 a = __builtin_elementwise_max(as_us2(v.x & 0x00ff00ffu), as_us2((v.x >> 8) & 0x00ff00ffu));
    us2 b = __builtin_elementwise_max(as_us2(v.y & 0x00ff00ffu), as_us2((v.y >> 8) & 0x00ff00ffu));
    us2 c = __builtin_elementwise_max(as_us2(v.z & 0x00ff00ffu), as_us2((v.z >> 8) & 0x00ff00ffu));
    us2 d = __builtin_elementwise_max(as_us2(v.w & 0x00ff00ffu), as_us2((v.w >> 8) & 0x00ff00ffu));
    us2 m = __builtin_elementwise_max(__builtin_elementwise_max(a, b), __builtin_elementwise_max(c, d));
    return max((uint32_t)m.x, (uint32_t)m.y);
}

// bit 7 of each byte set where byte >= m (m in 1..255); SWAR carry-out of byte + (256-m)
__device__ __forceinline__ uint32_t swar_ge(uint32_t w, uint32_t C)
{
    uint32_t s = (w & 0x7f7f7f7fu) + (C & 0x7f7f7f7fu);
    return ((w & C) | ((w | C) & s)) & 0x80808080u;
}

// 16-bit mask of the bytes of a RAW granule equal to 0x7F (signed 127, the largest possible
// byte): exact zero-byte test of d ^ 0x7F7F7F7F (flag = bit 7 of the byte; no carries cross bytes),
// then v_dot4_u32_u8 with byte weights 1,2,4,8 / 16..128 gathers the 16 flags.  ~18 VALU per tile.
__device__ __forceinline__ uint32_t ff_flags(uint32_t d)
{
    const uint32_t s = (~d & 0x7f7f7f7fu) + 0x7f7f7f7fu;   // bit 7 clear <=> low 7 bits all set
    return ~s & ~d & 0x80808080u;
}
__device__ __forceinline__ uint32_t ffmask16(uint4 v)
{
    const uint32_t lo = __builtin_amdgcn_udot4(ff_flags(v.y), 0x80402010u,
                                               __builtin_amdgcn_udot4(ff_flags(v.x), 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(ff_flags(v.w), 0x80402010u,
                                               __builtin_amdgcn_udot4(ff_flags(v.z), 0x08040201u, 0u, false), false);
    return (lo | (hi << 8)) >> 7;                     // 0x80 * weight: bits 7..14 and 15..22
}

// keep bytes i (0..3) with a <= i <= b, as bit-7 flags
__device__ __forceinline__ uint32_t byte_range_mask(int a, int b)
{
    uint32_t lo = a <= 0 ? 0xffffffffu : (a >= 4 ? 0u : (0xffffffffu << (8 * a)));
    uint32_t hi = b >= 3 ? 0xffffffffu : (b < 0 ? 0u : ((1u << (8 * (b + 1))) - 1u));
    return lo & hi & 0x80808080u;
}

// ---- the chain walker ---------------------------------------------------------------------
// A wave streams its region as 1 KiB tiles (lane l holds bytes [16l, 16l+16) of a tile).  The
// "view" is two biased tiles A = [T, T+1024), B = [T+1024, T+2048); two more raw tiles are in
// flight.  Tiles rotate through four register sets (R0..R3) in a 4-way unrolled loop, so there is
// exactly one advance site per phase and no register copies.  Per tile only the 0x7F-byte mask and
// its lane ballot are computed (~19 VALU); the biased granule maxima needed by the general path
// (windows without a 0x7F byte, ~6% of random-data chunks) are computed on demand.

struct WalkCfg {
    const uint8_t *base;
    int avail;     // readable bytes
    int size;      // block length
    int w;         // window (700)
    int maxlen;    // forced-cut length (1,000,000)
    const uint8_t *gm;   // the block's granule maxima (gmax_kernel), for long searches
};

enum : int { kWindow = 0, kSearchFF = 1, kSearchGen = 2 };

struct Chain {
    int p;         // last cut (chunk start)
    int state;
    int q, lim;    // pending search range
    uint32_t m;    // threshold (biased) of a general search
    bool first;    // the very first chunk of a block: M has no 0 floor
    bool ended;    // chain ended because the data ended
    bool jump;     // the search skipped ahead (granule maxima): re-seed the view at q
};

__device__ __forceinline__ uint4 tile_raw(const WalkCfg &c, int X)
{
    const int off = X + 16 * lane_id();
    if (X + 1024 <= c.avail) return ld16(c.base + off);       // wave-uniform fast path
    return load16_guard(c.base, off, c.avail);
}
__device__ __forceinline__ uint4 bias(uint4 v)
{
    v.x ^= 0x80808080u; v.y ^= 0x80808080u; v.z ^= 0x80808080u; v.w ^= 0x80808080u;
    return v;
}
// Biased copies of the view for the general (no-0x7F) path.  The empty asm pins the copies (and
// everything computed from them) inside that rarely taken path, so the compiler cannot hoist the
// granule maxima into the per-tile stream.
__device__ __forceinline__ void biased_view(const uint4 &A, const uint4 &B, uint4 &a, uint4 &b)
{
    a = A; b = B;
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z), "+v"(b.w));
    a = bias(a); b = bias(b);
}

// 4 dwords of granule g (0..127) of the view, as uniform scalars
__device__ __forceinline__ void granule(const uint4 &A, const uint4 &B, int g, uint32_t &w0, uint32_t &w1,
                                        uint32_t &w2, uint32_t &w3)
{
    const int l = g & 63;
    if (g < 64) { w0 = rdlane(A.x, l); w1 = rdlane(A.y, l); w2 = rdlane(A.z, l); w3 = rdlane(A.w, l); }
    else        { w0 = rdlane(B.x, l); w1 = rdlane(B.y, l); w2 = rdlane(B.z, l); w3 = rdlane(B.w, l); }
}

__device__ __forceinline__ uint32_t partial_max(const uint4 &A, const uint4 &B, int g, int lo, int hi)
{
    uint32_t w0, w1, w2, w3;
    granule(A, B, g, w0, w1, w2, w3);
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t wd = i < 4 ? w0 : i < 8 ? w1 : i < 12 ? w2 : w3;
        const uint32_t bv = (wd >> (8 * (i & 3))) & 0xffu;
        if (i >= lo && i <= hi) m = max(m, bv);
    }
    return m;
}

// M(p) in biased form (general path); requires T <= p < T+1024 and p+w < size.
__device__ __forceinline__ uint32_t window_max(const uint4 &rA, const uint4 &rB, int T, int p, int w, bool first)
{
    uint4 A, B;
    biased_view(rA, rB, A, B);
    const uint32_t gA = gmax16(A), gB = gmax16(B);
    const int e = p + w;
    const int gp = (p - T) >> 4, ge = (e - T) >> 4;
    const int l = lane_id();
    const uint32_t va = (l > gp && l < ge) ? gA : 0u;
    const uint32_t vb = (l + 64 > gp && l + 64 < ge) ? gB : 0u;
    uint32_t m = wave_max_u32(max(va, vb));
    const uint32_t gpm = rdlane(gp < 64 ? gA : gB, gp & 63);
    const uint32_t gem = rdlane(ge < 64 ? gA : gB, ge & 63);
    if (gpm > m) m = max(m, partial_max(A, B, gp, (p - T) & 15, 15));
    if (gem > m) m = max(m, partial_max(A, B, ge, 0, (e - T) & 15));
    if (!first) m = max(m, 0x80u);   // mValue reset to 0 after a cut (:281)
    return m;
}

// first byte index in [lo,hi] of granule g whose biased value >= m, or -1
__device__ __forceinline__ int first_ge(const uint4 &A, const uint4 &B, int g, int lo, int hi, uint32_t m)
{
    if (m == 0) return lo;
    uint32_t w0, w1, w2, w3;
    granule(A, B, g, w0, w1, w2, w3);
    const uint32_t C = (256u - m) * 0x01010101u;
    uint32_t h;
    h = swar_ge(w0, C) & byte_range_mask(lo, hi);
    if (h) return (__builtin_ctz(h) >> 3);
    h = swar_ge(w1, C) & byte_range_mask(lo - 4, hi - 4);
    if (h) return 4 + (__builtin_ctz(h) >> 3);
    h = swar_ge(w2, C) & byte_range_mask(lo - 8, hi - 8);
    if (h) return 8 + (__builtin_ctz(h) >> 3);
    h = swar_ge(w3, C) & byte_range_mask(lo - 12, hi - 12);
    if (h) return 12 + (__builtin_ctz(h) >> 3);
    return -1;
}

// first j in [q, hi] (inside the view) with biased byte >= m, or -1 (general path)
__device__ __forceinline__ int ge_in_view(const uint4 &rA, const uint4 &rB, int T, int q, int hi, uint32_t m)
{
    uint4 A, B;
    biased_view(rA, rB, A, B);
    const uint32_t gA = gmax16(A), gB = gmax16(B);
    const int gq = (q - T) >> 4, gh = (hi - T) >> 4;
    unsigned long long ma = ballot64(gA >= m);
    unsigned long long mb = ballot64(gB >= m);
    if (gq >= 64) ma = 0; else ma &= ~0ull << gq;
    if (gq > 64) mb &= ~0ull << (gq - 64);
    if (gh < 64) { mb = 0; ma &= (gh == 63) ? ~0ull : ((1ull << (gh + 1)) - 1); }
    else if (gh < 127) mb &= (1ull << (gh - 63)) - 1;
    while (ma | mb) {
        const int g = ma ? __builtin_ctzll(ma) : 64 + __builtin_ctzll(mb);
        const int lo = (g == gq) ? ((q - T) & 15) : 0;
        const int hb = (g == gh) ? ((hi - T) & 15) : 15;
        const int r = first_ge(A, B, g, lo, hb, m);
        if (r >= 0) return T + 16 * g + r;
        if (g < 64) ma &= ma - 1; else mb &= mb - 1;
    }
    return -1;
}

// First 0x7F byte at a position >= x (T <= x < T+2048) inside the view, or INT_MAX.  fA/fB are the
// per-lane 0x7F masks of the two tiles, bA/bB the per-tile ballots of lanes holding one (computed
// once per tile), so a query is one or two v_readlane plus scalar bit scans.  When the window
// holds a 0x7F byte, M(p) = 127 and the cut is simply the next 0x7F after the window.
__device__ __forceinline__ int next_ff(uint32_t fA, uint32_t fB, unsigned long long bA, unsigned long long bB, int T,
                                       int x)
{
    const int r = x - T, g = r >> 4, o = r & 15;
    if (g < 64) {
        const uint32_t w = rdlane(fA, g) & (0xffffu << o);
        if (w) return T + 16 * g + __builtin_ctz(w);
        const unsigned long long m = bA & (~1ull << g);          // lanes after g
        if (m) {
            const int L = __builtin_ctzll(m);
            return T + 16 * L + __builtin_ctz(rdlane(fA, L));
        }
        if (bB) {
            const int L = __builtin_ctzll(bB);
            return T + 1024 + 16 * L + __builtin_ctz(rdlane(fB, L));
        }
        return 0x7fffffff;
    }
    const int gb = g - 64;
    const uint32_t w = rdlane(fB, gb) & (0xffffu << o);
    if (w) return T + 16 * g + __builtin_ctz(w);
    const unsigned long long m = bB & (~1ull << gb);
    if (m) {
        const int L = __builtin_ctzll(m);
        return T + 1024 + 16 * L + __builtin_ctz(rdlane(fB, L));
    }
    return 0x7fffffff;
}

// the same for a dword of already biased bytes: maj(x7, C7, s7)
__device__ __forceinline__ uint32_t ge_flags_b(uint32_t x, uint32_t C, uint32_t Cm)
{
    const uint32_t s = (x & 0x7f7f7f7fu) + Cm;
    return __builtin_amdgcn_bitop3_b32(x, C, s, 0xe8) & 0x80808080u;   // 0xe8: maj(x, C, s)
}
// gather the bit-7 flags of four dwords into 16 bits (v_dot4_u32_u8, weights 1..128 per pair)
__device__ __forceinline__ uint32_t gather16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3)
{
    const uint32_t lo = __builtin_amdgcn_udot4(f1, 0x80402010u, __builtin_amdgcn_udot4(f0, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(f3, 0x80402010u, __builtin_amdgcn_udot4(f2, 0x08040201u, 0u, false), false);
    return (lo | (hi << 8)) >> 7;
}
// First position >= q (inside a granule whose maximum is >= m, biased) up to lim, or lim + 1: the
// wave scans the granule maxima 1,024 at a time (16 per lane, one 16-B load), so a long search
// (the forced-cut regime, text windows with high maxima) costs a load per 16 KiB instead of a pass
// over every tile.
__device__ int gm_skip(const uint8_t *gm, int q, int lim, uint32_t m)
{
    if (m == 0) return q;
    const uint32_t C = __builtin_amdgcn_perm(256u - m, 256u - m, 0u), Cm = C & 0x7f7f7f7fu;
    const int gq = q >> 4, gl = lim >> 4;
    for (int g0 = gq & ~15; g0 <= gl; g0 += 1024) {
        const int gb = g0 + 16 * lane_id();
        uint32_t h = 0;
        if (gb <= gl) {
            const uint4 v = ld16(gm + gb);
            h = gather16(ge_flags_b(v.x, C, Cm), ge_flags_b(v.y, C, Cm), ge_flags_b(v.z, C, Cm), ge_flags_b(v.w, C, Cm));
            if (gb < gq) h &= gq - gb >= 16 ? 0u : (0xffffu << (gq - gb));
            if (gl - gb < 15) h &= 0xffffu >> (15 - (gl - gb));
        }
        const unsigned long long bal = ballot64(h != 0);
        if (bal) {
            const int L = __builtin_ctzll(bal);
            const int g = g0 + 16 * L + __builtin_ctz(rdlane(h, L));
            return max(16 * g, q);
        }
    }
    return lim + 1;
}

struct ListSink;

// Advance the chain as far as the view [T, T+2048) allows.  Returns true when the view must
// advance (the chain continues), false when the chain ended (ch.ended) or the sink/stop said stop.
template <class Sink, class Stop>
__device__ __forceinline__ bool process_view(const WalkCfg &c, Chain &ch, const uint4 &A, const uint4 &B,
                                             uint32_t fA, uint32_t fB, unsigned long long bA, unsigned long long bB,
                                             int T, Sink &sink, Stop &stop)
{
    for (;;) {
        if (ch.state == kWindow) {
            // Fast path: windows holding a 0x7F byte (M = 127): cut = next 0x7F after the window + 1.
            // Scalar only, one exit test per condition; the general state machine below takes over
            // (from the same p) when a window has no 0x7F, the search leaves the view or reaches
            // lim, the data ends, or a cut crosses the stop predicate's thresholds.
            {
                int p = ch.p, cnt = sink.cnt;
                uint32_t stage = sink.stage;
                const int pe = min(T + 1024, c.size - c.w);            // window complete & inside the view
                const int hiv = min(T + 2047, c.size - 1);
                const int cut_thr = stop.cut_thr(), cnt_thr = min(stop.cnt_thr(), sink.cap);
                bool pushed = false, resume = false;
                int lim_r = 0;
                while (p < pe && cnt < cnt_thr) {
                    const int e = p + c.w;
                    if (next_ff(fA, fB, bA, bB, T, p) > e) break;      // no 0x7F in the window
                    const int f2 = next_ff(fA, fB, bA, bB, T, e + 1);
                    if (f2 > min(p + c.maxlen, hiv)) {
                        // no 0x7F in [e+1, view end]: unless lim or the data end is inside the
                        // view, the search simply continues in the next view (no generic step)
                        lim_r = min(p + c.maxlen, c.size - 1);
                        resume = lim_r > T + 2047;
                        break;
                    }
                    p = f2 + 1;                                        // :276-283
                    if (lane_id() == (cnt & 63)) stage = (uint32_t)p;
                    cnt++;
                    if ((cnt & 63) == 0) sink.store64(cnt, stage);
                    pushed = true;
                    if (p >= cut_thr) break;
                }
                sink.cnt = cnt;
                sink.stage = stage;
                if (pushed) {
                    ch.p = p;
                    ch.first = false;
                    if (stop(p, cnt)) return false;
                }
                if (resume) {
                    ch.p = p;
                    ch.lim = lim_r;
                    ch.q = T + 2048;
                    ch.state = kSearchFF;
                    return true;
                }
            }
            if (ch.p >= T + 1024) return true;
            const int e = ch.p + c.w;
            if (e >= c.size) { ch.ended = true; return false; }       // window incomplete: no more cuts
            ch.lim = min(ch.p + c.maxlen, c.size - 1);
            ch.q = e + 1;
            if (next_ff(fA, fB, bA, bB, T, ch.p) <= e) {
                ch.state = kSearchFF;                                  // M(p) = 127
            } else {
                ch.m = window_max(A, B, T, ch.p, c.w, ch.first);
                ch.state = kSearchGen;
            }
        }
        const int vend = T + 2047;
        const int hi = min(ch.lim, vend);
        int j = -1;
        if (ch.q <= hi) {
            if (ch.state == kSearchFF) {
                const int f = next_ff(fA, fB, bA, bB, T, ch.q);
                j = f <= hi ? f : -1;
            } else {
                j = ge_in_view(A, B, T, ch.q, hi, ch.m);
            }
        }
        int cut;
        if (j >= 0) {
            cut = j + 1;                                               // :276-283
        } else if (ch.lim <= vend) {
            if (ch.p + c.maxlen <= c.size - 1) cut = ch.p + c.maxlen + 1;   // forced cut :288-294
            else { ch.ended = true; return false; }
        } else {
            ch.q = max(ch.q, T + 2048);                                // continue after the advance
            if (c.gm && ch.lim > T + 4096) {
                // long search: the granule maxima say where the next candidate byte can be (without
                // them — the fused front computes none — the search goes on tile by tile)
                const int q2 = gm_skip(c.gm, ch.q, ch.lim, ch.state == kSearchFF ? 0xffu : ch.m);
                if (q2 >= T + 4096) { ch.q = min(q2, ch.lim); ch.jump = true; }
            }
            return true;
        }
        cut = __builtin_amdgcn_readfirstlane(cut);
        ch.first = false;
        ch.state = kWindow;
        ch.p = cut;
        if (!sink.push((uint32_t)cut)) return false;
        if (stop(cut, sink.cnt)) return false;
    }
}

// Cut sink that stages 64 cuts in a VGPR and writes them coalesced.
struct ListSink {
    uint32_t *out;
    int cap;
    int cnt;
    uint32_t stage;
    __device__ __forceinline__ void store64(int c, uint32_t st) { out[c - 64 + lane_id()] = st; }
    __device__ __forceinline__ bool push(uint32_t cut)
    {
        if (cnt >= cap) return false;
        if (lane_id() == (cnt & 63)) stage = cut;
        cnt++;
        if ((cnt & 63) == 0) store64(cnt, stage);
        return true;
    }
    __device__ __forceinline__ void flush()
    {
        const int r = cnt & 63;
        if (r && lane_id() < r) out[(cnt & ~63) + lane_id()] = stage;
    }
};

// Cut sink of the repair's count pass: counts, and keeps the first 64 cuts in a VGPR (lane i = cut
// i; the fast path stages through the same register), so a walk that met its shared cut within 64
// cuts hands the n_ext - 1 cuts before it to the emit pass without a second walk.
struct KeepSink {
    int cap;
    int cnt;
    uint32_t stage;
    __device__ __forceinline__ void store64(int, uint32_t) {}
    __device__ __forceinline__ bool push(uint32_t cut)
    {
        if (cnt >= cap) return false;
        if (lane_id() == (cnt & 63)) stage = cut;
        cnt++;
        return true;
    }
};

// Stop predicate of the sequential fallback walk: never stops (operator() is evaluated after every
// cut; cut_thr/cnt_thr tell the fast path the first cut position / count at which it could change).
struct NoStop {
    __device__ __forceinline__ bool operator()(int, int) { return false; }
    __device__ __forceinline__ int cut_thr() const { return 0x7fffffff; }
    __device__ __forceinline__ int cnt_thr() const { return 0x7fffffff; }
};

// Walk the chain from p (a cut, or the block start when first) calling sink.push(cut) for
// every cut until the data ends (returns true) or the sink/stop predicate says stop (false).
template <class Sink, class Stop>
__device__ __forceinline__ bool walk_chain(const WalkCfg &c, int p, bool first, Sink &sink, Stop &stop)
{
    Chain ch;
    ch.p = p; ch.state = kWindow; ch.q = 0; ch.lim = 0; ch.m = 0; ch.first = first; ch.ended = false;
    ch.jump = false;
    int T = p & ~1023;
    for (;;) {                                    // (re)seed the view at T
        uint4 R0 = tile_raw(c, T), R1 = tile_raw(c, T + 1024), R2 = tile_raw(c, T + 2048), R3 = tile_raw(c, T + 3072);
        uint32_t f0 = ffmask16(R0), f1 = ffmask16(R1), f2 = 0, f3 = 0;
        unsigned long long b0 = ballot64(f0 != 0), b1 = ballot64(f1 != 0), b2 = 0, b3 = 0;
        bool go;
        for (;;) {
            if (!(go = process_view(c, ch, R0, R1, f0, f1, b0, b1, T, sink, stop)) || ch.jump) break;
            T += 1024; f2 = ffmask16(R2); b2 = ballot64(f2 != 0); R0 = tile_raw(c, T + 3072);
            if (!(go = process_view(c, ch, R1, R2, f1, f2, b1, b2, T, sink, stop)) || ch.jump) break;
            T += 1024; f3 = ffmask16(R3); b3 = ballot64(f3 != 0); R1 = tile_raw(c, T + 3072);
            if (!(go = process_view(c, ch, R2, R3, f2, f3, b2, b3, T, sink, stop)) || ch.jump) break;
            T += 1024; f0 = ffmask16(R0); b0 = ballot64(f0 != 0); R2 = tile_raw(c, T + 3072);
            if (!(go = process_view(c, ch, R3, R0, f3, f0, b3, b0, T, sink, stop)) || ch.jump) break;
            T += 1024; f1 = ffmask16(R1); b1 = ballot64(f1 != 0); R3 = tile_raw(c, T + 3072);
        }
        if (!go) break;
        ch.jump = false;
        T = ch.q & ~1023;
    }
    return ch.ended;
}


// ------------------------------------------------------------------------------------------
// 1a. granule maxima: gm[b][g] = max of the biased bytes of granule g (bytes [16g, 16g + 16)) of
//     block b.  One coalesced streaming pass (16 B in, 1 B out per granule) — the only pass of the
//     speculative walk that reads every byte; it is HBM-bound.
constexpr int kGmPerWg = 4096;           // granules per workgroup (64 KiB of data, 16 per thread)

template <bool NT>
__global__ void __launch_bounds__(256) gmax_kernel(const BlockDesc *__restrict__ blocks, uint8_t *__restrict__ gm,
                                                   int gstride, int prio)
{
    if (prio) __builtin_amdgcn_s_setprio(2);        // HDRF_SETPRIO bit 4: ahead of SHA's VALU stream
    const BlockDesc bd = blocks[blockIdx.y];
    const int64_t ngran = (int64_t)((bd.len + 15) >> 4);
    const int64_t g0 = (int64_t)blockIdx.x * kGmPerWg;
    if (g0 >= ngran) return;
    const uint8_t *base = bd.data;
    HDRF_GLOBAL uint8_t *out = gptr_w<uint8_t>(gm + (size_t)blockIdx.y * gstride);
    const int t = threadIdx.x;
    uint4 v[16];
    if ((g0 + kGmPerWg) * 16 <= (int64_t)bd.readable) {
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = ld16_t<NT>(base + (g0 + 256 * i + t) * 16);
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int64_t g = g0 + 256 * i + t;
            v[i] = g < ngran ? load16_guard(base, g * 16, (int64_t)bd.readable) : make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int64_t g = g0 + 256 * i + t;
        if (g < ngran) out[g] = (uint8_t)gmax16(bias(v[i]));
    }
}

// gmax16 without the bias pass: the signed maximum of the 16 bytes from packed signed 16-bit maxima
// (a 16-bit signed compare orders by its high byte first, so the high byte of a v_pk_max_i16 result is
// the signed maximum of the high bytes), odd bytes from the raw words, even bytes from the words
// shifted up by 8; then the biased byte.  15 VALU per granule instead of ~27.
typedef short ss2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ ss2 as_ss2(uint32_t x) { return __builtin_bit_cast(ss2, x); }
__device__ __forceinline__ uint32_t gmax16_s(uint4 v)
{
    const ss2 o = __builtin_elementwise_max(__builtin_elementwise_max(as_ss2(v.x), as_ss2(v.y)),
                                            __builtin_elementwise_max(as_ss2(v.z), as_ss2(v.w)));
    const ss2 e = __builtin_elementwise_max(__builtin_elementwise_max(as_ss2(v.x << 8), as_ss2(v.y << 8)),
                                            __builtin_elementwise_max(as_ss2(v.z << 8), as_ss2(v.w << 8)));
    const uint32_t t = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(o, e));
    const int hi = (int)t >> 24, lo = (int)(t << 16) >> 24;       // sign-extended high bytes of both halves
    return (uint32_t)(max(hi, lo) + 128);                         // biased: signed order == unsigned order
}

// 1a'. the same pass, 15 VALU per granule, and the 16 granule bytes of a thread (256 apart) staged
// through LDS so each thread writes one 16-B word of consecutive maxima (1 store instead of 16).
// COND (the fused front): only the blocks whose cond[b] is set (a boundary of theirs went to the
// repair walk, whose long searches and the sequential fallback read the maxima)
template <bool NT, bool COND = false>
__global__ void __launch_bounds__(256) gmax2_kernel(const BlockDesc *__restrict__ blocks, uint8_t *__restrict__ gm,
                                                    int gstride, int prio, const int *__restrict__ cond = nullptr)
{
    if (COND && cond[blockIdx.y] == 0) return;
    if (prio) __builtin_amdgcn_s_setprio(2);
    __shared__ __attribute__((aligned(16))) uint8_t s_g[kGmPerWg];
    const BlockDesc bd = blocks[blockIdx.y];
    const int64_t ngran = (int64_t)((bd.len + 15) >> 4);
    const int64_t g0 = (int64_t)blockIdx.x * kGmPerWg;
    if (g0 >= ngran) return;
    const uint8_t *base = bd.data;
    uint8_t *out = gm + (size_t)blockIdx.y * gstride;
    const int t = threadIdx.x;
    uint4 v[16];
    if ((g0 + kGmPerWg) * 16 <= (int64_t)bd.readable) {
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = ld16_t<NT>(base + (g0 + 256 * i + t) * 16);
    } else {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int64_t g = g0 + 256 * i + t;
            v[i] = g < ngran ? load16_guard(base, g * 16, (int64_t)bd.readable) : make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; i++) s_g[256 * i + t] = (uint8_t)gmax16_s(v[i]);
    __syncthreads();
    const int64_t gw = g0 + 16 * t;                               // this thread's 16 consecutive granules
    if (gw + 16 <= ngran) {
        *(uint4 *)(out + gw) = *(const uint4 *)&s_g[16 * t];    // gstride and g0 + 16 t: 16-B aligned
    } else {
        for (int j = 0; j < 16 && gw + j < ngran; j++) out[gw + j] = s_g[16 * t + j];
    }
}

// 1b. lane walk (the speculative pass).  Every block is cut into segments of seg_len bytes (a
//     multiple of 702); lane l of a wave walks the chain from the start of segment k = 63*wl + l as
//     if a cut were there, one CHUNK per loop iteration, in VALU, from the granule maxima:
//       window   M(p) = max over the granule maxima of the 42-44 granules inside [p, p+700] plus
//                the exact partial maxima of the two edge granules (raw 16-B loads)
//       search   the first granule after p+700 whose maximum is >= M (SWAR carry test on the
//                maxima, v_dot4 bit gather, 64-bit bit scan), then its first byte >= M (raw load);
//                none up to min(p+maxlen, size-1): the forced cut p+maxlen
//                (DN/DataDeduplicator.java:276-294)
//     A lane's working set per chunk is 128 granule maxima (8 x 16-B loads, 2 KiB of data) and two
//     or three raw granules, so a chunk costs two dependent memory round trips and ~400 VALU instead
//     of re-reading its ~950 bytes.  Its cuts go to an LDS list (u16 offsets from the segment start;
//     written to the segment's global list when the lane stops).  Past its segment end (overrun) a
//     lane compares each cut with the next lane's list (the next segment's chain, walked
//     concurrently and seg_len bytes ahead): the first shared cut proves the chains equal from there
//     on, the lane records (i, j) and stops.  Lane 63 walks the NEXT wave's first segment (a helper:
//     LDS only), so every boundary is settled inside one wave.  A lane that meets no shared cut
//     within kLaneOver cuts or ~seg_len bytes reports kSyncFail and queues its boundary for the
//     repair pass.
constexpr int kGmWin = 16;               // dwords of granule maxima a lane holds (64 granules)

__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(as_us2(a), as_us2(b)));
}
// bytes [lo, hi) of a dword (lo, hi clamped to [0, 4])
__device__ __forceinline__ uint32_t keep_bytes(int lo, int hi)
{
    lo = min(max(lo, 0), 4);
    hi = min(max(hi, 0), 4);
    return (uint32_t)(~0ull << (8 * lo)) & (uint32_t)((1ull << (8 * hi)) - 1ull);
}
struct BMax {                             // running max of biased bytes: even / odd bytes as u16 lanes
    uint32_t e = 0, o = 0;
    __device__ __forceinline__ void add(uint32_t x)
    {
        e = pk_max(e, x & 0x00ff00ffu);
        o = pk_max(o, x & 0xff00ff00u);
    }
    __device__ __forceinline__ uint32_t get() const
    {
        const uint32_t m = pk_max(e, o >> 8);
        return max(m & 0xffffu, m >> 16);
    }
};
// biased max over bytes [lo, hi] of a raw granule
__device__ __forceinline__ uint32_t gran_max(uint4 v, int lo, int hi)
{
    BMax m;
    m.add((v.x ^ 0x80808080u) & keep_bytes(lo, hi + 1));
    m.add((v.y ^ 0x80808080u) & keep_bytes(lo - 4, hi - 3));
    m.add((v.z ^ 0x80808080u) & keep_bytes(lo - 8, hi - 7));
    m.add((v.w ^ 0x80808080u) & keep_bytes(lo - 12, hi - 11));
    return m.get();
}
// bit 7 of each byte of raw dword d whose biased value (d ^ 0x80) is >= m, with C = (256 - m) in
// every byte and Cm = C & 0x7f7f7f7f: the carry out of the byte sum = maj(NOT d7, C7, s7), s the
// low-7-bit sum (and, add, bitop3, and)
__device__ __forceinline__ uint32_t ge_flags(uint32_t d, uint32_t C, uint32_t Cm)
{
    const uint32_t s = (d & 0x7f7f7f7fu) + Cm;
    return __builtin_amdgcn_bitop3_b32(d, C, s, 0x8e) & 0x80808080u;   // 0x8e: maj(NOT d, C, s)
}
// 16-bit mask of the bytes of a raw granule whose biased value is >= m (m >= 1)
__device__ __forceinline__ uint32_t gran_ge(uint4 v, uint32_t C, uint32_t Cm)
{
    return gather16(ge_flags(v.x, C, Cm), ge_flags(v.y, C, Cm), ge_flags(v.z, C, Cm), ge_flags(v.w, C, Cm));
}
// 64-bit mask of the granule maxima d[16 h .. 16 h + 16) that are >= m
__device__ __forceinline__ unsigned long long gm_ge64(const uint32_t (&d)[kGmWin], int h, uint32_t C, uint32_t Cm)
{
    uint32_t q[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int o = 16 * h + 4 * i;
        q[i] = gather16(ge_flags_b(d[o], C, Cm), ge_flags_b(d[o + 1], C, Cm), ge_flags_b(d[o + 2], C, Cm),
                        ge_flags_b(d[o + 3], C, Cm));
    }
    return (unsigned long long)(q[0] | (q[1] << 16)) | ((unsigned long long)(q[2] | (q[3] << 16)) << 32);
}
__device__ __forceinline__ unsigned long long bits_from(int x)
{
    return x <= 0 ? ~0ull : (x >= 64 ? 0ull : (~0ull << x));
}
__device__ __forceinline__ unsigned long long bits_to(int y)     // bits 0..y
{
    return y < 0 ? 0ull : (y >= 63 ? ~0ull : ((2ull << y) - 1ull));
}
__device__ __forceinline__ uint32_t range16(int lo, int hi)      // bits lo..hi of 16
{
    const uint32_t a = lo >= 16 ? 0u : (0xffffu << max(lo, 0));
    const uint32_t b = hi < 0 ? 0u : (hi >= 15 ? 0xffffu : ((2u << hi) - 1u));
    return a & b;
}
__device__ __forceinline__ void load_gm(uint32_t (&d)[kGmWin], const uint8_t *p)
{
#pragma unroll
    for (int i = 0; i < kGmWin / 4; i++) {
        const uint4 v = ld16(p + 16 * i);
        d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
    }
}

typedef __attribute__((address_space(3))) volatile uint16_t lds_u16v;
typedef __attribute__((address_space(3))) volatile uint8_t lds_u8v;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// A lane's granule maxima, staged through LDS: a ring of two 64-granule units (128 granules = 2 KiB
// of data) in front of the lane's walk, so each granule maximum is fetched from memory once per lane
// (they used to be re-fetched by every chunk step: ~2 line fetches per chunk, the lane's window lines
// did not survive in L2 between its steps; PMC r03 1.55e7 -> 8.3e6 requests per 4 GiB batch).  The
// window of a step (64 maxima from W0 = G0 & ~3) is read from the ring at any dword offset.  The
// next unit is prefetched into registers at the end of a chunk step once the window has moved into
// the ring's second unit (after the step's raw load was waited for, so that wait never covers the
// prefetch), and written into the ring when the window reaches it.  12 KiB of LDS per wave.
#ifndef HDRF_COOP
#define HDRF_COOP 1                      // wave-cooperative list and offsets copies (0: per-lane rows, the A/B
#endif                                   // baseline; profiles/r06_coop*_ab.txt)
#ifndef HDRF_COOP_META
#define HDRF_COOP_META 0                 // (build flag, A/B) the walk's SegMeta records stored together
#endif
#ifndef HDRF_WALK_LINE
#define HDRF_WALK_LINE 1                 // (0: half-line units, the A/B baseline; profiles/r06_walkline*_ab.txt)
#endif
constexpr int kRingU = 4 * kGmWin;       // granules per ring unit (= the window)
constexpr int kRingDw = 2 * kGmWin;      // ring dwords per lane (lanes read at their own, unrelated
constexpr int kRingPitch = kRingDw;      // offsets, so rows are not padded)
struct GmRing {
    lds_u32 *r;                          // this lane's row
    int rb = -(1 << 20);                 // ring holds granules [rb, rb + 2U), rb a multiple of U
    int w0 = 0;                          // the last window start
    int pfg = -1;                        // granule of the unit held in pf (-1: none)
    uint4 pf[kGmWin / 4];
#if HDRF_WALK_LINE
    int pfg2 = -1;                       // the unit held in pf2: a line's second half (-1: none)
    uint4 pf2[kGmWin / 4];
#endif
    __device__ __forceinline__ void put(int g, const uint4 (&v)[kGmWin / 4])
    {
#pragma unroll
        for (int i = 0; i < kGmWin / 4; i++) {
            const int w = ((g >> 2) + 4 * i) & (kRingDw - 1);
            r[w] = v[i].x; r[w + 1] = v[i].y; r[w + 2] = v[i].z; r[w + 3] = v[i].w;
        }
    }
    __device__ __forceinline__ void fill(const uint8_t *gmb, int g)      // the unit of granules [g, g + U)
    {
        uint4 v[kGmWin / 4];
#pragma unroll
        for (int i = 0; i < kGmWin / 4; i++) v[i] = ld16(gmb + g + 16 * i);
        put(g, v);
    }
    // HDRF_WALK_LINE (build flag, default 1): a unit that starts a 128-B line is fetched with the line's
    // second half, which is kept in pf2 for the next unit (a unit is half a line: fetched apart, a line's
    // halves came from memory twice when the first was evicted between the lane's chunk steps; half the
    // ring's scattered 16-B load instructions).  Walk counted bytes 1.20 -> 1.11 GB per batch; config 2
    // 1098 / 1105 / 1110 vs 1058 / 1057 / 1056 and 1113 / 1118 / 1116 vs 1114 / 1104 / 1106 GB/s on two boxes
    __device__ __forceinline__ void prefetch(const uint8_t *gmb)
    {
        if (on && pfg != rb + 2 * kRingU && w0 >= rb + kRingU / 2) {
            pfg = rb + 2 * kRingU;
#if HDRF_WALK_LINE
            if (pfg2 == pfg) {
#pragma unroll
                for (int i = 0; i < kGmWin / 4; i++) pf[i] = pf2[i];
                pfg2 = -1;
                return;
            }
#endif
#pragma unroll
            for (int i = 0; i < kGmWin / 4; i++) pf[i] = ld16(gmb + pfg + 16 * i);
#if HDRF_WALK_LINE
            if ((pfg & 127) == 0) {
#pragma unroll
                for (int i = 0; i < kGmWin / 4; i++) pf2[i] = ld16(gmb + pfg + kRingU + 16 * i);
                pfg2 = pfg + kRingU;
            }
#endif
        }
    }
    bool on = true;                      // false: HDRF_WALK_RING=0, the maxima straight from memory (A/B)
    __device__ __forceinline__ void direct(uint32_t (&d)[kGmWin], const uint8_t *gmb, int W0)
    {
#pragma unroll
        for (int i = 0; i < kGmWin / 4; i++) {
            const uint4 v = ld16(gmb + W0 + 16 * i);
            d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
    }
    __device__ __forceinline__ void get(uint32_t (&d)[kGmWin], const uint8_t *gmb, int W0)
    {
        w0 = W0;
        if (!on) {
            direct(d, gmb, W0);
            return;
        }
        if (W0 < rb || W0 > rb + kRingU) {
            if (W0 <= rb + 2 * kRingU) {                          // the window moved on by one unit
                if (pfg == rb + 2 * kRingU) put(pfg, pf);
#if HDRF_WALK_LINE
                else if (pfg2 == rb + 2 * kRingU) put(pfg2, pf2);
#endif
                else fill(gmb, rb + 2 * kRingU);
                rb += kRingU;
            } else {                                              // first use, or a long search jumped
                rb = W0 & ~(kRingU - 1);
                fill(gmb, rb);
                fill(gmb, rb + kRingU);
            }
        }
        const int wd = W0 >> 2;
#pragma unroll
        for (int i = 0; i < kGmWin; i++) d[i] = r[(wd + i) & (kRingDw - 1)];
    }
};

// RING: the granule maxima through the per-lane LDS ring (32 KiB of the workgroup's 48.6 KiB).  Off
// under compressor 2: a CU holding 16 LZ4 waves has 16 KiB of LDS left, so a ring workgroup could
// only start in the pass tails (config 4 walk 47 -> 65 ms per batch with the ring, r03).
template <bool RING>
__global__ void __launch_bounds__(256) lane_walk_kernel(const BlockDesc *__restrict__ blocks, int nblocks,
                                                        int total_waves, const uint8_t *__restrict__ gm,
                                                        int gstride, int w, int maxlen,
                                                        uint32_t *__restrict__ spec, int cap,
                                                        SegMeta *__restrict__ meta, int *__restrict__ rq,
                                                        int *__restrict__ rq_count, int rq_cap,
                                                        uint32_t *__restrict__ irr, int *__restrict__ err, int ring_on, int prio)
{    if (prio) __builtin_amdgcn_s_setprio(3);        // latency-bound chain: issue before co-running waves

    __shared__ uint16_t s_cuts[4][64 * kLdsCuts];
    __shared__ uint8_t s_cnt[4][64];
    __shared__ uint32_t s_ring[4][RING ? 64 * kRingPitch : 1];
    const int wv = blockIdx.x * 4 + wave_id();
    if (wv >= total_waves) return;
    lds_u16v *vcuts = (lds_u16v *)s_cuts[wave_id()];      // read by the neighbouring lane:
    lds_u8v *vcnt = (lds_u8v *)s_cnt[wave_id()];          // volatile, never cached
    int bi = 0;
    for (int i = 1; i < nblocks; i++)
        if (blocks[i].wave0 <= wv) bi = i;
    const BlockDesc bd = blocks[bi];
    const int l = lane_id();
    const int wl = wv - bd.wave0;
    const int nseg = bd.nseg, Ls = bd.seg_len, size = (int)bd.len;
    const uint8_t *base = bd.data;                        // raw loads stay < size + 16 <= readable
    const uint8_t *gmb = gm + (size_t)bi * gstride;
    const int k = wl * kWaveSegs + l;                     // lane 63: the next wave's first segment
    const bool exists = k < nseg;
    const bool real = exists && l < kWaveSegs;
    const int s = k * Ls;
    const bool has_next = exists && k + 1 < nseg;
    const int e = (real && has_next) ? (k + 1) * Ls : 0x7fffffff;     // overrun (sync) threshold
    const int over_lim = has_next ? (k + 1) * Ls + Ls - 64 : 0x7fffffff;   // byte cap (helper too)
    const int ncap = min(cap, kLdsCuts);

    int p = s;
    bool first = s == 0;                                  // the block's first chunk: no 0 floor (:281)
    int n = 0, n_main = -1, ptr = 0, sync = kSyncEnd;
    bool active = exists, overflow = false;
    vcnt[l] = 0;
    uint32_t d[kGmWin];
    GmRing ring;
    ring.r = (lds_u32 *)&s_ring[wave_id()][RING ? l * kRingPitch : 0];
    ring.on = RING && ring_on != 0;
    uint4 rh = make_uint4(0, 0, 0, 0);                    // raw bytes of the last hit granule gh
    int gh = -1;
    for (;;) {
        if (!ballot64(active && l < kWaveSegs)) break;
        if (!active) continue;
        const int wend = p + w;
        if (wend > size - 1) { active = false; continue; }     // window incomplete: no more cuts
        const int lim = min(p + maxlen, size - 1);
        const int G0 = p >> 4, G1 = wend >> 4;
        int W0 = G0 & ~3;
        ring.get(d, gmb, W0);
        // M(p): granules G0+1 .. G1-1 are whole (bytes [a, b] of d, 1 <= a <= 4, 42 <= b <= 46); the
        // two edge granules need their raw bytes only when their maximum exceeds the rest (rare:
        // ~6 % of random-data windows), so most chunks touch no raw byte before the hit granule
        const int a = G0 + 1 - W0, b = G1 - 1 - W0;
        BMax mx;
        mx.add(d[0] & keep_bytes(a, b + 1));
#pragma unroll
        for (int i = 1; i < 10; i++) mx.add(d[i]);
        mx.add(d[10] & keep_bytes(a - 40, b - 39));
        mx.add(d[11] & keep_bytes(a - 44, b - 43));
        uint32_t M = mx.get();
        if (!first) M = max(M, 0x80u);                    // mValue reset to 0 after a cut (:281)
        const uint32_t e0 = (d[0] >> (8 * (G0 - W0))) & 0xffu;
        const int i1 = G1 - W0;
        const uint32_t e1 = (((i1 >> 2) == 10 ? d[10] : d[11]) >> (8 * (i1 & 3))) & 0xffu;
        if (e0 > M) {
            if ((p & 15) == 0) M = e0;
            else {
                const uint4 r0 = G0 == gh ? rh : ld16(base + 16 * G0);   // usually the last hit granule
                M = max(M, gran_max(r0, p & 15, 15));
            }
        }
        uint4 r1 = make_uint4(0, 0, 0, 0);
        bool have1 = false;
        if (e1 > M) {
            if ((wend & 15) == 15) M = e1;
            else {
                r1 = ld16(base + 16 * G1);
                have1 = true;
                M = max(M, gran_max(r1, 0, wend & 15));
            }
        }
        int j = -1;
        bool capped = false;
        if (M == 0) {
            j = wend + 1 <= lim ? wend + 1 : -1;          // every byte qualifies
        } else {
            const uint32_t C = __builtin_amdgcn_perm(256u - M, 256u - M, 0u), Cm = C & 0x7f7f7f7fu;
            uint32_t h1 = 0;
            if (e1 >= M && (wend & 15) != 15) {           // bytes of G1 after the window may qualify
                if (!have1) r1 = ld16(base + 16 * G1);
                h1 = gran_ge(r1, C, Cm) & range16((wend & 15) + 1, lim - 16 * G1);
            }
            if (h1) {
                j = 16 * G1 + __builtin_ctz(h1);
            } else {
                const int Glim = lim >> 4;
                int Gs = G1 + 1;
                int adv = 0;
                while (Gs <= Glim) {
                    if (Gs >= W0 + 4 * kGmWin) {
                        if (16 * Gs > over_lim) { capped = true; break; }
                        W0 = Gs & ~3;
                        // the first advance usually stays in the ring's next unit; a long search
                        // (forced-cut regime: runs of >= 1 MB under the maximum) reads each unit
                        // once, straight from memory: through the ring every unit also cost an LDS
                        // write + read round trip (config 4 walk 47 -> 71 ms per batch, r03)
                        if (adv++ == 0) ring.get(d, gmb, W0);
                        else ring.direct(d, gmb, W0);
                    }
                    const unsigned long long m0 = gm_ge64(d, 0, C, Cm) & bits_from(Gs - W0) & bits_to(Glim - W0);
                    if (m0) {
                        const int g = W0 + __builtin_ctzll(m0);
                        rh = ld16(base + 16 * g);
                        gh = g;
                        const uint32_t h = gran_ge(rh, C, Cm) & range16(0, lim - 16 * g);
                        if (h) j = 16 * g + __builtin_ctz(h);
                        break;                            // h == 0 only in the last granule (g == Glim)
                    }
                    Gs = W0 + 4 * kGmWin;
                }
            }
            if (j < 0 && !capped && p + maxlen <= size - 1) j = p + maxlen;   // forced cut (:288-294)
        }
        if (capped) { sync = kSyncFail; active = false; continue; }
        if (j < 0) { active = false; continue; }          // the data ended
        const int cut = j + 1;                            // :276-283
        const int ci = min(n, ncap - 1);                  // n < ncap always (the caps bound it)
        overflow |= n >= ncap;
        vcuts[l * kLdsCuts + ci] = (uint16_t)min(cut - s, 0xffff);
        vcnt[l] = (uint8_t)(ci + 1);
        n = ci + 1;
        if (cut >= e) {                                   // overrun: look for a shared cut
            if (n_main < 0) n_main = ci;
            const int sc = vcnt[l + 1];
            const int rel = cut - e;
            lds_u16v *sl = vcuts + (l + 1) * kLdsCuts;
            while (ptr < sc && (int)sl[ptr] < rel) ptr++;
            if (rel >= Ls) { sync = kSyncFail; active = false; }       // past the next segment's own cuts
            else if (ptr < sc && (int)sl[ptr] == rel) { sync = (ci - n_main) | (ptr << 16); active = false; }
            else if (n - n_main >= kLaneOver) { sync = kSyncFail; active = false; }
        }
        p = cut;
        first = false;
        ring.prefetch(gmb);
        if (active && p >= over_lim && p + w <= size - 1) { sync = kSyncFail; active = false; }   // byte cap
        if (overflow) active = false;
    }
    if (overflow && real) atomicOr(err, 64);
#if HDRF_COOP
    {
        // the wave's lists, written together: its 63 segments' lists are consecutive rows of `cap`
        // words (segment G at G * cap), so the lanes store the rows' words in order (coalesced) instead
        // of each lane walking its own row (63 scattered streams of ~15 stores)
        const int nreal = min(kWaveSegs, nseg - wl * kWaveSegs);
        uint32_t *rows = spec + (size_t)(bd.seg0 + wl * kWaveSegs) * cap;
        int j = l / cap, i = l - (l / cap) * cap;
        const int jstep = 64 / cap, istep = 64 - (64 / cap) * cap;
        for (int t = l; t < nreal * cap; t += 64) {
            if (i < (int)vcnt[j]) rows[t] = (uint32_t)((wl * kWaveSegs + j) * Ls) + (uint32_t)vcuts[j * kLdsCuts + i];
            j += jstep;
            i += istep;
            if (i >= cap) { i -= cap; j++; }
        }
    }
#endif
    if (real) {
        const int G = bd.seg0 + k;
#if !HDRF_COOP
        uint32_t *list = spec + (size_t)G * cap;
        for (int i = 0; i < n; i++) list[i] = (uint32_t)s + (uint32_t)vcuts[l * kLdsCuts + i];
#endif
        if (n_main < 0) n_main = n;
#if !HDRF_COOP_META
        SegMeta m;
        m.n_main = n_main; m.n_over = n - n_main; m.sync = sync; m.jmp = 0; m.jj = 0; m.n_ext = 0; m.ext_dst = -1;
        m.cp_from = 0; m.cp_n = 0; m.cp_dst = 0; m.pad[0] = m.pad[1] = m.pad[2] = 0;
        meta[G] = m;
#endif
        if (k < nseg - 1 && sync < 0) atomicOr(irr + (G >> 5), 1u << (G & 31));   // irregular boundary
        if (sync == kSyncFail) {
            const int q = atomicAdd(rq_count, 1);
            if (q < rq_cap) rq[q] = G;                        // beyond rq_cap: no repair, stitch falls back
        }
    }
#if HDRF_COOP_META
    {
        // the wave's SegMeta records (consecutive, 13 words each) through its LDS list rows, which the
        // list copy above has read: each lane stages its record, the lanes store the words in order
        static_assert(sizeof(SegMeta) == 52 && 63 * 52 <= 64 * kLdsCuts * 2, "SegMeta staging");
        const int nreal = min(kWaveSegs, nseg - wl * kWaveSegs);
        __attribute__((address_space(3))) volatile uint32_t *st32 =
            (__attribute__((address_space(3))) volatile uint32_t *)vcuts;
        if (real) {
            const int nm = n_main < 0 ? n : n_main;
            const uint32_t w[13] = {(uint32_t)nm, (uint32_t)(n - nm), (uint32_t)sync, 0u, 0u, 0u, 0xffffffffu,
                                    0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < 13; i++) st32[l * 13 + i] = w[i];
        }
        uint32_t *mrow = (uint32_t *)(meta + bd.seg0 + wl * kWaveSegs);
        for (int t = l; t < nreal * 13; t += 64) mrow[t] = st32[t];
    }
#endif
}

// 2. repair: one wave per failed boundary k (queued by the lane walk), the exact sequential walker
//    continues segment k's chain from its last cut.  find: every new cut c is looked up in the list
//    of the segment m = c / seg_len holding it (m > k); once found at index j, segment k's chain
//    continues as segment m's from there (kSyncJump, k + jmp = m, jj = j, n_ext cuts walked); no
//    shared cut within kRepairCuts cuts / kRepairBytes bytes, or the block end: kSyncGiveUp.
//    emit (after the stitch placed it): the n_ext - 1 cuts before the shared one go into the block's
//    offsets, for repairs on the block's path — copied from what the find pass kept when there were
//    at most 63 of them (queue entries below kRqKeep), else by the same walk again.
struct MergeStop {
    const uint32_t *spec;
    const SegMeta *meta;
    int cap, seg0, k, nseg, Ls, lim_cut;
    int m_cached = -1;
    uint32_t lane_val = 0xffffffffu;
    int status = 0, res_m = 0, res_j = 0;             // status 1 merged, 2 gave up
    __device__ __forceinline__ bool operator()(int cut, int)
    {
        if (cut > lim_cut) { status = 2; return true; }
        const int m = cut / Ls;
        if (m <= k || m >= nseg) return false;
        if (m != m_cached) {
            m_cached = m;
            const int nm = min(meta[seg0 + m].n_main, 64);
            lane_val = lane_id() < nm ? spec[(size_t)(seg0 + m) * cap + lane_id()] : 0xffffffffu;
        }
        const unsigned long long hit = ballot64(lane_val == (uint32_t)cut);
        if (hit) { status = 1; res_m = m; res_j = __builtin_ctzll(hit); return true; }
        return false;
    }
    __device__ __forceinline__ int cut_thr() const { return 0; }      // every cut is looked up
    __device__ __forceinline__ int cnt_thr() const { return 0x7fffffff; }
};

__global__ void __launch_bounds__(64) lane_repair_kernel(const BlockDesc *__restrict__ blocks, int nblocks,
                                                          const int *__restrict__ rq, const int *__restrict__ rq_count,
                                                          int rq_cap, int w, int maxlen,
                                                          const uint32_t *__restrict__ spec, int cap,
                                                          SegMeta *__restrict__ meta, uint32_t *__restrict__ offsets,
                                                          int cap_blk, const uint8_t *__restrict__ gm, int gstride,
                                                          int emit, int prio, uint32_t *__restrict__ keep)
{    if (prio) __builtin_amdgcn_s_setprio(3);        // latency-bound chain: issue before co-running waves

    const int nw = gridDim.x;
    const int cnt = min(*rq_count, rq_cap);
    for (int q = blockIdx.x; q < cnt; q += nw) {
        const int G = __builtin_amdgcn_readfirstlane(rq[q]);
        int bi = 0;
        for (int i = 1; i < nblocks; i++)
            if (blocks[i].seg0 <= G) bi = i;
        const BlockDesc bd = blocks[bi];
        const int k = G - bd.seg0;
        const SegMeta m = meta[G];
        if (emit && (m.sync != kSyncJump || m.ext_dst < 0 || m.n_ext <= 1)) continue;
        if (emit && q < kRqKeep && m.n_ext <= 64) {      // kept by the count pass (same q, same walk)
            if (lane_id() < m.n_ext - 1)
                offsets[(size_t)bi * cap_blk + m.ext_dst + lane_id()] = keep[(size_t)q * 64 + lane_id()];
            continue;
        }
        const int n = m.n_main + m.n_over;
        const int s_k = k * bd.seg_len;
        const int p0 = n > 0 ? (int)spec[(size_t)G * cap + n - 1] : s_k;
        const bool first = n == 0 && s_k == 0;
        WalkCfg W;
        W.base = bd.data; W.avail = (int)min(bd.readable, (uint64_t)0x7fffffff); W.size = (int)bd.len;
        W.w = w; W.maxlen = maxlen; W.gm = gm ? gm + (size_t)bi * gstride : nullptr;
        if (!emit) {
            KeepSink sink;
            sink.cap = kRepairCuts; sink.cnt = 0; sink.stage = 0;
            MergeStop st;
            st.spec = spec; st.meta = meta; st.cap = cap; st.seg0 = bd.seg0; st.k = k; st.nseg = bd.nseg;
            st.Ls = bd.seg_len; st.lim_cut = p0 + kRepairBytes;
            (void)walk_chain(W, p0, first, sink, st);
            if (st.status == 1 && q < kRqKeep && sink.cnt <= 64 && lane_id() < sink.cnt - 1)
                keep[(size_t)q * 64 + lane_id()] = sink.stage;
            if (lane_id() == 0) {
                if (st.status == 1) {
                    meta[G].jmp = st.res_m - k;
                    meta[G].jj = st.res_j;
                    meta[G].n_ext = sink.cnt;
                    meta[G].sync = kSyncJump;
                } else {
                    meta[G].sync = kSyncGiveUp;
#ifdef HDRF_DEBUG_CHUNK
                    printf("repair give-up: block %d seg %d p0 %d cuts %d status %d lim %d\n", bi, k, p0, sink.cnt,
                           st.status, st.lim_cut);
#endif
                }
            }
        } else {
            ListSink sink;
            sink.out = offsets + (size_t)bi * cap_blk + m.ext_dst; sink.cap = m.n_ext - 1; sink.cnt = 0; sink.stage = 0;
            NoStop ns;
            (void)walk_chain(W, p0, first, sink, ns);
            sink.flush();
        }
    }
}

// 3. stitch.  The block's chain is segment 0's list, then, boundary by boundary, the next
//    segment's list from the shared cut: synced boundaries go to k + 1 (seg k keeps its overrun
//    cuts [0, i)), repaired ones jump to k + jmp (seg k keeps all its cuts and the repair's n_ext - 1
//    cuts; the segments jumped over are off the path); the path ends at the last segment, at a chain
//    that ran to the block end, or at a failed boundary (seg k keeps all its cuts and the sequential
//    fallback continues from the last one).  Four wide kernels:
//      path   one wave per block: the irregular boundaries (not "synced to k + 1"; a bitmask the
//             lane walk wrote) are compacted in order with their status, thread 0 follows the path
//             through them (LDS only) and writes the on-path jumps, the terminal and the fallback flag
//      count  one thread per segment: its piece (first list index, cuts, repair cuts) + workgroup sums
//      scan   one wave per block: prefix over the workgroup sums; n_cuts / fail_dst
//      copy   one thread per segment: workgroup prefix -> destination; the piece is copied
// The irregular boundaries are compacted kStitchNodes at a time (a window of the ordered node list
// in LDS); thread 0 follows the path through a window and the next window is loaded when the path
// leaves it, so any number of irregular boundaries is followed (round 2 capped them at 2048 per block
// and handed the rest of the block to the sequential fallback: config-4 blocks of binary records
// reach that many, and their last 1-18 MiB were walked by one wave, 34 ms per batch, r03).  The
// on-path jumps go to jx / jt (jcap per block: every segment boundary at most once).  8.5 KiB of LDS
// (path) and 2 KiB (count) let both start beside a compressor-2 LZ4 pass (16 KiB free per CU).
constexpr int kStitchNodes = 1024;

__global__ void __launch_bounds__(64) stitch_path_kernel(const BlockDesc *__restrict__ blocks,
                                                          const uint32_t *__restrict__ irr,
                                                          const SegMeta *__restrict__ meta,
                                                          PathInfo *__restrict__ path, int *__restrict__ jx_all,
                                                          uint32_t *__restrict__ jt_all, int jcap, int prio)
{
    if (prio) __builtin_amdgcn_s_setprio(3);        // latency-bound chain: issue before co-running waves
    __shared__ int s_nx[kStitchNodes];       // compacted irregular nodes of the window (ascending)
    __shared__ uint32_t s_nv[kStitchNodes];  // status: bit 31 jump (jmp in bits 0..23, jj in 24..29), bit 30 end
    __shared__ int s_go;
    const int b = blockIdx.x, t = threadIdx.x;
    const BlockDesc bd = blocks[b];
    const int nseg = bd.nseg, s0 = bd.seg0;
    const SegMeta *mt = meta + s0;
    const int nb = nseg - 1;                 // boundaries 0 .. nseg - 2
    const int nwords = (nb + 31) >> 5;
    auto word = [&](int i) -> uint32_t {     // boundaries 32 i .. 32 i + 31 of this block
        const int gbit = s0 + 32 * i, wi = gbit >> 5, sh = gbit & 31;
        uint32_t v = irr[wi] >> sh;
        if (sh) v |= irr[wi + 1] << (32 - sh);
        const int rem = nb - 32 * i;
        return rem >= 32 ? v : (v & ((1u << rem) - 1u));
    };
    const int per = (nwords + 63) >> 6;       // one wave per block: a run of words per lane
    const int w0 = min(nwords, t * per), w1 = min(nwords, w0 + per);
    uint32_t cnt = 0;
    for (int i = w0; i < w1; i++) cnt += (uint32_t)__popc(word(i));
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t pos0 = incl - cnt;        // this lane's first node in the ordered list
    const int tot = (int)rdlane(incl, 63);
    int *jx = jx_all + (size_t)b * jcap;
    uint32_t *jt = jt_all + (size_t)b * jcap;
    int cur = 0, nj = 0, term = nseg - 1, fb = 0;        // thread 0's path state
    for (int wb = 0;; wb += kStitchNodes) {
        // window [wb, wb + kStitchNodes) of the node list
        if (pos0 < (uint32_t)(wb + kStitchNodes) && pos0 + cnt > (uint32_t)wb) {
            uint32_t pos = pos0;
            for (int i = w0; i < w1 && pos < (uint32_t)(wb + kStitchNodes); i++)
                for (uint32_t v = word(i); v; v &= v - 1) {
                    if (pos >= (uint32_t)wb && pos < (uint32_t)(wb + kStitchNodes)) {
                        const int k = 32 * i + __builtin_ctz(v);
                        const int sy = mt[k].sync;
                        s_nx[pos - wb] = k;
                        s_nv[pos - wb] = sy == kSyncJump ? (0x80000000u | ((uint32_t)mt[k].jj << 24) | (uint32_t)mt[k].jmp)
                                                         : (sy == kSyncEnd ? 0x40000000u : 0u);
                    }
                    pos++;
                }
        }
        __syncthreads();
        if (t == 0) {
            const int nnx = min(tot - wb, kStitchNodes);
            int i = 0, go = 0;
            for (;;) {
                while (i < nnx && s_nx[i] < cur) i++;
                if (i >= nnx) {
                    go = wb + kStitchNodes < tot;          // nodes ahead: the next window
                    break;
                }
                const int x = s_nx[i];
                const uint32_t v = s_nv[i];
                if (v & 0x80000000u) {
                    if (nj >= jcap) { term = x; fb = 1; break; }    // (cannot happen: one jump per boundary)
                    const int tgt = x + (int)(v & 0xffffffu);
                    jx[nj] = x; jt[nj] = (uint32_t)tgt | (v & 0x3f000000u); nj++;
                    cur = tgt;
                    continue;
                }
                term = x;
                fb = (v & 0x40000000u) == 0;
                break;
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go) break;
    }
    if (t == 0) {
        PathInfo pi;
        pi.nj = nj; pi.term = term; pi.fb = fb; pi.pad = 0;
        path[b] = pi;
    }
}

// block-wide (256 threads) sum / exclusive prefix through 4 wave partials
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t *s_w, uint32_t &total)
{
    const uint32_t incl = wave_incl_scan(v);
    if (lane_id() == 63) s_w[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < (int)(threadIdx.x >> 6); i++) base += s_w[i];
    total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    return base + incl - v;
}

__global__ void __launch_bounds__(256) stitch_count_kernel(const BlockDesc *__restrict__ blocks,
                                                           SegMeta *__restrict__ meta,
                                                           const PathInfo *__restrict__ path,
                                                           const int *__restrict__ jx_all,
                                                           const uint32_t *__restrict__ jt_all, int jcap,
                                                           uint32_t *__restrict__ wgsum, int maxw,
                                                           int *__restrict__ err)
{
    // the jumps that matter to this workgroup's 256 segments: the last one with source < k0 and those
    // with source in [k0, k0 + 256) (sources ascend along the path, one per boundary at most)
    __shared__ int s_jx[257];
    __shared__ uint32_t s_jt[257];
    __shared__ int s_j0, s_nr;
    __shared__ uint32_t s_w[4];
    const int b = blockIdx.y, t = threadIdx.x;
    const BlockDesc bd = blocks[b];
    const int nseg = bd.nseg;
    if ((int)blockIdx.x * 256 >= nseg) return;            // whole workgroup
    const int k0 = blockIdx.x * 256;
    const int k = k0 + t;
    const PathInfo pi = path[b];
    const int term = pi.term;
    const int *jxb = jx_all + (size_t)b * jcap;
    const uint32_t *jtb = jt_all + (size_t)b * jcap;
    if (t == 0) {
        int lo = 0, hi = pi.nj;                            // first jump with source >= k0
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (jxb[mid] < k0) lo = mid + 1; else hi = mid; }
        int e = lo, ehi = pi.nj;                           // first jump with source >= k0 + 256
        while (e < ehi) { const int mid = (e + ehi) >> 1; if (jxb[mid] < k0 + 256) e = mid + 1; else ehi = mid; }
        s_j0 = lo - 1;
        s_nr = e - (lo - 1);
    }
    __syncthreads();
    const int j0 = s_j0, nr = s_nr;
    for (int i = t; i < nr; i += 256)
        if (j0 + i >= 0) { s_jx[i] = jxb[j0 + i]; s_jt[i] = jtb[j0 + i]; }
    __syncthreads();
    const int nj = nr;                                     // local indices: jump j0 + i at i
    SegMeta *mt = meta + bd.seg0;
    int from = 0, cnt = 0, ext = -1;
    bool entered_by_jump = false;
    if (k < nseg && k <= term) {
        const int i0 = j0 < 0 ? 1 : 0;                     // local entry 0 is jump j0 (none when j0 < 0)
        int lo = i0, hi = nj;                              // last jump with source < k
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (s_jx[mid] < k) lo = mid + 1; else hi = mid; }
        const int ji = lo - 1 >= i0 ? lo - 1 : -1;
        bool target = false, over = false;
        if (ji >= 0) {
            const int tgt = (int)(s_jt[ji] & 0xffffffu);
            over = tgt > k;                                // jumped over
            target = tgt == k;
        }
        entered_by_jump = target;
        if (!over) {
            const SegMeta m = mt[k];
            if (k == 0) from = 0;
            else if (target) from = (int)(s_jt[ji] >> 24);
            else from = (mt[k - 1].sync >> 16) & 0xffff;
            if (from > m.n_main) { atomicOr(err, 128); from = m.n_main; }   // never: a shared cut is a main cut
            cnt = m.n_main - from;
            if (k == term) cnt += m.n_over;
            else if (m.sync == kSyncJump) { cnt += m.n_over; ext = cnt; cnt += m.n_ext - 1; }
            else cnt += m.sync & 0xffff;
        }
    }
    if (k < nseg) {
        mt[k].cp_from = from;
        mt[k].cp_n = ext >= 0 ? ext : cnt;                 // list cuts; the repair's cuts follow (emit)
        mt[k].pad[0] = cnt;
        mt[k].pad[1] = ext;
        mt[k].pad[2] = k == 0 ? 0 : (entered_by_jump ? 2 : 1);   // how the path entered (fused digests)
    }
    uint32_t total;
    (void)wg_excl_scan((uint32_t)cnt, s_w, total);
    if (t == 0) wgsum[(size_t)b * maxw + blockIdx.x] = total;
}

__global__ void __launch_bounds__(64) stitch_scan_kernel(const BlockDesc *__restrict__ blocks,
                                                         const PathInfo *__restrict__ path,
                                                         uint32_t *__restrict__ wgsum, int maxw,
                                                         BlockState *__restrict__ bst, int cap_blk,
                                                         int *__restrict__ err)
{
    const int b = blockIdx.x, t = threadIdx.x;          // one wave per block
    const int nw = (blocks[b].nseg + 255) >> 8;
    uint32_t run = 0;
    for (int i0 = 0; i0 < nw; i0 += 64) {
        const int i = i0 + t;
        const uint32_t v = i < nw ? wgsum[(size_t)b * maxw + i] : 0u;
        const uint32_t incl = wave_incl_scan(v);
        if (i < nw) wgsum[(size_t)b * maxw + i] = run + incl - v;
        run += rdlane(incl, 63);
    }
    if (t == 0) {
        BlockState s;
        s.n_cuts = (int)run;
        s.fail_dst = path[b].fb ? (int)run : -1;
        s.fail_p0 = 0; s.n_chunks = 0;
        if (run > (uint32_t)cap_blk) { atomicOr(err, 1); s.n_cuts = 0; s.fail_dst = -1; }
        bst[b] = s;
    }
}

// With the fused pass (lanehash.hip, sdig != nullptr) the digests of the copied list cuts move to the
// batch's digest rows too and their need[] flags are cleared: list cut from + i of segment k ends a
// chunk of lane k's chain that starts on the path for i > 0, and for i == 0 at the block start (k == 0);
// the first cut after a sync is the chunk lane k - 1 cut up to the shared cut (bdig[k]), on the path
// when segment k - 1 contributed a cut of its own (or is segment 0).  A jump target's first cut, the
// repair's cuts and the fallback's are hashed by the fix-up pass (sha.hip).
// the wave's 64 segments four at a time, a 16-lane group per segment, one digest row per lane: the
// loads of up to 48 rows per segment are issued before any store (one memory round trip per four
// segments; one segment per step with a word per lane left the stitch 0.55 ms slower per batch)
template <int HW>
__device__ __forceinline__ void copy_digests_wave(int n_l, int G, int from, int dst, bool head, int k, int cap,
                                                  const uint32_t *__restrict__ sdig, const uint32_t *__restrict__ bdig,
                                                  uint32_t *__restrict__ dig, uint8_t *__restrict__ need)
{
    const int l = lane_id(), r = l & 15;
    for (int j0 = 0; j0 < 64; j0 += 4) {
        const int j = j0 + (l >> 4);
        const int nj = __shfl(n_l, j, 64);
        if (!ballot64(nj > 0)) continue;
        const int Gj = __shfl(G, j, 64), fj = __shfl(from, j, 64), dj = __shfl(dst, j, 64), kj = __shfl(k, j, 64);
        const bool hj = __shfl((int)head, j, 64) != 0;
        uint32_t v[3][HW];
        bool ok[3];
#pragma unroll
        for (int u = 0; u < 3; u++) {
            const int i = r + 16 * u;
            ok[u] = i < nj && (i > 0 || kj == 0 || hj);
            const uint32_t *ds = (i > 0 || kj == 0) ? sdig + ((size_t)Gj * cap + fj + i) * HW : bdig + (size_t)Gj * HW;
#pragma unroll
            for (int w = 0; w < HW; w++) v[u][w] = ok[u] ? ds[w] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 3; u++) {
            const int i = r + 16 * u;
            if (!ok[u]) continue;
#pragma unroll
            for (int w = 0; w < HW; w++) dig[(size_t)(dj + i) * HW + w] = v[u][w];
            need[dj + i] = 0;
        }
        for (int i = r + 48; i < nj; i += 16) {           // (longer lists than kSegMaxWinF allows: none)
#pragma unroll
            for (int w = 0; w < HW; w++) dig[(size_t)(dj + i) * HW + w] = sdig[((size_t)Gj * cap + fj + i) * HW + w];
            need[dj + i] = 0;
        }
    }
}
__global__ void __launch_bounds__(256) stitch_copy_kernel(const BlockDesc *__restrict__ blocks,
                                                          SegMeta *__restrict__ meta,
                                                          const uint32_t *__restrict__ spec, int cap,
                                                          const uint32_t *__restrict__ wgsum, int maxw,
                                                          const BlockState *__restrict__ bst,
                                                          uint32_t *__restrict__ offsets, int cap_blk,
                                                          const uint32_t *__restrict__ sdig = nullptr,
                                                          const uint32_t *__restrict__ bdig = nullptr,
                                                          uint32_t *__restrict__ dig = nullptr,
                                                          uint8_t *__restrict__ need = nullptr, int HW = 0)
{
    __shared__ uint32_t s_w[4];
    const int b = blockIdx.y, t = threadIdx.x;
    const BlockDesc bd = blocks[b];
    const int nseg = bd.nseg;
    if ((int)blockIdx.x * 256 >= nseg) return;
    if (bst[b].n_cuts == 0) return;                       // nothing on the path (or capacity error)
    const int k = blockIdx.x * 256 + t;
    const int G = bd.seg0 + k;
    const int cnt = k < nseg ? meta[G].pad[0] : 0;
    uint32_t total;
    const uint32_t dst = wgsum[(size_t)b * maxw + blockIdx.x] + wg_excl_scan((uint32_t)cnt, s_w, total);
    if (k < nseg && cnt > 0) {
        const int ext = meta[G].pad[1];
        if (ext >= 0) meta[G].ext_dst = (int)dst + ext;  // the repair's cuts (emit pass)
#if !HDRF_COOP
        const int n = meta[G].cp_n, from = meta[G].cp_from;
        const uint32_t *src = spec + (size_t)G * cap + from;
        uint32_t *out = offsets + (size_t)b * cap_blk + dst;
        for (int i = 0; i < n; i++) out[i] = src[i];
#endif
    }
#if HDRF_COOP
    {                                                     // (uniform) the pieces, 16 lanes per segment
        const bool mine = k < nseg && cnt > 0;
        const int n_l = mine ? meta[G].cp_n : 0, from_l = mine ? meta[G].cp_from : 0;
        const int l = lane_id(), r = l & 15;
        uint32_t *orow = offsets + (size_t)b * cap_blk;
        for (int j0 = 0; j0 < 64; j0 += 4) {
            const int jj = j0 + (l >> 4);
            const int nj = __shfl(n_l, jj, 64);
            if (!ballot64(nj > 0)) continue;
            const int Gj = __shfl(G, jj, 64), fj = __shfl(from_l, jj, 64), dj = __shfl((int)dst, jj, 64);
            uint32_t v[3];
#pragma unroll
            for (int u = 0; u < 3; u++) v[u] = r + 16 * u < nj ? spec[(size_t)Gj * cap + fj + r + 16 * u] : 0u;
#pragma unroll
            for (int u = 0; u < 3; u++)
                if (r + 16 * u < nj) orow[dj + r + 16 * u] = v[u];
            for (int i = r + 48; i < nj; i += 16) orow[dj + i] = spec[(size_t)Gj * cap + fj + i];
        }
    }
#endif
    if (sdig) {                                           // (uniform) the fused pass's digests
        const bool mine = k < nseg && cnt > 0;
        const int n_l = mine ? meta[G].cp_n : 0, from_l = mine ? meta[G].cp_from : 0;
        const bool head = mine && (k == 0 || (meta[G].pad[2] == 1 && (k == 1 || meta[G - 1].pad[0] > 0)));
        uint32_t *drow = dig + (size_t)b * cap_blk * HW;
        uint8_t *nrow = need + (size_t)b * cap_blk;
        if (HW == 5) copy_digests_wave<5>(n_l, G, from_l, (int)dst, head, k, cap, sdig, bdig, drow, nrow);
        else copy_digests_wave<7>(n_l, G, from_l, (int)dst, head, k, cap, sdig, bdig, drow, nrow);
    }
}

// 4. fallback + drop-last/append-size: one wave per block.  A block whose path ends at a failed
//    boundary continues with the exact sequential walk from the last proven cut (or from the
//    block start under the first-chunk rule); then :300-304 — the last detected cut is dropped and
//    the block size appended.
__global__ void __launch_bounds__(64) spec_fallback_kernel(const BlockDesc *__restrict__ blocks, int w, int maxlen,
                                                           uint32_t *__restrict__ offsets, int cap_blk,
                                                           BlockState *__restrict__ bst, const uint8_t *__restrict__ gm,
                                                           int gstride, int *__restrict__ err, int prio,
                                                           uint8_t *__restrict__ need = nullptr)
{    if (prio) __builtin_amdgcn_s_setprio(3);        // latency-bound chain: issue before co-running waves

    const int b = blockIdx.x;
    const BlockDesc bd = blocks[b];
    BlockState s = bst[b];
    uint32_t *off = offsets + (size_t)b * cap_blk;
    if (s.fail_dst >= 0) {
        WalkCfg W;
        W.base = bd.data; W.avail = (int)min(bd.readable, (uint64_t)0x7fffffff); W.size = (int)bd.len;
        W.w = w; W.maxlen = maxlen; W.gm = gm ? gm + (size_t)b * gstride : nullptr;
        const bool first = s.fail_dst == 0;
        const int p0 = first ? 0 : (int)off[s.fail_dst - 1];
        ListSink sink;
        sink.out = off + s.fail_dst; sink.cap = cap_blk - s.fail_dst; sink.cnt = 0; sink.stage = 0;
        NoStop nostop;
        bool ok = walk_chain(W, p0, first, sink, nostop);
        sink.flush();
#ifdef HDRF_DEBUG_CHUNK
        if (lane_id() == 0)
            printf("fallback: block %d fail_dst %d p0 %d cuts %d len %d\n", b, s.fail_dst, p0, sink.cnt, (int)bd.len);
#endif
        if (!ok && lane_id() == 0) atomicOr(err, 1);
        s.n_cuts = s.fail_dst + sink.cnt;
    }
    const int c = s.n_cuts;
    const int n = c > 0 ? c : 1;
    __builtin_amdgcn_s_waitcnt(0);
    if (lane_id() == 0) {
        off[n - 1] = (uint32_t)bd.len;
        s.n_chunks = n;
        bst[b] = s;
        if (need) need[(size_t)b * cap_blk + n - 1] = 1;  // [off[n - 2], len): not a chunk any lane cut
    }
}

}  // namespace hdrf

// ---- host-side launchers (called from api.hip) -------------------------------------------
namespace hdrf {
int lane_spec_cap(int seg_len, int w) { return seg_len / (w + 2) + 2 + kLaneOver; }

int setprio_mask()
{
    static const int m = [] { const char *e = getenv("HDRF_SETPRIO"); return e ? atoi(e) : 0; }();
    return m;
}

// The fused front (HDRF_FUSED=1): lanehash.hip's pass cuts and hashes the lane segments; the granule
// maxima are computed only when a boundary was queued for the repair walk (whose long searches and the
// sequential fallback read them); then the stitch as in the two-pass front, carrying the digests.
// Stage markers: the granule slot stays empty, the walk slot times the fused pass, the stitch slot the
// conditional granule pass, repair, stitch and fallback.
static hipError_t launch_fused_front(const BlockDesc *d_blocks, int nblocks, int64_t max_len, int total_waves, int nsegs,
                                     const ChunkScratch &X, int w, int maxlen, uint32_t *spec, int spec_cap,
                                     SegMeta *meta, BlockState *bst, uint32_t *offsets, int cap_blk, int *err,
                                     hipStream_t st, Marker *mk, const FusedFront &fz, int maxw)
{
    mk->mark(st);
    hipError_t e = hipMemsetAsync(X.rq_count, 0, sizeof(int), st);
    if (e == hipSuccess) e = hipMemsetAsync(X.irr, 0, sizeof(uint32_t) * (size_t)(nsegs / 32 + 2), st);
    if (e == hipSuccess) e = hipMemsetAsync(fz.need, 1, (size_t)nblocks * cap_blk, st);
    if (e == hipSuccess) e = hipMemsetAsync(fz.gm_need, 0, sizeof(int) * (size_t)nblocks, st);
    if (e != hipSuccess) return e;
    const int prio = setprio_mask();
    mk->mark(st);
    if ((e = launch_lane_hash(fz.hasher, d_blocks, nblocks, total_waves, w, maxlen, spec, spec_cap, meta, X.rq, X.rq_count,
                              X.rq_cap, X.irr, fz.sdig, fz.bdig, fz.gm_need, err, st)) != hipSuccess)
        return e;
    mk->mark(st);
    // HDRF_FUSED_GM=1: the granule maxima of the blocks with a repaired boundary (the repair walk's
    // long searches skip by them); default none: a boundary of every 4 GiB batch's blocks goes to the
    // repair walk, so the pass ran over the whole batch (4.56 GB, profiles/r06_fz_traffic.json)
    static const bool fz_gm = [] { const char *v = getenv("HDRF_FUSED_GM"); return v && atoi(v) != 0; }();
    const uint8_t *gm = fz_gm ? X.gm : nullptr;
    if (fz_gm) {
        const int gx = (int)(((max_len + 15) / 16 + kGmPerWg - 1) / kGmPerWg);
        hipLaunchKernelGGL((gmax2_kernel<true, true>), dim3(gx > 0 ? gx : 1, nblocks), dim3(256), 0, st, d_blocks, X.gm,
                           X.gstride, (prio >> 4) & 1, (const int *)fz.gm_need);
    }
    const int rgrid = 2048;                            // single-wave workgroups (below)
    const int HW = fz.hasher == 0 ? 5 : 7;
    hipLaunchKernelGGL(lane_repair_kernel, dim3(rgrid), dim3(64), 0, st, d_blocks, nblocks, X.rq, X.rq_count, X.rq_cap,
                       w, maxlen, spec, spec_cap, meta, offsets, cap_blk, gm, X.gstride, 0, (prio >> 1) & 1, X.rqkeep);
    hipLaunchKernelGGL(stitch_path_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, X.irr, meta, X.path, X.jx, X.jt, X.jcap,
                       (prio >> 1) & 1);
    hipLaunchKernelGGL(stitch_count_kernel, dim3(maxw, nblocks), dim3(256), 0, st, d_blocks, meta, X.path, X.jx, X.jt, X.jcap,
                       X.wgsum, maxw, err);
    hipLaunchKernelGGL(stitch_scan_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, X.path, X.wgsum, maxw, bst,
                       cap_blk, err);
    hipLaunchKernelGGL(stitch_copy_kernel, dim3(maxw, nblocks), dim3(256), 0, st, d_blocks, meta, spec, spec_cap,
                       X.wgsum, maxw, bst, offsets, cap_blk, (const uint32_t *)fz.sdig, (const uint32_t *)fz.bdig,
                       fz.dig, fz.need, HW);
    hipLaunchKernelGGL(lane_repair_kernel, dim3(rgrid), dim3(64), 0, st, d_blocks, nblocks, X.rq, X.rq_count, X.rq_cap,
                       w, maxlen, spec, spec_cap, meta, offsets, cap_blk, gm, X.gstride, 1, (prio >> 1) & 1, X.rqkeep);
    hipLaunchKernelGGL(spec_fallback_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, w, maxlen, offsets,
                       cap_blk, bst, gm, X.gstride, err, (prio >> 1) & 1, fz.need);
    return hipGetLastError();
}

hipError_t launch_chunking(const BlockDesc *d_blocks, int nblocks, int64_t max_len, int max_nseg, int total_waves,
                           int nsegs, const ChunkScratch &X, int w, int maxlen, uint32_t *spec, int spec_cap,
                           SegMeta *meta, BlockState *bst, uint32_t *offsets, int cap_blk, int *err, hipStream_t st,
                           Marker *mk, hipStream_t stg, hipEvent_t gdone, const FusedFront *fz)
{
    if ((max_len + 15) / 16 + 4 * kGmWin > X.gstride) return hipErrorInvalidValue;
    const int maxw = (max_nseg + 255) / 256;
    if (maxw > X.maxw) return hipErrorInvalidValue;
    if (fz) return launch_fused_front(d_blocks, nblocks, max_len, total_waves, nsegs, X, w, maxlen, spec, spec_cap, meta,
                                      bst, offsets, cap_blk, err, st, mk, *fz, maxw);
    const bool split = stg && stg != st && gdone;     // granule pass on its own stream, the walk waits for it
    hipStream_t sg = split ? stg : st;
    mk->mark(sg);
    hipError_t e = hipMemsetAsync(X.rq_count, 0, sizeof(int), st);
    if (e == hipSuccess) e = hipMemsetAsync(X.irr, 0, sizeof(uint32_t) * (size_t)(nsegs / 32 + 2), st);
    if (e != hipSuccess) return e;
    // HDRF_SETPRIO (bit mask): raise the issue priority of kernels over the co-running waves (bit 0
    // the lane walk, bit 1 repair / stitch path / sequential fallback, bit 2 the long SHA lanes, bit 3
    // all SHA lanes (sha.hip), bit 4 the granule pass, bit 5 place (store.hip))
    const int prio = setprio_mask();
    const int gx = (int)(((max_len + 15) / 16 + kGmPerWg - 1) / kGmPerWg);
    // HDRF_GMAX_V: 2 (default) gmax2 (15 VALU per granule, one 16-B store per thread), 1 the round-2 pass
    static const int gver = [] { const char *e = getenv("HDRF_GMAX_V"); return e ? atoi(e) : 2; }();
    if (gver == 2 && (stream_knobs() & 1))
        hipLaunchKernelGGL(gmax2_kernel<true>, dim3(gx > 0 ? gx : 1, nblocks), dim3(256), 0, sg, d_blocks, X.gm, X.gstride, (prio >> 4) & 1);
    else if (gver == 2)
        hipLaunchKernelGGL(gmax2_kernel<false>, dim3(gx > 0 ? gx : 1, nblocks), dim3(256), 0, sg, d_blocks, X.gm, X.gstride, (prio >> 4) & 1);
    else if (stream_knobs() & 1)
        hipLaunchKernelGGL(gmax_kernel<true>, dim3(gx > 0 ? gx : 1, nblocks), dim3(256), 0, sg, d_blocks, X.gm, X.gstride, (prio >> 4) & 1);
    else
        hipLaunchKernelGGL(gmax_kernel<false>, dim3(gx > 0 ? gx : 1, nblocks), dim3(256), 0, sg, d_blocks, X.gm, X.gstride, (prio >> 4) & 1);
    mk->mark(sg);
    if (split) {
        if ((e = hipEventRecord(gdone, sg)) != hipSuccess || (e = hipStreamWaitEvent(st, gdone, 0)) != hipSuccess)
            return e;
    }
    // HDRF_WALK_LDS: dynamic LDS per walk workgroup (occupancy throttle: fewer lanes in flight keep
    // their granule-maximum lines in L2 between chunk steps)
    static const int walk_lds = [] { const char *v = getenv("HDRF_WALK_LDS"); return v ? atoi(v) : 0; }();
    // HDRF_WALK_RING: 1 / 0 force the ring on / off; default: X.ring (the caller's choice)
    static const int ring_env = [] { const char *v = getenv("HDRF_WALK_RING"); return v ? atoi(v) : -1; }();
    const int ring_on = ring_env >= 0 ? ring_env : X.ring;
    if (ring_on)
        hipLaunchKernelGGL(lane_walk_kernel<true>, dim3((total_waves + 3) / 4), dim3(256), walk_lds, st, d_blocks, nblocks, total_waves,
                           X.gm, X.gstride, w, maxlen, spec, spec_cap, meta, X.rq, X.rq_count, X.rq_cap, X.irr, err, 1,
                           prio & 1);
    else
    hipLaunchKernelGGL(lane_walk_kernel<false>, dim3((total_waves + 3) / 4), dim3(256), walk_lds, st, d_blocks, nblocks, total_waves,
                       X.gm, X.gstride, w, maxlen, spec, spec_cap, meta, X.rq, X.rq_count, X.rq_cap, X.irr, err, ring_on, prio & 1);
    mk->mark(st);
    // 2048 repair waves loop over the queue, one per workgroup: the chain's small kernels start in
    // whatever wave slots the co-running kernels leave (a 4-wave workgroup needs four on one CU)
    const int rgrid = 2048;
    hipLaunchKernelGGL(lane_repair_kernel, dim3(rgrid), dim3(64), 0, st, d_blocks, nblocks, X.rq, X.rq_count, X.rq_cap,
                       w, maxlen, spec, spec_cap, meta, offsets, cap_blk, X.gm, X.gstride, 0, (prio >> 1) & 1, X.rqkeep);
    hipLaunchKernelGGL(stitch_path_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, X.irr, meta, X.path, X.jx, X.jt, X.jcap,
                       (prio >> 1) & 1);
    hipLaunchKernelGGL(stitch_count_kernel, dim3(maxw, nblocks), dim3(256), 0, st, d_blocks, meta, X.path, X.jx, X.jt, X.jcap,
                       X.wgsum, maxw, err);
    hipLaunchKernelGGL(stitch_scan_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, X.path, X.wgsum, maxw, bst,
                       cap_blk, err);
    hipLaunchKernelGGL(stitch_copy_kernel, dim3(maxw, nblocks), dim3(256), 0, st, d_blocks, meta, spec, spec_cap,
                       X.wgsum, maxw, bst, offsets, cap_blk);
    hipLaunchKernelGGL(lane_repair_kernel, dim3(rgrid), dim3(64), 0, st, d_blocks, nblocks, X.rq, X.rq_count, X.rq_cap,
                       w, maxlen, spec, spec_cap, meta, offsets, cap_blk, X.gm, X.gstride, 1, (prio >> 1) & 1, X.rqkeep);
    hipLaunchKernelGGL(spec_fallback_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, w, maxlen, offsets,
                       cap_blk, bst, X.gm, X.gstride, err, (prio >> 1) & 1);
    return hipGetLastError();
}
}  // namespace hdrf
