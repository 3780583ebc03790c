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
//   1. spec_walk  — each block is cut into segments; one wave walks the chain from each
//                   segment start as if a cut were there, recording its cuts plus up to
//                   64 "overrun" cuts past the segment end.  Bytes are streamed as 1 KiB
//                   tiles (64 lanes x 16 B, coalesced) with two tiles of prefetch; the
//                   window max is a per-granule max + DPP reduction, the search is a
//                   ballot over granules >= M followed by a scalar SWAR byte test.
//   2. spec_sync  — chains are deterministic in p, so the true chain (from segment k's
//                   overrun) and segment k+1's speculative chain agree from the first cut
//                   they share.  One wave per segment boundary finds that cut.
//   3. spec_plan / spec_copy — prefix-sum the pieces and compact them into offsets[].
//   4. spec_fallback — blocks whose chains did not meet (periodic data) are finished by a
//                   sequential exact walk from the last proven cut; every block then gets
//                   the reference's drop-last/append-size rule.
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
};

enum : int { kWindow = 0, kSearchFF = 1, kSearchGen = 2 };

struct Chain {
    int p;         // last cut (chunk start)
    int state;
    int q, lim;    // pending search range
    uint32_t m;    // threshold (biased) of a general search
    bool first;    // the very first chunk of a block: M has no 0 floor
    bool ended;    // chain ended because the data ended
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

// Cut sink that only counts (the repair pass finds where a chain merges before anything is written).
struct CountSink {
    int cap;
    int cnt;
    uint32_t stage;
    __device__ __forceinline__ void store64(int, uint32_t) {}
    __device__ __forceinline__ bool push(uint32_t)
    {
        if (cnt >= cap) return false;
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
    int T = p & ~1023;
    uint4 R0 = tile_raw(c, T), R1 = tile_raw(c, T + 1024), R2 = tile_raw(c, T + 2048), R3 = tile_raw(c, T + 3072);
    uint32_t f0 = ffmask16(R0), f1 = ffmask16(R1), f2 = 0, f3 = 0;
    unsigned long long b0 = ballot64(f0 != 0), b1 = ballot64(f1 != 0), b2 = 0, b3 = 0;
    for (;;) {
        if (!process_view(c, ch, R0, R1, f0, f1, b0, b1, T, sink, stop)) break;
        T += 1024; f2 = ffmask16(R2); b2 = ballot64(f2 != 0); R0 = tile_raw(c, T + 3072);
        if (!process_view(c, ch, R1, R2, f1, f2, b1, b2, T, sink, stop)) break;
        T += 1024; f3 = ffmask16(R3); b3 = ballot64(f3 != 0); R1 = tile_raw(c, T + 3072);
        if (!process_view(c, ch, R2, R3, f2, f3, b2, b3, T, sink, stop)) break;
        T += 1024; f0 = ffmask16(R0); b0 = ballot64(f0 != 0); R2 = tile_raw(c, T + 3072);
        if (!process_view(c, ch, R3, R0, f3, f0, b3, b0, T, sink, stop)) break;
        T += 1024; f1 = ffmask16(R1); b1 = ballot64(f1 != 0); R3 = tile_raw(c, T + 3072);
    }
    return ch.ended;
}


// ------------------------------------------------------------------------------------------
// 1. lane walk (the speculative pass).  Every block is cut into segments of seg_len bytes (a
//    multiple of 702); lane l of a wave walks the chain from the start of segment k = 63*wl + l
//    as if a cut were there, one 32-B unit at a time, entirely in VALU:
//      window part   M = max(M, unit max) while the unit lies inside [p, p+700]; the unit
//                    holding p (a cut, or the segment start) is folded in later from a saved
//                    copy (every 8 units, always before the window can end); the unit holding
//                    p+700 needs its exact prefix only when its max exceeds M
//      search part   the 32-bit mask of bytes >= M (SWAR carry test + v_dot4 bit gather), cut to
//                    [p+701, min(p+maxlen, size-1)], plus the forced position p+maxlen; the first
//                    set bit j gives the cut j+1 (DN/DataDeduplicator.java:276-294)
//    Its cuts go to an LDS list (u16 offsets from the segment start; written to the segment's
//    global list when the lane stops).  Past its segment end (overrun) a lane compares each cut
//    with the next lane's list (the next segment's chain, walked concurrently and seg_len bytes
//    ahead): the first shared cut proves the chains equal from there on, the lane records (i, j)
//    and stops.  Lane 63 walks the NEXT wave's first segment (a helper: LDS only), so every
//    boundary is settled inside one wave.  A lane that meets no shared cut within kLaneOver cuts
//    or ~seg_len bytes reports kSyncFail and queues its boundary for the repair pass.
//    Bytes move HBM -> VGPR -> LDS in 4 KiB steps (each lane fetches 16 B of four segments, so a
//    wave-instruction reads 16 x 64 contiguous bytes), prefetched two steps ahead, and every lane
//    reads its own 64 B back with conflict-free ds_read_b128 (XOR-swizzled 16-B slots).

// A unit is 32 bytes (two granules, 8 dwords) of one lane's segment.  Biasing (XOR 0x80, signed
// order == unsigned order) is folded into the masks below.
struct Unit {
    uint32_t d[8];
};

// max over the 32 biased bytes: even bytes and odd bytes as u16 lanes (odd ones scaled by 256,
// which keeps their order), v_pk_max_u16 trees, then the two halves
__device__ __forceinline__ uint32_t unit_max(const Unit &u)
{
    uint32_t e = 0, o = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        e = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(as_us2(e), as_us2((u.d[i] ^ 0x80808080u) & 0x00ff00ffu)));
        o = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(as_us2(o), as_us2((u.d[i] ^ 0x80808080u) & 0xff00ff00u)));
    }
    const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(as_us2(e), as_us2(o >> 8)));
    return max(m & 0xffffu, m >> 16);
}

// max over the biased bytes whose unit index is in [lo, hi] (0 <= lo, hi <= 31)
__device__ __forceinline__ uint32_t unit_range_max(const Unit &u, int lo, int hi)
{
    Unit m;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int a = min(max(lo - 4 * i, 0), 4), b = min(max(hi - 4 * i + 1, 0), 4);   // keep bytes [a, b)
        const uint32_t keep = (a >= b) ? 0u : ((b == 4 ? ~0u : ((1u << (8 * b)) - 1u)) & (~0u << (8 * a)));
        m.d[i] = ((u.d[i] ^ 0x80808080u) & keep) ^ 0x80808080u;     // dropped bytes read as biased 0
    }
    return unit_max(m);
}

// 32-bit mask of the biased bytes >= m (1 <= m <= 255): SWAR carry-out of byte + (256 - m), the
// bit-7 flags gathered with v_dot4_u32_u8 (weights 1..128 per dword pair)
// bit 7 of each byte of raw dword d where the biased byte (d ^ 0x80) >= m: the carry out of the
// byte sum (d ^ 0x80) + (256 - m) = maj(NOT d7, C7, s7) with s = low-7-bit sum; 4 VALU (and, add,
// bitop3, and)
__device__ __forceinline__ uint32_t ge_flags(uint32_t d, uint32_t C, uint32_t Cm)
{
    const uint32_t s = (d & 0x7f7f7f7fu) + Cm;
    return __builtin_amdgcn_bitop3_b32(d, C, s, 0x8e) & 0x80808080u;   // 0x8e: maj(NOT d, C, s)
}
__device__ __forceinline__ uint32_t unit_ge(const Unit &u, uint32_t m)
{
    const uint32_t C = __builtin_amdgcn_perm(256u - m, 256u - m, 0u), Cm = C & 0x7f7f7f7fu;
    uint32_t x[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const uint32_t f0 = ge_flags(u.d[2 * p], C, Cm), f1 = ge_flags(u.d[2 * p + 1], C, Cm);
        x[p] = __builtin_amdgcn_udot4(f1, 0x80402010u, __builtin_amdgcn_udot4(f0, 0x08040201u, 0u, false), false);
    }
    return (x[0] >> 7) | (x[1] << 1) | (x[2] << 9) | (x[3] << 17);
}

constexpr int kNegPos = -(1 << 30);      // "no forced cut possible" relative position

// LDS of one wave (one array for the whole workgroup: a second __shared__ object beside LDS-DMA
// staging makes hipcc drain vmcnt before LDS reads): a ring of 3 step images of 2 KiB (lane l's
// 32 B at 16-B slots 2l + (c ^ ((l >> 3) & 1)), filled by LDS-DMA), each lane's cuts as u16 offsets
// from its segment start, and their counts.
constexpr int kRingSlot = 2048;
constexpr int kWaveLds = 3 * kRingSlot + 64 * kLdsCuts * 2 + 64;
typedef __attribute__((address_space(3))) u32x4v lds_u4;
typedef __attribute__((address_space(3))) volatile uint16_t lds_u16v;
typedef __attribute__((address_space(3))) volatile uint8_t lds_u8v;
typedef __attribute__((address_space(3))) uint8_t lds_u8;

__global__ void __launch_bounds__(256) lane_walk_kernel(const BlockDesc *__restrict__ blocks, int nblocks,
                                                        int total_waves, int w, int maxlen,
                                                        uint32_t *__restrict__ spec, int cap,
                                                        SegMeta *__restrict__ meta, int *__restrict__ rq,
                                                        int *__restrict__ rq_count, int rq_cap,
                                                        int *__restrict__ err)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[4 * kWaveLds];
    const int wv = blockIdx.x * 4 + wave_id();
    if (wv >= total_waves) return;
    lds_u8 *wl_lds = (lds_u8 *)s_lds + kWaveLds * wave_id();
    lds_u16v *vcuts = (lds_u16v *)(wl_lds + 3 * kRingSlot);          // read by the neighbouring lane:
    lds_u8v *vcnt = (lds_u8v *)(wl_lds + 3 * kRingSlot + 64 * kLdsCuts * 2);   // volatile, never cached
    int bi = 0;
    for (int i = 1; i < nblocks; i++)
        if (blocks[i].wave0 <= wv) bi = i;
    const BlockDesc bd = blocks[bi];
    const int l = lane_id();
    const int wl = wv - bd.wave0;
    const int nseg = bd.nseg, Ls = bd.seg_len, size = (int)bd.len;
    const int avail = (int)min(bd.readable, (uint64_t)0x7fffffff);
    const uint8_t *base = bd.data;
    const int k = wl * kWaveSegs + l;                 // lane 63: the next wave's first segment
    const bool exists = k < nseg;
    const bool real = exists && l < kWaveSegs;
    const int s = k * Ls;
    const int e = (real && k + 1 < nseg) ? (k + 1) * Ls : 0x7fffffff;   // the next segment's start
    const int over_lim = (e == 0x7fffffff) ? 0x7fffffff : e + Ls - 64;  // overrun byte cap (unit start)
    const int ncap = min(cap, kLdsCuts);

    // loader: per step (one 32-B unit per segment) two LDS-DMA wave-instructions; in instruction i
    // this lane moves 16 B of segment lane j = 32 i + l/2 (chunk c) into ring slot 2j + (l & 1), as
    // long as that lane is active and the bytes are readable
    uint32_t ld_off[2];
    int ld_last[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int j = 32 * i + (l >> 1);
        const int kj = wl * kWaveSegs + j;
        const int c = (l & 1) ^ ((j >> 3) & 1);
        const int off = ((kj * Ls) & ~15) + 16 * c;
        ld_off[i] = (uint32_t)off;
        ld_last[i] = kj < nseg && off + 16 <= avail ? (avail - 16 - off) >> 5 : -1;
    }
    const int jsh = l >> 1;
    const uint32_t rd0 = 32u * (uint32_t)l + 16u * (uint32_t)((l >> 3) & 1);   // this lane's chunk 0 / 1
    const uint32_t rd1 = 32u * (uint32_t)l + 16u * (uint32_t)(((l >> 3) & 1) ^ 1);

    // chain state (positions relative to the current unit start g)
    int g = s & ~15;
    int rb = s + w - g;                                           // window end p + w
    int rL = min(s + maxlen, size - 1) - g;                       // search limit
    int rf = (s + maxlen <= size - 1) ? s + maxlen - g : kNegPos; // forced-cut position
    uint32_t M = (s == 0) ? 0u : 0x80u;                           // biased; 0x80 = the 0 floor (:281)
    bool pend = false;
    int pend_lo = 0;
    Unit pend_u;
#pragma unroll
    for (int i = 0; i < 8; i++) pend_u.d[i] = 0;
    int n = 0, n_main = -1, ptr = 0, sync = kSyncEnd;
    bool active = exists && g <= size - 1, overflow = false;
    vcnt[l] = 0;

    // step t's two LDS-DMAs into ring slot t % 3 (vmcnt counted by hand: exactly 2 per step, no other
    // vector-memory instruction in the loop)
    auto issue = [&](int t, unsigned long long am) {
        const unsigned long long amj = am >> jsh;                // bit 32 i = segment lane j_i
        lds_u8 *slot = wl_lds + kRingSlot * (t % 3);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const bool ok = t <= ld_last[i] && ((amj >> (32 * i)) & 1ull);
            const uint32_t off = ok ? ld_off[i] + 32u * (uint32_t)t : 0u;     // finished: re-read byte 0
            __builtin_amdgcn_global_load_lds((const HDRF_GLOBAL void *)(base + off),
                                             (__attribute__((address_space(3))) void *)(slot + 1024 * i), 16, 0, 0);
        }
    };
    auto unit = [&](const Unit &u) {
        const uint32_t um = unit_max(u);
        M = (unsigned)(rb - 31) <= (unsigned)(w - 31) ? max(M, um) : M;                 // inside the window
        if ((unsigned)rb <= 30u && um > M) M = max(M, unit_range_max(u, 0, rb));        // window ends here (rare)
        const int lo = min(max(rb + 1, 0), 32), hi = min(max(rL, -1), 31);
        const uint32_t smask = (lo > 31 ? 0u : (~0u << lo)) & (hi < 0 ? 0u : (~0u >> (31 - hi)));
        const uint32_t V = M == 0 ? ~0u : unit_ge(u, max(M, 1u));
        const uint32_t F = (unsigned)rf <= 31u ? (1u << rf) : 0u;
        const uint32_t H = (V | F) & smask;
        if (H) {
            const int h = __builtin_ctz(H);
            const int cut = g + h + 1;
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
                if (ptr < sc && (int)sl[ptr] == rel) { sync = (ci - n_main) | (ptr << 16); active = false; }
                else if (n - n_main >= kLaneOver) { sync = kSyncFail; active = false; }
            }
            M = 0x80u;
            rb = h + 1 + w;
            rL = min(h + 1 + maxlen, size - 1 - g);
            rf = (cut + maxlen <= size - 1) ? h + 1 + maxlen : kNegPos;
        }
        if ((unsigned)(rb - w - 1) <= 30u) { pend = true; pend_u = u; pend_lo = rb - w; }   // window starts here
        rb -= 32; rL -= 32; rf -= 32; g += 32;
        const bool capped = active && g >= over_lim && g <= size - 1;    // overrun byte cap
        sync = capped ? kSyncFail : sync;
        active = active && g <= size - 1 && !capped && !overflow;        // data end: no more cuts
    };
    unsigned long long am = ballot64(active);
    issue(0, am);
    issue(1, am);
    for (int t = 0;; t++) {
        if ((t & 7) == 0 && ballot64(pend)) {                 // fold in the window-start units
            if (pend) { M = max(M, unit_range_max(pend_u, pend_lo, 31)); pend = false; }
        }
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");     // step t landed (step t + 1 may be in flight)
        const lds_u8 *slot = wl_lds + kRingSlot * (t % 3);
        const u32x4v x0 = *(const lds_u4 *)(slot + rd0), x1 = *(const lds_u4 *)(slot + rd1);
        Unit U;
        U.d[0] = x0.x; U.d[1] = x0.y; U.d[2] = x0.z; U.d[3] = x0.w;
        U.d[4] = x1.x; U.d[5] = x1.y; U.d[6] = x1.z; U.d[7] = x1.w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slot t % 3 read before step t + 3 refills it
        issue(t + 2, am);
        if (active) unit(U);
        am = ballot64(active);
        if (!ballot64(active && l < kWaveSegs)) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // no LDS-DMA lands after the wave is gone
    if (overflow && real) atomicOr(err, 64);
    if (real) {
        const int G = bd.seg0 + k;
        uint32_t *list = spec + (size_t)G * cap;
        for (int i = 0; i < n; i++) list[i] = (uint32_t)s + (uint32_t)vcuts[l * kLdsCuts + i];
        if (n_main < 0) n_main = n;
        SegMeta m;
        m.n_main = n_main; m.n_over = n - n_main; m.sync = sync; m.jmp = 0; m.jj = 0; m.n_ext = 0; m.ext_dst = -1;
        m.cp_from = 0; m.cp_n = 0; m.cp_dst = 0; m.pad[0] = m.pad[1] = m.pad[2] = 0;
        meta[G] = m;
        if (sync == kSyncFail) {
            const int q = atomicAdd(rq_count, 1);
            if (q < rq_cap) rq[q] = G;                        // beyond rq_cap: no repair, stitch falls back
        }
    }
}

// 2. repair: one wave per failed boundary k (queued by the lane walk), the exact sequential walker
//    continues segment k's chain from its last cut.  find: every new cut c is looked up in the list
//    of the segment m = c / seg_len holding it (m > k); once found at index j, segment k's chain
//    continues as segment m's from there (kSyncJump, k + jmp = m, jj = j, n_ext cuts walked); no
//    shared cut within kRepairCuts cuts / kRepairBytes bytes, or the block end: kSyncGiveUp.
//    emit (after the stitch placed it): the same walk writes its n_ext - 1 cuts before the shared
//    one into the block's offsets, for repairs on the block's path.
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

__global__ void __launch_bounds__(256) lane_repair_kernel(const BlockDesc *__restrict__ blocks, int nblocks,
                                                          const int *__restrict__ rq, const int *__restrict__ rq_count,
                                                          int rq_cap, int w, int maxlen,
                                                          const uint32_t *__restrict__ spec, int cap,
                                                          SegMeta *__restrict__ meta, uint32_t *__restrict__ offsets,
                                                          int cap_blk, int emit)
{
    const int nw = gridDim.x * 4;
    const int cnt = min(*rq_count, rq_cap);
    for (int q = blockIdx.x * 4 + wave_id(); q < cnt; q += nw) {
        const int G = __builtin_amdgcn_readfirstlane(rq[q]);
        int bi = 0;
        for (int i = 1; i < nblocks; i++)
            if (blocks[i].seg0 <= G) bi = i;
        const BlockDesc bd = blocks[bi];
        const int k = G - bd.seg0;
        const SegMeta m = meta[G];
        if (emit && (m.sync != kSyncJump || m.ext_dst < 0 || m.n_ext <= 1)) continue;
        const int n = m.n_main + m.n_over;
        const int s_k = k * bd.seg_len;
        const int p0 = n > 0 ? (int)spec[(size_t)G * cap + n - 1] : s_k;
        const bool first = n == 0 && s_k == 0;
        WalkCfg W;
        W.base = bd.data; W.avail = (int)min(bd.readable, (uint64_t)0x7fffffff); W.size = (int)bd.len;
        W.w = w; W.maxlen = maxlen;
        if (!emit) {
            CountSink sink;
            sink.cap = kRepairCuts; sink.cnt = 0; sink.stage = 0;
            MergeStop st;
            st.spec = spec; st.meta = meta; st.cap = cap; st.seg0 = bd.seg0; st.k = k; st.nseg = bd.nseg;
            st.Ls = bd.seg_len; st.lim_cut = p0 + kRepairBytes;
            (void)walk_chain(W, p0, first, sink, st);
            if (lane_id() == 0) {
                if (st.status == 1) {
                    meta[G].jmp = st.res_m - k;
                    meta[G].jj = st.res_j;
                    meta[G].n_ext = sink.cnt;
                    meta[G].sync = kSyncJump;
                } else {
                    meta[G].sync = kSyncGiveUp;
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

// 3. stitch: one 1024-thread workgroup per block.  The block's chain is segment 0's list, then,
//    boundary by boundary, the next segment's list from the shared cut: synced boundaries go to
//    k + 1 (seg k keeps its overrun cuts [0, i)), repaired ones jump to k + jmp (seg k keeps all
//    its cuts and the repair's n_ext - 1 cuts; the segments jumped over are off the path); the
//    path ends at the last segment, at a chain that ran to the block end, or at a failed boundary
//    (seg k keeps all its cuts and the sequential fallback continues from the last one).  The
//    nodes that are not "synced to k + 1" are compacted (prefix over the threads' segment runs)
//    and thread 0 follows the path through them; then each thread sizes its segments' pieces, a
//    prefix places them and each thread copies its pieces.
constexpr int kStitchNodes = 4096;       // compacted irregular boundaries per block (more: fallback)
__global__ void __launch_bounds__(1024) lane_stitch_kernel(const BlockDesc *__restrict__ blocks,
                                                           const uint32_t *__restrict__ spec, int cap,
                                                           SegMeta *__restrict__ meta,
                                                           uint32_t *__restrict__ offsets, int cap_blk,
                                                           BlockState *__restrict__ bst, int *__restrict__ err)
{
    __shared__ uint32_t s_sum[1024];
    __shared__ int s_nx[kStitchNodes];       // compacted irregular nodes (ascending)
    __shared__ int s_jx[kStitchNodes];       // on-path jumps: source node, target, shared-cut index
    __shared__ int s_jm[kStitchNodes];
    __shared__ int s_jj[kStitchNodes];
    __shared__ int s_nj, s_term, s_fb;
    const int b = blockIdx.x;
    const BlockDesc bd = blocks[b];
    const int nseg = bd.nseg, t = threadIdx.x;
    SegMeta *mt = meta + bd.seg0;
    const int per = (nseg + 1023) / 1024;
    const int k0 = min(nseg, t * per), k1 = min(nseg, k0 + per);
    auto scan = [&](uint32_t v) -> uint32_t {           // exclusive prefix over the threads; s_sum[1023] = total
        s_sum[t] = v;
        __syncthreads();
        for (int d = 1; d < 1024; d <<= 1) {
            const uint32_t x = t >= d ? s_sum[t - d] : 0u;
            __syncthreads();
            s_sum[t] += x;
            __syncthreads();
        }
        return s_sum[t] - v;
    };
    // (a) compact the irregular boundaries (sync < 0), k < nseg - 1
    uint32_t nirr = 0;
    for (int k = k0; k < k1; k++) nirr += (k < nseg - 1 && mt[k].sync < 0);
    uint32_t pos = scan(nirr);
    const int tot_irr = (int)s_sum[1023];
    for (int k = k0; k < k1; k++)
        if (k < nseg - 1 && mt[k].sync < 0) {
            if (pos < (uint32_t)kStitchNodes) s_nx[pos] = k;
            pos++;
        }
    __syncthreads();
    // (b) thread 0 follows the path through the irregular nodes
    if (t == 0) {
        const int nnx = min(tot_irr, kStitchNodes);
        int cur = 0, i = 0, nj = 0, term = nseg - 1, fb = 0;
        for (;;) {
            while (i < nnx && s_nx[i] < cur) i++;
            if (i >= nnx) {
                if (tot_irr > kStitchNodes) { term = cur; fb = 1; }   // uncompacted nodes ahead: fall back here
                break;
            }
            const int x = s_nx[i];
            const int sy = mt[x].sync;
            if (sy == kSyncJump && nj < kStitchNodes) {
                s_jx[nj] = x; s_jm[nj] = x + mt[x].jmp; s_jj[nj] = mt[x].jj; nj++;
                cur = x + mt[x].jmp;
                continue;
            }
            term = x;
            fb = sy != kSyncEnd;
            break;
        }
        s_nj = nj; s_term = term; s_fb = fb;
    }
    __syncthreads();
    const int nj = s_nj, term = s_term;
    // (c) the piece of every segment on the path
    auto piece = [&](int k, int &from, int &cnt, int &ext) {
        from = 0; cnt = 0; ext = -1;
        if (k > term) return;
        int lo = 0, hi = nj;                               // last jump with source < k
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (s_jx[mid] < k) lo = mid + 1; else hi = mid; }
        const int ji = lo - 1;
        bool target = false;
        if (ji >= 0) {
            if (s_jm[ji] > k) return;                      // jumped over
            target = s_jm[ji] == k;
        }
        const SegMeta m = mt[k];
        if (k == 0) from = 0;
        else if (target) from = s_jj[ji];
        else from = (mt[k - 1].sync >> 16) & 0xffff;
        if (from > m.n_main) { atomicOr(err, 128); from = m.n_main; }   // never: a shared cut is a main cut
        cnt = m.n_main - from;
        if (k == term) cnt += m.n_over;
        else if (m.sync == kSyncJump) { cnt += m.n_over; ext = cnt; cnt += m.n_ext - 1; }
        else cnt += m.sync & 0xffff;
    };
    uint32_t local = 0;
    for (int k = k0; k < k1; k++) {
        int from, cnt, ext;
        piece(k, from, cnt, ext);
        local += (uint32_t)cnt;
    }
    uint32_t dst = scan(local);
    const uint32_t total = s_sum[1023];
    if (total > (uint32_t)cap_blk) {
        if (t == 0) atomicOr(err, 1);
        for (int k = k0; k < k1; k++) mt[k].cp_n = 0;
        return;
    }
    for (int k = k0; k < k1; k++) {                        // the plan; lane_copy_kernel moves the cuts
        int from, cnt, ext;
        piece(k, from, cnt, ext);
        if (ext >= 0) mt[k].ext_dst = (int)dst + ext;      // the repair's cuts (emit pass)
        mt[k].cp_from = from;
        mt[k].cp_n = ext >= 0 ? ext : cnt;
        mt[k].cp_dst = b * cap_blk + (int)dst;
        dst += (uint32_t)cnt;
    }
    if (t == 0) {
        BlockState s;
        s.n_cuts = (int)total;
        s.fail_dst = s_fb ? (int)total : -1;
        s.fail_p0 = 0; s.n_chunks = 0;
        bst[b] = s;
    }
}

// 3b. copy: 32 lanes per segment move its planned piece of the speculative list into the offsets
__global__ void __launch_bounds__(256) lane_copy_kernel(const uint32_t *__restrict__ spec, int cap,
                                                        const SegMeta *__restrict__ meta, int nsegs,
                                                        uint32_t *__restrict__ offsets)
{
    const int G = blockIdx.x * 8 + (threadIdx.x >> 5);
    const int i = threadIdx.x & 31;
    if (G >= nsegs) return;
    const int n = meta[G].cp_n;
    if (i < n) offsets[meta[G].cp_dst + i] = spec[(size_t)G * cap + meta[G].cp_from + i];
}

// 4. fallback + drop-last/append-size: one wave per block.  A block whose path ends at a failed
//    boundary continues with the exact sequential walk from the last proven cut (or from the
//    block start under the first-chunk rule); then :300-304 — the last detected cut is dropped and
//    the block size appended.
__global__ void __launch_bounds__(64) spec_fallback_kernel(const BlockDesc *__restrict__ blocks, int w, int maxlen,
                                                           uint32_t *__restrict__ offsets, int cap_blk,
                                                           BlockState *__restrict__ bst, int *__restrict__ err)
{
    const int b = blockIdx.x;
    const BlockDesc bd = blocks[b];
    BlockState s = bst[b];
    uint32_t *off = offsets + (size_t)b * cap_blk;
    if (s.fail_dst >= 0) {
        WalkCfg W;
        W.base = bd.data; W.avail = (int)min(bd.readable, (uint64_t)0x7fffffff); W.size = (int)bd.len;
        W.w = w; W.maxlen = maxlen;
        const bool first = s.fail_dst == 0;
        const int p0 = first ? 0 : (int)off[s.fail_dst - 1];
        ListSink sink;
        sink.out = off + s.fail_dst; sink.cap = cap_blk - s.fail_dst; sink.cnt = 0; sink.stage = 0;
        NoStop nostop;
        bool ok = walk_chain(W, p0, first, sink, nostop);
        sink.flush();
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
    }
}

}  // namespace hdrf

// ---- host-side launchers (called from api.hip) -------------------------------------------
namespace hdrf {
int lane_spec_cap(int seg_len, int w) { return seg_len / (w + 2) + 2 + kLaneOver; }

hipError_t launch_chunking(const BlockDesc *d_blocks, int nblocks, int total_waves, int nsegs, int w, int maxlen,
                           uint32_t *spec, int spec_cap, SegMeta *meta, int *rq, int *rq_count, int rq_cap,
                           BlockState *bst, uint32_t *offsets, int cap_blk, int *err, hipStream_t st, Marker *mk)
{
    mk->mark(st);
    hipError_t e = hipMemsetAsync(rq_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lane_walk_kernel, dim3((total_waves + 3) / 4), dim3(256), 0, st, d_blocks, nblocks, total_waves,
                       w, maxlen, spec, spec_cap, meta, rq, rq_count, rq_cap, err);
    mk->mark(st);
    const int rgrid = 512;                             // 2048 repair waves loop over the queue
    hipLaunchKernelGGL(lane_repair_kernel, dim3(rgrid), dim3(256), 0, st, d_blocks, nblocks, rq, rq_count, rq_cap, w,
                       maxlen, spec, spec_cap, meta, offsets, cap_blk, 0);
    hipLaunchKernelGGL(lane_stitch_kernel, dim3(nblocks), dim3(1024), 0, st, d_blocks, spec, spec_cap, meta, offsets,
                       cap_blk, bst, err);
    hipLaunchKernelGGL(lane_copy_kernel, dim3((nsegs + 7) / 8), dim3(256), 0, st, spec, spec_cap, meta, nsegs, offsets);
    hipLaunchKernelGGL(lane_repair_kernel, dim3(rgrid), dim3(256), 0, st, d_blocks, nblocks, rq, rq_count, rq_cap, w,
                       maxlen, spec, spec_cap, meta, offsets, cap_blk, 1);
    hipLaunchKernelGGL(spec_fallback_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, w, maxlen, offsets,
                       cap_blk, bst, err);
    return hipGetLastError();
}
}  // namespace hdrf
