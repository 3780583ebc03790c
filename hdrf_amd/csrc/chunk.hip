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
                    if ((cnt & 63) == 0) sink.out[cnt - 64 + lane_id()] = stage;
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
    __device__ __forceinline__ bool push(uint32_t cut)
    {
        if (cnt >= cap) return false;
        if (lane_id() == (cnt & 63)) stage = cut;
        cnt++;
        if ((cnt & 63) == 0) out[cnt - 64 + lane_id()] = stage;
        return true;
    }
    __device__ __forceinline__ void flush()
    {
        const int r = cnt & 63;
        if (r && lane_id() < r) out[(cnt & ~63) + lane_id()] = stage;
    }
};

// Stop predicates: operator() is evaluated after every cut; cut_thr/cnt_thr tell the fast path the
// first cut position / count at which the predicate can change, so it only asks then.
struct SpecStop {          // segment walk: cuts past s_next are overrun; stop after kOverrun of them
    int s_next;
    int n_main;
    __device__ __forceinline__ bool operator()(int cut, int cnt)
    {
        if (n_main < 0 && cut >= s_next) n_main = cnt - 1;
        return n_main >= 0 && cnt - n_main >= kOverrun;
    }
    __device__ __forceinline__ int cut_thr() const { return n_main < 0 ? s_next : 0x7fffffff; }
    __device__ __forceinline__ int cnt_thr() const { return n_main < 0 ? 0x7fffffff : n_main + kOverrun; }
};
struct NoStop {
    __device__ __forceinline__ bool operator()(int, int) { return false; }
    __device__ __forceinline__ int cut_thr() const { return 0x7fffffff; }
    __device__ __forceinline__ int cnt_thr() const { return 0x7fffffff; }
};

// Walk the chain from p (a cut, or the block start when first) calling sink.push(cut) for
// every cut until the data ends (returns true) or the sink/stop predicate says stop (false).
template <class Stop>
__device__ __forceinline__ bool walk_chain(const WalkCfg &c, int p, bool first, ListSink &sink, Stop &stop)
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
// 1. speculative walk: a pool of waves (HDRF_WALK_WAVES per SIMD, default 8 = one segment per
//    wave for a 64 x 128 MiB batch) strides over the (block, segment) pairs.  The walk is bound
//    by the scalar unit (one SALU issue per SIMD per 4 cycles), so it wants every wave slot.
__global__ void __launch_bounds__(256) spec_walk_kernel(const BlockDesc *__restrict__ blocks, int nblocks,
                                                        int max_nseg, int w, int maxlen,
                                                        uint32_t *__restrict__ spec, int spec_cap,
                                                        SegMeta *__restrict__ meta)
{
    const int total = nblocks * max_nseg;
    const int nw = gridDim.x * 4;
    for (int t = blockIdx.x * 4 + wave_id(); t < total; t += nw) {
        const int b = t / max_nseg;
        const int k = t - b * max_nseg;
        const BlockDesc bd = blocks[b];
        if (k >= bd.nseg) continue;
        const int size = (int)bd.len;
        const int s_k = k * bd.seg_len;
        const int s_next = (k + 1 == bd.nseg) ? 0x7fffffff : (k + 1) * bd.seg_len;  // last: every cut is main
        WalkCfg W;
        W.base = bd.data; W.avail = (int)min(bd.readable, (uint64_t)0x7fffffff); W.size = size;
        W.w = w; W.maxlen = maxlen;
        ListSink sink;
        const int idx = b * kMaxSegs + k;
        sink.out = spec + (size_t)idx * spec_cap; sink.cap = spec_cap; sink.cnt = 0; sink.stage = 0;
        SpecStop stop{s_next, -1};
        bool ended = walk_chain(W, s_k, k == 0, sink, stop);
        sink.flush();
        const int n_main = stop.n_main < 0 ? sink.cnt : stop.n_main;
        if (lane_id() == 0) {
            SegMeta m;
            m.n_main = n_main; m.n_over = sink.cnt - n_main; m.ended = ended ? 1 : 0; m.pad = 0;
            meta[idx] = m;
        }
    }
}

// 2. sync: one wave per (block, boundary k -> k+1).  sync[idx] = i | j<<16, or -1 END, -2 FAIL.
//    Lane i holds overrun cut O_k[i]; lane j holds segment k+1's cut M_{k+1}[j] (first 64);
//    a lower_bound through ds_bpermute finds whether O_k[i] is one of them.
__global__ void __launch_bounds__(256) spec_sync_kernel(const BlockDesc *__restrict__ blocks,
                                                        const uint32_t *__restrict__ spec, int spec_cap,
                                                        const SegMeta *__restrict__ meta, int32_t *__restrict__ sync)
{
    const int b = blockIdx.y;
    const int k = blockIdx.x * 4 + wave_id();
    const int l = lane_id();
    const BlockDesc bd = blocks[b];
    if (k + 1 >= bd.nseg) return;
    const int idx = b * kMaxSegs + k;
    const SegMeta m0 = meta[idx], m1 = meta[idx + 1];
    const uint32_t *L0 = spec + (size_t)idx * spec_cap;
    const uint32_t *L1 = spec + (size_t)(idx + 1) * spec_cap;
    const int n1 = min(m1.n_main, 64);
    const uint32_t mv = l < n1 ? L1[l] : 0xffffffffu;
    const uint32_t o = l < m0.n_over ? L0[m0.n_main + l] : 0xfffffffeu;
    int pos = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t v = (uint32_t)__shfl((int)mv, pos + step - 1, 64);
        if (v < o) pos += step;
    }
    const uint32_t v = (uint32_t)__shfl((int)mv, pos, 64);
    const bool found = (l < m0.n_over) && pos < n1 && v == o;
    const unsigned long long bal = ballot64(found);
    const int i = bal ? __builtin_ctzll(bal) : 0;
    const int jsel = __shfl(pos, i, 64);
    if (l == 0) sync[idx] = bal ? (i | (jsel << 16)) : (m0.ended ? -1 : -2);
}

// 3a. plan: one 256-thread workgroup per block; thread k handles segment k.
__global__ void __launch_bounds__(256) spec_plan_kernel(const BlockDesc *__restrict__ blocks,
                                                        const uint32_t *__restrict__ spec, int spec_cap,
                                                        const SegMeta *__restrict__ meta, const int32_t *__restrict__ sync,
                                                        SegPlan *__restrict__ plan, BlockState *__restrict__ bst)
{
    __shared__ int s_bad;
    __shared__ uint32_t s_cnt[256];
    const int b = blockIdx.x;
    const int k = threadIdx.x;
    const BlockDesc bd = blocks[b];
    const int nseg = bd.nseg;
    if (k == 0) s_bad = nseg;          // first boundary whose status is not "found"
    __syncthreads();
    const int idx = b * kMaxSegs + k;
    int st = 0;
    if (k + 1 < nseg) {
        st = sync[idx];
        if (st < 0) atomicMin(&s_bad, k);
    }
    __syncthreads();
    const int bad = s_bad;
    int main_begin = 0, main_count = 0, over_count = 0;
    if (k < nseg && k <= bad) {
        const SegMeta m = meta[idx];
        main_begin = (k == 0) ? 0 : ((sync[idx - 1] >> 16) & 0xffff);
        main_count = m.n_main - main_begin;
        if (k + 1 < nseg) over_count = (k == bad) ? m.n_over : (st & 0xffff);
    }
    uint32_t c = (uint32_t)(main_count + over_count);
    s_cnt[k] = c;
    __syncthreads();
    // exclusive scan over 256 entries (Hillis-Steele in LDS)
    for (int d = 1; d < 256; d <<= 1) {
        uint32_t t = k >= d ? s_cnt[k - d] : 0u;
        __syncthreads();
        s_cnt[k] += t;
        __syncthreads();
    }
    const uint32_t incl = s_cnt[k];
    if (k < kMaxSegs) {
        SegPlan p;
        p.main_begin = main_begin; p.main_count = main_count; p.over_count = over_count; p.dst = (int)(incl - c);
        plan[idx] = p;
    }
    if (k == 255) {
        BlockState s;
        s.n_cuts = (int)incl;
        s.fail_dst = -1; s.fail_p0 = 0; s.n_chunks = 0;
        if (bad < nseg - 1 && sync[b * kMaxSegs + bad] == -2) {
            const SegMeta m = meta[b * kMaxSegs + bad];
            s.fail_dst = (int)incl;
            s.fail_p0 = spec[(size_t)(b * kMaxSegs + bad) * spec_cap + m.n_main + m.n_over - 1];
        }
        bst[b] = s;
    }
}

// 3b. copy: one wave per (block, segment): plan piece -> offsets.
__global__ void __launch_bounds__(256) spec_copy_kernel(const BlockDesc *__restrict__ blocks,
                                                        const uint32_t *__restrict__ spec, int spec_cap,
                                                        const SegPlan *__restrict__ plan,
                                                        uint32_t *__restrict__ offsets, int cap_blk)
{
    const int b = blockIdx.y;
    const int k = blockIdx.x * 4 + wave_id();
    if (k >= blocks[b].nseg) return;
    const int idx = b * kMaxSegs + k;
    const SegPlan p = plan[idx];
    const uint32_t *src = spec + (size_t)idx * spec_cap + p.main_begin;
    uint32_t *dst = offsets + (size_t)b * cap_blk + p.dst;
    const int n = p.main_count + p.over_count;
    for (int i = lane_id(); i < n; i += 64) dst[i] = src[i];
}

// 4. fallback + drop-last/append-size: one wave per block.
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
        ListSink sink;
        sink.out = off + s.fail_dst; sink.cap = cap_blk - s.fail_dst; sink.cnt = 0; sink.stage = 0;
        NoStop nostop;
        bool ok = walk_chain(W, (int)s.fail_p0, false, sink, nostop);
        sink.flush();
        if (!ok && lane_id() == 0) atomicOr(err, 1);
        s.n_cuts = s.fail_dst + sink.cnt;
    }
    // :300-304 — drop the last detected cut, append size
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

// ---- host-side launchers (called from api.cpp) -------------------------------------------
namespace hdrf {
hipError_t launch_chunking(const BlockDesc *d_blocks, int nblocks, int max_nseg, int w, int maxlen,
                           uint32_t *spec, int spec_cap, SegMeta *meta, int32_t *sync, SegPlan *plan,
                           BlockState *bst, uint32_t *offsets, int cap_blk, int *err, hipStream_t st, Marker *mk)
{
    mk->mark(st);
    dim3 g((max_nseg + 3) / 4, nblocks);
    static const int per_simd = [] { const char *e = getenv("HDRF_WALK_WAVES"); return e ? atoi(e) : 8; }();
    const int total = nblocks * max_nseg;
    const int nwg = std::max(1, std::min((total + 3) / 4, per_simd * 1024 / 4));
    hipLaunchKernelGGL(spec_walk_kernel, dim3(nwg), dim3(256), 0, st, d_blocks, nblocks, max_nseg, w, maxlen, spec,
                       spec_cap, meta);
    mk->mark(st);
    hipLaunchKernelGGL(spec_sync_kernel, g, dim3(256), 0, st, d_blocks, spec, spec_cap, meta, sync);
    hipLaunchKernelGGL(spec_plan_kernel, dim3(nblocks), dim3(256), 0, st, d_blocks, spec, spec_cap, meta, sync,
                       plan, bst);
    hipLaunchKernelGGL(spec_copy_kernel, g, dim3(256), 0, st, d_blocks, spec, spec_cap, plan, offsets, cap_blk);
    hipLaunchKernelGGL(spec_fallback_kernel, dim3(nblocks), dim3(64), 0, st, d_blocks, w, maxlen, offsets,
                       cap_blk, bst, err);
    return hipGetLastError();
}
}  // namespace hdrf
