// lz4.hip — compression stage (compressor == 2) on gfx950: closed containers -> Lz4Codec files.
//
// Reference: DataDeduplicator.java:748-786 — when a container overflows it is rewritten whole as
// codec.createOutputStream(file).write(prevData || buf); close() with Hadoop's Lz4Codec, i.e.
// BlockCompressorStream framing (MAX_INPUT_SIZE 261,100) around lz4 r123 LZ4_compress blocks
// (hadoop-common 3.1.0 native Lz4Compressor).  tests/ check the output byte for byte against the
// CPU restatement in oracle/; parity vs Hadoop itself is unpinned.
//
// Every 261,100-B segment is an independent LZ4 block with a fresh hash table, so one wave owns
// one segment (table in LDS).  The greedy parse is sequential, but its expensive parts are made
// wave-parallel:
//   * match search: the positions the search loop visits do not depend on the data until a match
//     is found (ip += attempts++ >> 6), so a batch of 16, 32, then 64 attempts is evaluated at once
//     (lane i = attempt i, positions in closed form): hashes and the 4-byte candidate compare are
//     one gather each.  When the batch's hashes are distinct the table update is one LDS gather +
//     one scatter (attempts after the first match restore the old entry); otherwise the reads and
//     writes are replayed lane by lane in attempt order and the writes after the match undone;
//   * match extension, catch-up and literal copies are 64-lane compares / 16-B-per-lane copies.
//   lz4_pack then frames the segments ([BE32 len] ([BE32 clen] block)* [BE32 0]) in place.
#include <algorithm>
#include <cstdlib>

#include "bytes.hpp"

namespace hdrf {

constexpr int kLzMaxIn = 261100;                 // BlockCompressorStream MAX_INPUT_SIZE (256 KiB buffer)
constexpr int kLzSegBound = kLzMaxIn + kLzMaxIn / 255 + 16;
constexpr int kLzSegStride = kLzSegBound + 4;    // per-segment stride of the unpacked layout
constexpr int kMfLimit = 12, kLastLit = 5, kMaxDist = 65535, k64KLimit = 65536 + kMfLimit - 1;
constexpr int kLzFirstBatch = 8;                 // attempts per batch after a match (then 16, 32, 64)
// Bytes of one lane window (forward, reference, search, candidate): 4 per lane over kLzWin / 4
// lanes; with 128 the upper 32 lanes load the lower 32 lanes' words again (no extra line
// requests) and take no part in the compares.  HDRF_LZ4_WIN (A/B builds): 256 or 128.
#ifndef HDRF_LZ4_WIN
#define HDRF_LZ4_WIN 256
#endif
constexpr int kLzWin = HDRF_LZ4_WIN;
constexpr int kLzWinLanes = kLzWin / 4;
static_assert(kLzWin == 256 || kLzWin == 128, "LZ4 window: 256 or 128 bytes");

// length >= 15 continuation bytes (255 ... rest); returns the new output offset
__device__ __forceinline__ int put_len(uint8_t *out, int op, int len)
{
    const int n255 = len / 255;
    const int l = lane_id();
    for (int k = l; k < n255; k += 64) wr8(out + op + k, 255);
    if (l == 0) wr8(out + op + n255, (uint32_t)(len - 255 * n255));
    return op + n255 + 1;
}

// LDS of one wave's hash table.  byU16 (blocks < 64 KiB + 11): 8192 u16 entries (16 KiB) + a 2-bit
// tag per entry (2 KiB).  byU32 (larger blocks, <= 262,144 B): 4096 positions < 2^18 kept as a u16
// low half (8 KiB) + a 4-bit nibble per entry (2 KiB, 8 per dword, updated with LDS atomics): bits
// 0-1 the position's bits 16-17, bits 2-3 the tag.  10 KiB: 16 compressing waves per CU (the VGPR
// limit) fill the CU's 160 KiB.
// The tag is two bits of the hash product just below the table index bits: a function of the
// entry's 4-byte value, so a candidate whose tag differs from the tag of the bytes being matched
// cannot match (the sequential code's 4-byte compare fails) and is rejected without loading its
// bytes; only tag hits (true matches and 1 in 4 of the false candidates) pay the dependent global
// round trip (tools: a CPU count of the parse on the config-4 corpus finds 23 % (text) and 57 %
// (binary records) of the chain candidates false).
constexpr int kLzTabU16 = 16384 + 2048;
constexpr int kLzTabU32 = 8192 + 2048;

#ifdef HDRF_LZ4_PROF
// profiling build only (scripts/r02_lzp.sh): shader-clock time per parse phase, summed over waves
__device__ unsigned long long g_lzprof[16];
#define LZP_INIT uint64_t lzp_t = __builtin_amdgcn_s_memtime(); uint64_t lzp_a[8] = {0, 0, 0, 0, 0, 0, 0, 0}; uint32_t lzp_n[4] = {0, 0, 0, 0};
#define LZP(i) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); lzp_a[i] += t_ - lzp_t; lzp_t = t_; }
#define LZN(i) (lzp_n[i]++)
#define LZP_FLUSH if (lane_id() == 0) { for (int i_ = 0; i_ < 8; i_++) atomicAdd(&g_lzprof[i_], (unsigned long long)lzp_a[i_]); \
                                        for (int i_ = 0; i_ < 4; i_++) atomicAdd(&g_lzprof[8 + i_], (unsigned long long)lzp_n[i_]); }
#else
#define LZP_INIT
#define LZP(i)
#define LZN(i)
#define LZP_FLUSH
#endif

// One LZ4 block (lz4 r123 LZ4_compress, noDict): returns the compressed size.  Uniform control
// flow; `tabmem` is this wave's LDS hash table (layout above).
__device__ __forceinline__ int lz4_block(const uint8_t *src, int n, uint8_t *out, uint8_t *tabmem)
{
    const int l = lane_id();
    const bool u16 = n < k64KLimit;
    const int hshift = u16 ? 32 - 13 : 32 - 12;
    unsigned short *tab16 = (unsigned short *)tabmem;   // byU16 entries, or the byU32 low halves
    uint32_t *tabx = (uint32_t *)(tabmem + (u16 ? 16384 : 8192));   // byU16: 2-bit tags; byU32: nibbles
    auto hash = [&](uint32_t v) -> uint32_t { return (v * 2654435761u) >> hshift; };
    auto tagof = [&](uint32_t v) -> uint32_t { return ((v * 2654435761u) >> (hshift - 2)) & 3u; };
    {
        // every entry starts at position 0 (the zeroed table of LZ4_compress) with the tag of the
        // bytes there
        const uint32_t t0 = n >= 4 ? tagof(rd32u(src)) : 0u;
        const uint32_t xw = u16 ? t0 * 0x55555555u : (t0 << 2) * 0x11111111u;
        uint32_t *t32 = (uint32_t *)tabmem;
        const int nw0 = (u16 ? 16384 : 8192) / 4, nw = (u16 ? kLzTabU16 : kLzTabU32) / 4;
        for (int i = l; i < nw; i += 64) t32[i] = i < nw0 ? 0u : xw;
    }
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("" ::: "memory");
    auto xupd = [&](uint32_t h, int p, uint32_t tg) -> uint32_t {   // old nibble / tag field, then p, tg
        if (u16) {
            const uint32_t sh = 2 * (h & 15);
            const uint32_t cur = (tabx[h >> 4] >> sh) & 3u;
            atomicXor(&tabx[h >> 4], (cur ^ tg) << sh);   // lanes share words; unconditional (no
            return cur;                                    // exec-mask branch on the chain)
        }
        const uint32_t sh = 4 * (h & 7);
        const uint32_t cur = (tabx[h >> 3] >> sh) & 15u, want = (((uint32_t)p >> 16) & 3u) | (tg << 2);
        atomicXor(&tabx[h >> 3], (cur ^ want) << sh);
        return cur;
    };
    auto tput = [&](uint32_t h, int p, uint32_t tg) {   // no read of the entry: two non-returning
        tab16[h] = (unsigned short)p;                    // LDS atomics clear and set its field (lanes
        if (u16) {                                       // of one wave touch disjoint fields)
            const uint32_t sh = 2 * (h & 15);
            atomicAnd(&tabx[h >> 4], ~(3u << sh));
            atomicOr(&tabx[h >> 4], tg << sh);
        } else {
            const uint32_t sh = 4 * (h & 7);
            atomicAnd(&tabx[h >> 3], ~(15u << sh));
            atomicOr(&tabx[h >> 3], ((((uint32_t)p >> 16) & 3u) | (tg << 2)) << sh);
        }
    };
    auto tswap = [&](uint32_t h, int p, uint32_t tg, uint32_t &otg) -> int {   // old entry, then (p, tg)
        const int lo = (int)tab16[h];
        tab16[h] = (unsigned short)p;
        const uint32_t cur = xupd(h, p, tg);
        if (u16) { otg = cur; return lo; }
        otg = cur >> 2;
        return lo | (int)((cur & 3u) << 16);
    };

    const int mflimit = n - kMfLimit, matchlimit = n - kLastLit;
    int op = 0, anchor = 0, ip = 0;
    LZP_INIT
    if (n >= kMfLimit + 1) {
        if (l == 0) { const uint32_t v0 = rd32u(src); tput(hash(v0), 0, tagof(v0)); }   // first byte
        ip = 1;
        int fip = ip, attempts = (1 << 6) + 3, m = kLzFirstBatch;
        // Windows: lane l holds the 4 bytes at wb + 4l (forward) and at wb + dr + 4l (the
        // reference, dr = mref - ip during a match).  A verified candidate arrives with both
        // windows already loaded (its check loaded them), so a match chain costs one global round
        // trip per sequence: the candidate bytes and the next forward bytes together.  The search
        // takes its attempt words from a forward window (Sw at sb) when the batch fits in it, and a
        // match found by the search loads one window pair 64 bytes before the match that serves
        // the catch-up, the literals (<= 64 bytes) and the first extension step at once.
        // lane word at src + at + 4l, for at >= 0 (every caller: the fast catch-up below takes its
        // windows only when both start at or after byte 0).  A lane reaching past byte n - 4 reads
        // the last word instead; no such lane's bytes are ever used (every use is bounded by
        // mflimit / matchlimit, at least 5 bytes before n), so one clamp replaces the guards.
        const int nm4 = n - 4;
        const int lw = kLzWinLanes == 64 ? l : (l & (kLzWinLanes - 1));   // this lane's word of a window
        auto wload = [&](int at) -> uint32_t { return ld32u(src, (uint32_t)min(at + 4 * lw, nm4)); };
        auto lane_word = [&](uint32_t w, int o) -> uint32_t {   // bytes [o, o + 4) of a window
            const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((o >> 2) << 2, (int)w);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(((o >> 2) + 1) << 2, (int)w);
            return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(o & 3));
        };
        uint32_t Fw = 0, Rw = 0, Sw = 0;
        // sb: the search window Sw's base; far below every position while Sw holds nothing, so one
        // unsigned compare tests "the batch lies in the window"
        int hwb = 0, sb = -(1 << 30);
        // one exit, at the loop condition (as the chain loop below): the compiler keeps the parse
        // a plain loop nest instead of a dispatch over exit states
        for (bool more = true; more;) {
            // ---- match search: a batch of m attempts at once ------------------------------
            // attempt l advances by step_l = (a0 + l) >> 6, which takes only the values q and
            // q + 1 inside one batch, so the attempt positions have a closed form (no scan)
            fip = (int)rdfirst((uint32_t)fip); attempts = (int)rdfirst((uint32_t)attempts); m = (int)rdfirst((uint32_t)m);
            op = (int)rdfirst((uint32_t)op); anchor = (int)rdfirst((uint32_t)anchor); sb = (int)rdfirst((uint32_t)sb);
            const int a0 = attempts;
            const int q = a0 >> 6, rr = a0 & 63;
            const int step = q + (l >= 64 - rr ? 1 : 0);
            const int ipl = fip + l * q + max(0, l - (64 - rr));       // this lane's attempt
            const bool valid = l < m && ipl + step <= mflimit;
            const int last_at = fip + (m - 1) * q + max(0, m - 1 - (64 - rr));   // lane m-1's attempt
            bool inwin = (uint32_t)(last_at - sb) <= (uint32_t)(kLzWin - 5);     // (fip >= sb: last_at >= fip)
            if (!inwin && last_at - fip <= kLzWin - 5) { Sw = wload(fip); sb = fip; inwin = true; }
            const uint32_t vw = lane_word(Sw, (valid && inwin) ? ipl - sb : 0);
            const uint32_t v = !valid ? 0u : inwin ? vw : ld32u(src, (uint32_t)ipl);
            const uint32_t h = hash(v);
            const unsigned long long vmask = ballot64(valid);
            const int nv = vmask == ~0ull ? 64 : __builtin_ctzll(~vmask);   // valid lanes are a prefix
            // Table replay in attempt order, in parallel.  Distinct hashes (the common case): every
            // attempt reads the pre-batch entry and the writes commute — checked by scattering lane
            // tags into the entries and reading them back.  Equal hashes: attempt i reads the
            // position of the last earlier attempt with its hash (else the pre-batch entry), found
            // with one ballot per hash bit; each hash keeps its last attempt up to the first match.
            // The entry's two reads, the lane-id scatter and its read-back issue back to back (LDS
            // keeps a wave's operations in order) and are decoded after one round trip.
            const uint32_t vt = tagof(v);
            uint32_t r16 = 0, rx = 0, tg = 0;
            if (valid) {
                r16 = tab16[h];
                rx = tabx[u16 ? h >> 4 : h >> 3];
                asm volatile("" ::: "memory");
                tab16[h] = (unsigned short)l;
                asm volatile("" ::: "memory");
                tg = tab16[h];
            }
            int old;
            uint32_t otg;
            if (u16) {
                otg = (rx >> (2 * (h & 15))) & 3u;
                old = (int)r16;
            } else {
                const uint32_t nb = (rx >> (4 * (h & 7))) & 15u;
                otg = nb >> 2;
                old = (int)r16 | (int)((nb & 3u) << 16);
            }
            const bool collide = ballot64(valid && tg != (uint32_t)l) != 0;
            asm volatile("" ::: "memory");
            if (valid) tab16[h] = (unsigned short)old;     // (the high parts and tags were not touched)
            asm volatile("" ::: "memory");
            unsigned long long eq = 0;
            int ref = old;
            // the candidate's bytes: an earlier attempt of this batch is this wave's own value (no
            // load); a table entry whose tag differs from v's cannot hold v (no load); else load
            bool known = false;
            uint32_t cv = ~v;
            if (collide) {
                eq = vmask;
#pragma unroll
                for (int b = 0; b < 13; b++) {             // byU32: 12-bit hashes (bit 12 is 0)
                    const bool hb = (h >> b) & 1u;
                    const unsigned long long mb = ballot64(valid && hb);
                    eq &= hb ? mb : ~mb;
                }
                const unsigned long long below = eq & ((1ull << l) - 1ull);
                const int prev = below ? 63 - __builtin_clzll(below) : l;
                const int pipl = __builtin_amdgcn_ds_bpermute(prev << 2, ipl);
                const uint32_t pv = (uint32_t)__builtin_amdgcn_ds_bpermute(prev << 2, (int)v);
                if (below) { ref = pipl; cv = pv; known = true; }
            }
            const bool in = valid && ref + kMaxDist >= ipl;
            if (in && !known && otg == vt) cv = ld32u(src, (uint32_t)ref);   // ref is a position < n
            const bool ok = in && cv == v;
            const unsigned long long okm = ballot64(ok);
            LZN(0);
            {                                             // commit: attempts up to the first match
                const int last = okm ? __builtin_ctzll(okm) : 63;
                const unsigned long long upto = last == 63 ? ~0ull : ((2ull << last) - 1ull);
                const unsigned long long later = (l == 63 || !collide) ? 0ull : (eq & upto & (~0ull << (l + 1)));
                if (valid && l <= last && !later) tput(h, ipl, vt);
                asm volatile("" ::: "memory");
            }
            LZP(0);
            if (okm) {
                LZN(1);
                const int istar = __builtin_ctzll(okm);
                asm volatile("" ::: "memory");
                ip = (int)rdlane((uint32_t)ipl, istar);
                int mref = (int)rdlane((uint32_t)ref, istar);
                int tpos;
                uint32_t tok;
                const bool fast = ip - anchor <= 64 && ip >= 64 && mref >= 64;
                int plit = 0, plito = 0;                   // fast path: literals stored with the token
                uint32_t plitv = 0;
                // one window pair at ip - 64 (fast case): catch-up, literals and the first extension
                // step; hstop = the highest stop byte in [wb0, ip) (lanes 0-15): a byte that differs,
                // or one before the anchor or before the segment start on the reference side (bytes
                // j < lo of the lane's word) — one ballot, then the top stop byte of the top lane.
                // No stop byte (64 equal bytes) or not fast: the general catch-up.  (One if / else
                // on hstop, not two ifs on a flag.)
                const int wb0 = ip - 64, d0 = mref - ip;
                int hstop = -1;
                if (fast) {
                    Fw = wload(wb0);
                    Rw = wload(wb0 + d0);
                    uint32_t sx = Fw ^ Rw;
                    {
                        const int p0 = wb0 + 4 * l, lo = max(anchor - p0, -(p0 + d0));
                        if (lo > 0) sx |= lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
                    }
                    const unsigned long long bm = ballot64(l < 16 && sx != 0u);
                    if (bm) {
                        const int L = 63 - __builtin_clzll(bm);
                        hstop = 4 * L + ((31 - __builtin_clz(rdlane(sx, L))) >> 3);
                    }
                }
                if (hstop >= 0) {
                    const int back = 63 - hstop;
                    ip -= back; mref -= back;
                    tpos = op++;
                    const int lit = ip - anchor;
                    if (lit >= 15) { tok = 15u << 4; op = put_len(out, op, lit - 15); }
                    else tok = (uint32_t)lit << 4;
                    const int o = anchor + l - wb0;        // literal byte l from the window
                    const uint32_t wv = (uint32_t)__builtin_amdgcn_ds_bpermute(((o >> 2) & 63) << 2, (int)Fw);
                    plitv = wv >> (8 * (o & 3)); plit = lit; plito = op;
                    op += lit;
                    hwb = wb0;
                } else {
                    // ---- catch up ------------------------------------------------------
                    int back;
                    do {
                        const int k = l + 1;
                        const bool c = ip - k >= anchor && mref - k >= 0 && rd8(src + ip - k) == rd8(src + mref - k);
                        const unsigned long long bad = ballot64(!c);
                        back = bad ? __builtin_ctzll(bad) : 64;
                        ip -= back; mref -= back;
                    } while (back == 64);
                    // ---- literals ------------------------------------------------------
                    tpos = op++;
                    const int lit = ip - anchor;
                    if (lit >= 15) { tok = 15u << 4; op = put_len(out, op, lit - 15); }
                    else tok = (uint32_t)lit << 4;
                    wave_copy(out + op, src + anchor, lit);
                    op += lit;
                    Fw = wload(ip);                        // the window pair at the match
                    Rw = wload(mref);
                    hwb = ip;
                }
                LZP(1);
                // _next_match: one sequence per iteration, a single exit at the loop condition (the
                // compiler then keeps the chain a plain loop instead of a dispatch over exit states)
                bool fin = false;                          // the match reached mflimit: last literals
                for (bool chain = true; chain;) {
                    // the parse state is wave-uniform: keep it in scalar registers so the
                    // branches on it are scalar branches, not exec-mask regions
                    ip = (int)rdfirst((uint32_t)ip); mref = (int)rdfirst((uint32_t)mref);
                    op = (int)rdfirst((uint32_t)op); anchor = (int)rdfirst((uint32_t)anchor);
                    tpos = (int)rdfirst((uint32_t)tpos); tok = rdfirst(tok); hwb = (int)rdfirst((uint32_t)hwb);
                    // the offset is stored with the token after the extension: a store in flight here
                    // would be waited for by the window reads' vmcnt waits (gfx9 counts stores in vmcnt)
                    const int opo = op;
                    const uint32_t offv = (uint32_t)(ip - mref);
                    op += 2;
                    const int dr = mref - ip;
                    // the window pair (Fw, Rw) starts at hwb <= ip; lanes below l0 hold the minmatch
                    // (and the bytes before it)
                    int wb = hwb, l0 = (ip + 4 - hwb) >> 2;
                    anchor = ip + 4;
                    // match extension: the next window pair is loaded at the top of an iteration, so
                    // the loop's exit has waited for the pair it compared (no window load is still
                    // pending after it, so the reads of Fw below do not wait for the sequence's stores)
                    uint32_t x;
                    unsigned long long mm;
                    bool next = false;
                    do {
                        if (next) { wb += kLzWin; l0 = 0; Fw = wload(wb); Rw = wload(wb + dr); }
                        x = Fw ^ Rw;
                        if (wb + kLzWin > matchlimit) {    // (uniform) the window reaches matchlimit:
                            const int p = wb + 4 * l;      // a lane past it stops (x made non-zero
                            if (p + 4 > matchlimit)        // from the first byte at matchlimit on)
                                x = p < matchlimit ? x | (0xffffffffu << (8 * (matchlimit - p))) : 0xffffffffu;
                        }
                        if (l < l0 || (kLzWinLanes < 64 && l >= kLzWinLanes)) x = 0u;   // (256: the round-5 code)
                        mm = ballot64(x != 0u);
                        next = true;
                    } while (!mm);
                    {
                        const int L = __builtin_ctzll(mm);
                        const uint32_t xl = rdlane(x, L);
                        ip = wb + 4 * L + (xl ? (__builtin_ctz(xl) >> 3) : 4);
                        mref = ip + dr;
                    }
                    LZP(2);
                    const uint32_t Nw = wload(ip);        // the next position's window: in flight
                    int ml = ip - anchor;                 // under the stores and the table update
                    if (ml >= 15) {
                        tok += 15;
                        ml -= 15;
                        const int n510 = ml > 509 ? (ml - 510) / 510 + 1 : 0;   // pairs of 255
                        for (int k = l; k < 2 * n510; k += 64) wr8(out + op + k, 255);
                        op += 2 * n510;
                        ml -= 510 * n510;
                        if (ml >= 255) { wr8(out + op, 255); op++; ml -= 255; }
                        wr8(out + op, (uint32_t)ml);
                        op++;
                    } else {
                        tok += (uint32_t)ml;
                    }
                    // the sequence's token, offset and (fast path) literal bytes: uniform bytes at
                    // uniform addresses, stored by every lane (one coalesced write, no exec-mask
                    // region on the chain)
                    wr8(out + (uint32_t)tpos, tok); wr8(out + (uint32_t)opo, offv); wr8(out + (uint32_t)opo + 1, offv >> 8);
                    if (plit) { if (l < plit) wr8(out + plito + l, plitv); plit = 0; }
                    chain = false;
                    if (ip > mflimit) {
                        fin = true;
                    } else {
                        // fill table; test next position (its bytes are in the forward window unless
                        // the match ended right at a window start)
                        const int o2 = ip - 2 - wb;
                        uint32_t v2, v0;
                        if ((uint32_t)o2 <= (uint32_t)(kLzWin - 7)) {   // o2 >= 0, lane (o2 + 2) / 4 + 1 < kLzWinLanes
                            // three lanes of the window into scalar registers, the two words by 64-bit
                            // scalar shifts (the hashes below stay scalar too: no VALU round trip)
                            const int a2 = o2 >> 2, a0 = (o2 + 2) >> 2;
                            const uint64_t pA = ((uint64_t)rdlane(Fw, a2 + 1) << 32) | rdlane(Fw, a2);
                            const uint64_t pB = a0 == a2 ? pA : ((uint64_t)rdlane(Fw, a0 + 1) << 32) | (pA >> 32);
                            v2 = (uint32_t)(pA >> (8 * (o2 & 3)));
                            v0 = (uint32_t)(pB >> (8 * ((o2 + 2) & 3)));
                        } else {
                            v2 = rdfirst(ld32u(src, (uint32_t)(ip - 2)));
                            v0 = rdfirst(ld32u(src, (uint32_t)ip));
                        }
                        // table: [h2] = ip - 2, r = [h0], [h0] = ip.  Distinct hashes: lanes 0 and 1
                        // do the two slots in one pass; equal hashes: r is ip - 2.
                        const uint32_t h2 = hash(v2), h0 = hash(v0), t2 = tagof(v2), t0 = tagof(v0);
                        int r = 0;
                        uint32_t rt = 0;
                        asm volatile("" ::: "memory");
                        if (h2 == h0) {
                            if (l == 0) tput(h0, ip, t0);
                            r = ip - 2;
                            rt = t2;
                        } else {
                            uint32_t ot = 0;
                            if (l < 2) r = tswap(l == 0 ? h2 : h0, l == 0 ? ip - 2 : ip, l == 0 ? t2 : t0, ot);
                            r = (int)rdlane((uint32_t)r, 1);
                            rt = rdlane(ot, 1);
                        }
                        asm volatile("" ::: "memory");
                        LZP(3);
                        const bool near = r + kMaxDist >= ip;
                        uint32_t Cw = 0;
                        if (near && rt == t0) {            // a tag miss cannot chain: no load
                            Cw = wload(r);                 // one round trip
                            chain = rdlane(Cw, 0) == v0;
                        }
                        LZP(4);
                        if (chain) {
                            LZN(2);
                            mref = r;
                            tpos = op++;
                            tok = 0;
                            Fw = Nw; Rw = Cw; hwb = ip;
                        } else if (near) {
                            Sw = Nw; sb = ip;              // the search after the break starts in it
                        }
                    }
                }
                if (fin) {                                 // last literals
                    anchor = ip;
                    more = false;
                } else {
                    anchor = ip++;
                    fip = ip;
                    attempts = (1 << 6) + 3;
                    m = kLzFirstBatch;
                }
            } else if (nv < m) {
                more = false;                              // the next attempt passes mflimit
            } else {
                fip = (int)rdlane((uint32_t)(ipl + step), m - 1);
                attempts = a0 + m;
                m = min(64, 2 * m);
            }
        }
    }

    LZP(5);
    {
        int run = n - anchor;
        const int tpos = op++;
        if (run >= 15) {
            if (l == 0) wr8(out + tpos, 15u << 4);
            op = put_len(out, op, run - 15);
        } else if (l == 0) {
            wr8(out + tpos, (uint32_t)run << 4);
        }
        wave_copy(out + op, src + anchor, run);
        op += run;
    }
    LZP(6);
    LZP_FLUSH
    return op;
}


// 64 threads per segment.  Two instances: byU32 segments with the 9 KiB table (every 261,100-B
// segment) and byU16 ones with 16 KiB (a container's short last segment); each skips the other
// kind.  Persistent: a fixed grid of waves takes (container, segment) items from a per-batch
// counter (items of the byU16 instance: one per container), so the pass never dispatches the
// empty workgroups of a (nseg_max, closed_cap) grid, and the grid can leave wave slots free on
// every CU: with HDRF_LZ4_WAVES = 16 per CU (of the 17 the LDS table allows), the next batch's
// SHA and chunking kernels get a slot per SIMD while this pass runs, so the next pass is ready
// when this one drains (otherwise SHA waited for the pass's waves to retire: one pass at a time).
template <bool kSmall>
__device__ __forceinline__ void lz4_seg_body(const ClosedRec *__restrict__ closed,
                                             const uint32_t *__restrict__ nclosed, const uint8_t *__restrict__ arena,
                                             uint64_t cmax, uint8_t *__restrict__ carena, uint64_t cslot,
                                             uint32_t *__restrict__ seg_clen, int nseg_max, uint32_t *__restrict__ work,
                                             uint8_t *tabmem, int prio)
{
    if (prio) __builtin_amdgcn_s_setprio(3);                 // HDRF_SETPRIO bit 6
    const uint32_t nc = *nclosed;
    const uint32_t per = kSmall ? 1u : (uint32_t)nseg_max;
    const uint32_t total = nc * per;
    for (;;) {
        uint32_t item = 0;
        if (lane_id() == 0) item = atomicAdd(work, 1u);
        item = rdfirst(item);
        if (item >= total) break;                             // every wave reaches this exit
        const int c = (int)(item / per);
        const ClosedRec r = closed[c];
        const int s = kSmall ? (r.len ? (int)((r.len - 1) / kLzMaxIn) : 0) : (int)(item % per);
        const int64_t off = (int64_t)s * kLzMaxIn;
        if (off >= (int64_t)r.len) continue;
        const int n = (int)min((int64_t)kLzMaxIn, (int64_t)r.len - off);
        if ((n < k64KLimit) != kSmall) continue;
        const uint8_t *src = arena + (size_t)r.slot * cmax + off;
        uint8_t *out = carena + (size_t)r.slot * cslot + 8 + (size_t)s * kLzSegStride;
        const int cl = lz4_block(src, n, out, tabmem);
        if (lane_id() == 0) seg_clen[(size_t)c * nseg_max + s] = (uint32_t)cl;
        __builtin_amdgcn_s_waitcnt(0);                        // the table is reused by the next item
        asm volatile("" ::: "memory");
    }
}

template <bool kSmall>
__global__ void __launch_bounds__(64) lz4_seg_kernel(const ClosedRec *__restrict__ closed,
                                                     const uint32_t *__restrict__ nclosed, const uint8_t *__restrict__ arena,
                                                     uint64_t cmax, uint8_t *__restrict__ carena, uint64_t cslot,
                                                     uint32_t *__restrict__ seg_clen, int nseg_max, uint32_t *__restrict__ work,
                                                     int prio)
{
    __shared__ __attribute__((aligned(16))) uint8_t tabmem[kSmall ? kLzTabU16 : kLzTabU32];
    lz4_seg_body<kSmall>(closed, nclosed, arena, cmax, carena, cslot, seg_clen, nseg_max, work, tabmem, prio);
}

// grid nclosed x 256 threads: frame the segments in place, [BE32 len] ([BE32 clen] block)* [BE32 0].
// Every segment moves to a lower (or equal) offset, so tiles copied in order — all loads of a tile
// before any of its stores — never overwrite bytes not yet read.  A tile is 16 KiB (four 16-B
// words per thread, source realigned with load16_shift, destination 16-B aligned after a head).
__global__ void __launch_bounds__(256) lz4_pack_kernel(const ClosedRec *__restrict__ closed,
                                                       const uint32_t *__restrict__ nclosed, uint8_t *__restrict__ carena,
                                                       uint64_t cslot, const uint32_t *__restrict__ seg_clen, int nseg_max,
                                                       uint32_t *__restrict__ file_len)
{
    const int c = blockIdx.x, t = threadIdx.x;
    if ((uint32_t)c >= *nclosed) return;
    const ClosedRec r = closed[c];
    uint8_t *base = carena + (size_t)r.slot * cslot;
    const int nseg = r.len ? (int)((r.len + kLzMaxIn - 1) / kLzMaxIn) : 0;
    if (t == 0) put_be32(base, r.len);
    uint32_t pos = 4;
    for (int s = 0; s < nseg; s++) {
        const uint32_t cl = seg_clen[(size_t)c * nseg_max + s];
        const uint32_t from = 8 + (uint32_t)s * kLzSegStride;
        const uint32_t to = pos + 4;
        if (to != from && cl) {
            uint8_t *dst = base + to;
            const uint8_t *src = base + from;
            uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
            if (head > cl) head = cl;
            const uint8_t hb = (uint32_t)t < head ? src[t] : 0;
            __syncthreads();
            if ((uint32_t)t < head) dst[t] = hb;
            const uint32_t n16 = (cl - head) >> 4;
            const uint8_t *sp = src + head;
            const int sh = (int)((uintptr_t)sp & 15);
            const uint8_t *sa = sp - sh;
            uint8_t *d = dst + head;
            for (uint32_t w0 = 0; w0 < n16; w0 += 1024) {
                uint4 v[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t w = w0 + 256 * k + t;
                    v[k] = w < n16 ? load16_shift(sa + 16 * (size_t)w, sh) : make_uint4(0, 0, 0, 0);
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t w = w0 + 256 * k + t;
                    if (w < n16) st16(d + 16 * (size_t)w, v[k]);
                }
                __syncthreads();
            }
            const uint32_t tb = head + 16 * n16;
            const uint8_t tv = tb + t < cl ? src[tb + t] : 0;
            __syncthreads();
            if (tb + t < cl) dst[tb + t] = tv;
        }
        if (t == 0) put_be32(base + pos, cl);
        __syncthreads();
        pos = to + cl;
    }
    if (r.len > (uint32_t)kLzMaxIn) {                      // segmented write: close() trailer
        if (t == 0) put_be32(base + pos, 0);
        pos += 4;
    }
    if (r.len == 0) pos = 4;
    if (t == 0) file_len[c] = pos;
}

#ifdef HDRF_LZ4_PROF
extern "C" int hdrf_debug_lz4_prof(unsigned long long *out16, int reset)
{
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_lzprof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_lzprof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

uint64_t lz4_slot_bytes(uint32_t cmax)
{
    const uint64_t nseg = (cmax + kLzMaxIn - 1) / kLzMaxIn + 1;
    return 16 + nseg * (uint64_t)kLzSegStride;
}

// ---- stream mode (compressor 4): arbitrary pieces of one block -----------------------------
// grid n x 64: piece i of the block -> LZ4 block at stage + i * kLzSegStride, size -> clen[i]
__global__ void __launch_bounds__(64) lz4_list_kernel(const LzPiece *__restrict__ pieces, int n,
                                                      const uint8_t *__restrict__ base, uint8_t *__restrict__ stage,
                                                      uint32_t *__restrict__ clen)
{
    __shared__ __attribute__((aligned(16))) uint8_t tabmem[kLzTabU16];
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzPiece pc = pieces[i];
    const int c = lz4_block(base + pc.src, (int)pc.len, stage + (size_t)i * kLzSegStride, tabmem);
    if (lane_id() == 0) clen[i] = (uint32_t)c;
}

// grid n x 256: piece i -> file at its offset: [BE32 hval if hlen] [BE32 clen] [block]
__global__ void __launch_bounds__(256) lz4_emit_kernel(const LzOut *__restrict__ outs, int n,
                                                       const uint8_t *__restrict__ stage,
                                                       const uint32_t *__restrict__ clen, uint8_t *__restrict__ file)
{
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzOut o = outs[i];
    uint8_t *p = file + o.dst;
    const int c = (int)clen[i];
    if (threadIdx.x == 0) {
        if (o.hlen) put_be32(p, o.hval);
        put_be32(p + o.hlen, (uint32_t)c);
    }
    // four waves copy four quarters of the block
    const int w = wave_id(), q = (c + 3) / 4;
    const int a = min(c, w * q), b = min(c, a + q);
    if (b > a) wave_copy(p + o.hlen + 4 + a, stage + (size_t)i * kLzSegStride + a, b - a);
}

// ---- decoder (read side: DataConstructor's Lz4Codec input stream, DN/DataConstructor.java:
//      171-176,495-500): one wave per LZ4 block.  The sequence headers are parsed from an 8 KiB
//      LDS window of the compressed stream (refilled with coalesced loads), literals and matches
//      are wave-wide copies; a match may read output written moments before, so each match is
//      preceded by a fence.  Malformed input (bounds, zero offset, wrong decoded size) sets *err.
constexpr int kDecWin = 8192;

__global__ void __launch_bounds__(64) lz4_decode_kernel(const LzDec *__restrict__ items, int n,
                                                        const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                        int *__restrict__ err)
{
    __shared__ uint8_t win[kDecWin];
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzDec d = items[i];
    const uint8_t *in = src + d.src;
    uint8_t *out = dst + d.dst;
    const int64_t iend = d.clen, oend = d.rawlen;
    const int l = lane_id();
    int64_t wbase = -kDecWin;                            // window covers in[wbase, wbase + kDecWin)
    auto byte = [&](int64_t pos) -> uint32_t {          // wave-uniform pos < iend
        if (pos >= wbase + kDecWin) {
            wbase = pos & ~(int64_t)15;
            __builtin_amdgcn_s_waitcnt(0);
            asm volatile("" ::: "memory");
            for (int k = l * 16; k < kDecWin; k += 64 * 16) {
                const int64_t g = wbase + k;
                for (int b = 0; b < 16; b++) win[k + b] = g + b < iend ? rd8(in + g + b) : 0u;
            }
            __builtin_amdgcn_s_waitcnt(0);
            asm volatile("" ::: "memory");
        }
        return win[pos - wbase];
    };
    int64_t ip = 0, op = 0;
    bool bad = false;
    for (;;) {
        if (ip >= iend) { bad = true; break; }
        const uint32_t token = byte(ip++);
        int64_t lit = token >> 4;
        if (lit == 15) {
            uint32_t b;
            do {
                if (ip >= iend) { bad = true; break; }
                b = byte(ip++);
                lit += b;
            } while (b == 255);
            if (bad) break;
        }
        if (ip + lit > iend || op + lit > oend) { bad = true; break; }
        wave_copy(out + op, in + ip, (int)lit);
        ip += lit;
        op += lit;
        if (ip == iend) break;                           // the last sequence has literals only
        if (ip + 2 > iend) { bad = true; break; }
        const int64_t off = (int64_t)byte(ip) | ((int64_t)byte(ip + 1) << 8);
        ip += 2;
        int64_t ml = token & 15;
        if (ml == 15) {
            uint32_t b;
            do {
                if (ip >= iend) { bad = true; break; }
                b = byte(ip++);
                ml += b;
            } while (b == 255);
            if (bad) break;
        }
        ml += 4;
        if (off == 0 || off > op || op + ml > oend) { bad = true; break; }
        __threadfence();
        if (off >= ml) {
            wave_copy(out + op, out + op - off, (int)ml);
        } else {                                         // overlapping: the last `off` bytes repeat
            for (int64_t k = l; k < ml; k += 64) wr8(out + op + k, rd8(out + op - off + (k % off)));
        }
        __threadfence();
        op += ml;
    }
    if ((bad || op != oend) && l == 0) atomicOr(err, 1);
}

hipError_t launch_lz4_decode(const LzDec *items, int n, const uint8_t *src, uint8_t *dst, int *err, hipStream_t st)
{
    if (n > 0) hipLaunchKernelGGL(lz4_decode_kernel, dim3(n), dim3(64), 0, st, items, n, src, dst, err);
    return hipGetLastError();
}

hipError_t launch_lz4_stream(const LzPiece *pieces, int n, const uint8_t *base, uint8_t *stage, uint32_t *clen,
                             hipStream_t st)
{
    if (n > 0) hipLaunchKernelGGL(lz4_list_kernel, dim3(n), dim3(64), 0, st, pieces, n, base, stage, clen);
    return hipGetLastError();
}

hipError_t launch_lz4_emit(const LzOut *outs, int n, const uint8_t *stage, const uint32_t *clen, uint8_t *file,
                           hipStream_t st)
{
    if (n > 0) hipLaunchKernelGGL(lz4_emit_kernel, dim3(n), dim3(256), 0, st, outs, n, stage, clen, file);
    return hipGetLastError();
}

uint64_t lz4_piece_stride() { return kLzSegStride; }

hipError_t launch_lz4(const ClosedRec *closed, const uint32_t *nclosed, int closed_cap, uint32_t cmax,
                      const uint8_t *arena, uint8_t *carena, uint64_t cslot, uint32_t *seg_clen, uint32_t *file_len,
                      uint32_t *work, hipStream_t st)
{
    // persistent grids (no host round trip for the device-side closed count); the short last
    // segments (16 KiB tables, at most one per container) go first, the main pass's tail then
    // overlaps the next batch's pass on the other LZ4 stream
    static const int ncu = [] {
        int d = 0, n = 0;
        if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
            n = 256;
        return n > 0 ? n : 256;
    }();
    static const int wpc = [] { const char *e = getenv("HDRF_LZ4_WAVES"); const int v = e ? atoi(e) : 16; return v > 0 ? v : 16; }();
    const int nseg_max = (int)((cmax + kLzMaxIn - 1) / kLzMaxIn);
    if (hipError_t e = hipMemsetAsync(work, 0, 2 * sizeof(uint32_t), st)) return e;
    const int prio = (setprio_mask() >> 6) & 1;
    hipLaunchKernelGGL(lz4_seg_kernel<true>, dim3(std::min(closed_cap, 4 * ncu)), dim3(64), 0, st, closed, nclosed,
                       arena, (uint64_t)cmax, carena, cslot, seg_clen, nseg_max, work, prio);
    hipLaunchKernelGGL(lz4_seg_kernel<false>, dim3(std::min(closed_cap * nseg_max, wpc * ncu)), dim3(64), 0, st, closed,
                       nclosed, arena, (uint64_t)cmax, carena, cslot, seg_clen, nseg_max, work + 1, prio);
    hipLaunchKernelGGL(lz4_pack_kernel, dim3(closed_cap), dim3(256), 0, st, closed, nclosed, carena, cslot, seg_clen,
                       nseg_max, file_len);
    return hipGetLastError();
}

}  // namespace hdrf
