// lanehash.hip — content-defined chunking and SHA-1 / SHA-224 fingerprints in ONE pass over the
// bytes (HDRF_FUSED=1) on gfx950.
//
// Reference: DataDeduplicator.chunking (DN/DataDeduplicator.java:264-307) and threadedHasher.run
// (:578-641; DN/utilities.java:98-137), the same rules as chunk.hip and sha.hip.
//
// The two-pass front reads a batch's bytes about three times: the granule-maximum pass (4.56 GB
// counted per 4 GiB batch), the lane walk's raw lines (1.27 GB) and the SHA lanes' windows (7.00 GB,
// profiles/r06_c2_traffic.json).  Here a lane walks its speculative segment (chunk.hip §1b: the same
// segments, LDS cut lists, sync rule and SegMeta, so the repair / stitch / fallback kernels run
// unchanged) 64 bytes per step, and the 64 bytes of a step feed both the chunk rule and the SHA
// compression of the chunk being cut.  A step is one compression for every lane: a chunk's blocks
// are chunk-relative (64-B blocks from its start p, loaded at p + 64 blk, realigned with v_perm as in
// sha.hip), so the window [p, p + w] is blocks 0 .. w/64 and the search starts in block w/64 at the
// same offset for every chunk; the block holding the cut is padded in place when the message end
// leaves room for the length, else the lane's next step is the length-only block.
//   window   signed running maxima of the block's words (v_pk_max_i16 on the raw bytes and on the
//            bytes shifted up, chunk.hip gmax16_s), the snapshot at the window's last word
//   search   bit 7 of every byte whose biased value is >= M (SWAR carry test), gathered into a
//            64-bit mask (v_dot4), limited to the search range, first set bit
// Digests: spec_dig[segment][cut index] for every cut of a real lane's chain, and bdig[segment k + 1]
// for the chunk ending at the cut where lane k met segment k + 1 (that chunk starts on lane k's chain;
// segment k + 1's own digest for it started at a speculative cut).  stitch_copy moves the digests of
// the block's path next to its offsets and clears need[] for them; whatever the path took from a
// repair or the sequential fallback, and each block's last chunk (the drop-last rule), is hashed by
// sha.hip's kernel for the chunks still marked.
#define HDRF_SHA_K256_LINKAGE static
#include "sha_core.hpp"

namespace hdrf {

typedef __attribute__((address_space(3))) volatile uint16_t lds_u16h;
typedef __attribute__((address_space(3))) volatile uint8_t lds_u8h;
typedef short sh2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ sh2 as_sh2(uint32_t x) { return __builtin_bit_cast(sh2, x); }
__device__ __forceinline__ uint32_t pkmax_s(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(as_sh2(a), as_sh2(b)));
}
// signed maximum of the four bytes held as (odd, even) packed 16-bit running maxima (high bytes)
__device__ __forceinline__ int smax_of(uint32_t odd, uint32_t even)
{
    const uint32_t t = pkmax_s(odd, even);
    return max((int)t >> 24, (int)(t << 16) >> 24);
}
// bit 7 of each byte of word x whose biased value (x ^ 0x80) is >= m: C = 256 - m in every byte
// (m >= 1), Cm = C & 0x7f7f7f7f
__device__ __forceinline__ uint32_t ge_bits(uint32_t x, uint32_t C, uint32_t Cm)
{
    const uint32_t s = (x & 0x7f7f7f7fu) + Cm;
    return __builtin_amdgcn_bitop3_b32(x, C, s, 0x8e) & 0x80808080u;   // maj(NOT x, C, s)
}
// 16 bits (bit k = byte k of the four big-endian words: byte k of word i is bits 31-8(k&3) of it)
__device__ __forceinline__ uint32_t gather_be(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3)
{
    const uint32_t lo = __builtin_amdgcn_udot4(f1, 0x10204080u, __builtin_amdgcn_udot4(f0, 0x01020408u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(f3, 0x10204080u, __builtin_amdgcn_udot4(f2, 0x01020408u, 0u, false), false);
    return (lo | (hi << 8)) >> 7;
}
__device__ __forceinline__ unsigned long long bits_ge(int a)     // bits a..63
{
    return a <= 0 ? ~0ull : (a >= 64 ? 0ull : (~0ull << a));
}
__device__ __forceinline__ unsigned long long bits_le(int b)     // bits 0..b
{
    return b < 0 ? 0ull : (b >= 63 ? ~0ull : ((2ull << b) - 1ull));
}

// the 17 dwords (68 B) of one block at pos (4-aligned down).  Near the end of the readable bytes the
// words past it re-read the last readable word: no byte at or past the block's length is ever used
// (the chunk rule reads up to size - 1, pad_block clears the words after a message)
__device__ __forceinline__ void load17(const uint8_t *base, uint64_t readable, uint32_t pos, uint32_t d[17])
{
    const uint32_t apos = pos & ~3u;
    if ((uint64_t)apos + 68u <= readable) {
        const HDRF_GLOBAL uint32_t *q = gptr<uint32_t>(base + apos);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const u32x4a v = *(const HDRF_GLOBAL u32x4a *)(q + 4 * i);
            d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
        d[16] = q[16];
    } else {
        const uint32_t lim = (uint32_t)((readable - 4u) & ~3ull);
#pragma unroll
        for (int i = 0; i < 17; i++) d[i] = *gptr<uint32_t>(base + min(apos + 4u * i, lim));
    }
}

template <int HW>
__device__ __forceinline__ void put_digest(uint32_t *dst, const uint32_t st[8])
{
#pragma unroll
    for (int i = 0; i < HW; i++) dst[i] = __builtin_bswap32(st[i]);
}

// grid: one wave per 63 lane segments (chunk.hip's lane walk layout), 256 threads
template <int HW>
__global__ void __launch_bounds__(256, 4) lane_hash_kernel(const BlockDesc *__restrict__ blocks, int nblocks,
                                                        int total_waves, int w, int maxlen,
                                                        uint32_t *__restrict__ spec, int cap,
                                                        SegMeta *__restrict__ meta, int *__restrict__ rq,
                                                        int *__restrict__ rq_count, int rq_cap,
                                                        uint32_t *__restrict__ irr, uint32_t *__restrict__ sdig,
                                                        uint32_t *__restrict__ bdig, int *__restrict__ gm_need,
                                                        int *__restrict__ err)
{
    __shared__ uint16_t s_cuts[4][64 * kLdsCutsF];
    __shared__ uint8_t s_cnt[4][64];
    const int wv = blockIdx.x * 4 + wave_id();
    if (wv >= total_waves) return;
    lds_u16h *vcuts = (lds_u16h *)s_cuts[wave_id()];     // read by the neighbouring lane
    lds_u8h *vcnt = (lds_u8h *)s_cnt[wave_id()];
    int bix = 0;
    for (int i = 1; i < nblocks; i++)
        if (blocks[i].wave0 <= wv) bix = i;
    const BlockDesc bd = blocks[bix];
    const int l = lane_id();
    const int wl = wv - bd.wave0;
    const int nseg = bd.nseg, Ls = bd.seg_len, size = (int)bd.len;
    const uint8_t *base = bd.data;
    const uint64_t readable = bd.readable;
    const int k = wl * kWaveSegs + l;                     // lane 63: the next wave's first segment
    const bool exists = k < nseg;
    const bool real = exists && l < kWaveSegs;
    const int s = k * Ls;
    const bool has_next = exists && k + 1 < nseg;
    const int e = (real && has_next) ? (k + 1) * Ls : 0x7fffffff;      // overrun (sync) threshold
    const int over_lim = has_next ? (k + 1) * Ls + Ls - 64 : 0x7fffffff;
    const int ncap = min(cap, kLdsCutsF);
    const int G = bd.seg0 + k;
    uint32_t *dseg = sdig + (size_t)G * cap * HW;
    const int wb = w >> 6, wo = w & 63;                   // window byte w: block wb, byte wo
    const int wsw = wo >> 2, wsb = wo & 3;                // its word and byte (big-endian order)

    int p = s;                                            // chunk start
    bool first = s == 0;                                  // the block's first chunk: no 0 floor (:281)
    int n = 0, n_main = -1, ptr = 0, sync = kSyncEnd;
    bool active = exists, walking = exists, overflow = false;
    vcnt[l] = 0;
    uint32_t st[8];
    set_iv<HW>(st);
    int blk = 0;                                          // the chunk's next 64-B block
    uint32_t wodd = 0x80808080u, wev = 0x80808080u;       // window running maxima (raw, signed pairs)
    uint32_t M = 0;                                       // the window maximum, biased (final at block wb)
    bool pend = false, pbs = false;                       // length-only block due; its digest also to bdig
    uint32_t plen = 0;
    int pci = 0;
    // the block of the lane's next data step, loaded one step ahead: the load is issued after this
    // step's scan (which fixes where the next block starts) and lands under this step's compression
    uint32_t dn[17];
    if (active) load17(base, readable, (uint32_t)p, dn);
    for (;;) {
        if (!ballot64(active && l < kWaveSegs)) break;
        if (!active) continue;
        // One compression per lane and step, one code path for every lane (the lanes of a wave are
        // at different places of their chunks, so a branch per case would run every case each step):
        // the block is the chunk's next 64 bytes — padded in place when the cut is in it — or the
        // length-only block of the chunk cut last step (pad_block zeroes whatever the words held).
        const bool padstep = pend;
        const int pos = p + 64 * blk;                      // (a pad step: the next chunk's start)
        if (!padstep) {
            if (blk == 0 && p + w > size - 1) { active = walking = false; continue; }   // window incomplete
            if (walking && pos - 64 > over_lim) { sync = kSyncFail; active = walking = false; continue; }   // byte cap
        }
        uint32_t m[16];
        {
            const uint32_t sel = 0x00010203u + ((uint32_t)pos & 3u) * 0x01010101u;
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_perm(dn[i + 1], dn[i], sel);
        }
        // ---- window: running signed maxima over the words; the snapshot at window word wsw --------
        uint32_t ro = wodd, re = wev, so = 0, se = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (i == wsw) {                                // (uniform) the window's last word: its bytes
                const uint32_t keep = wsb == 3 ? 0xffffffffu : ~(0xffffffffu >> (8 * (wsb + 1)));
                const uint32_t x = (m[i] & keep) | (0x80808080u & ~keep);   // after byte wo: -128
                so = pkmax_s(ro, x);
                se = pkmax_s(re, x << 8);
            }
            ro = pkmax_s(ro, m[i]);
            re = pkmax_s(re, m[i] << 8);
        }
        int mx = smax_of(so, se) + 128;                    // biased
        if (!first) mx = max(mx, 0x80);                    // mValue reset to 0 after a cut (:281)
        const uint32_t Mb = blk == wb ? (uint32_t)mx : M;  // the threshold this block's search uses
        if (!padstep) {
            if (blk < wb) { wodd = ro; wev = re; }
            if (blk == wb) M = Mb;
        }
        // ---- search: the first byte >= M in [w + 1, ub] (chunk-relative), ub = min(maxlen, size - 1 - p)
        const int ub = min(maxlen, size - 1 - p);
        const int sa = blk < wb ? 64 : (blk == wb ? wo + 1 : 0), sb = ub - 64 * blk;
        unsigned long long hit;
        {
            const uint32_t C = __builtin_amdgcn_perm(256u - Mb, 256u - Mb, 0u), Cm = C & 0x7f7f7f7fu;
            uint32_t q[4];
#pragma unroll
            for (int g = 0; g < 4; g++)
                q[g] = gather_be(ge_bits(m[4 * g], C, Cm), ge_bits(m[4 * g + 1], C, Cm), ge_bits(m[4 * g + 2], C, Cm),
                                 ge_bits(m[4 * g + 3], C, Cm));
            hit = (unsigned long long)(q[0] | (q[1] << 16)) | ((unsigned long long)(q[2] | (q[3] << 16)) << 32);
            if (Mb == 0) hit = ~0ull;                      // every byte qualifies
            hit &= bits_ge(sa) & bits_le(sb);
        }
        int jb = -1;
        if (hit) jb = __builtin_ctzll(hit);
        else if (sb <= 63 && sa <= 63 && ub == maxlen) jb = sb;   // forced cut at p + maxlen (:288-294)
        if (!padstep && jb < 0 && sa <= 63 && sb <= 63) { active = walking = false; continue; }   // data ended
        if (padstep) jb = -1;
        // padding: the cut's block (length in place when it fits), the length-only block, or none
        uint32_t len, pj, nb;
        if (padstep) { len = plen; nb = (plen + 8) / 64 + 1; pj = nb - 1; }
        else if (jb >= 0) { len = (uint32_t)(64 * blk + jb + 1); nb = (len + 8) / 64 + 1; pj = (uint32_t)blk; }
        else { len = (uint32_t)(64 * blk + 64); pj = (uint32_t)blk; nb = pj + 2; }   // a full block: unchanged
        pad_block(m, len, pj, nb);
        if (!padstep)                                      // the next data step's block: the chunk's next
            load17(base, readable, (uint32_t)(jb < 0 ? pos + 64 : pos + jb + 1), dn);   // 64 B, or the next chunk
        if (HW == 5) sha1_compress(st, m);
        else sha256_compress(st, m);
        bool fin = padstep, fbs = pbs;                     // the digest is final: write it
        int fci = pci;
        if (padstep) {
            pend = false;
        } else if (jb < 0) {
            blk++;                                         // a message block of the chunk
        } else {
            const int cut = pos + jb + 1;                  // :276-283
            const int ci = min(n, ncap - 1);
            overflow |= n >= ncap;
            vcuts[l * kLdsCutsF + ci] = (uint16_t)min(cut - s, 0xffff);
            vcnt[l] = (uint8_t)(ci + 1);
            n = ci + 1;
            bool bs = false;
            if (cut >= e) {                                // overrun: look for a shared cut
                if (n_main < 0) n_main = ci;
                const int sc = vcnt[l + 1];
                const int rel = cut - e;
                lds_u16h *sl = vcuts + (l + 1) * kLdsCutsF;
                while (ptr < sc && (int)sl[ptr] < rel) ptr++;
                if (rel >= Ls) { sync = kSyncFail; walking = false; }
                else if (ptr < sc && (int)sl[ptr] == rel) { sync = (ci - n_main) | (ptr << 16); walking = false; bs = true; }
                else if (n - n_main >= kLaneOver) { sync = kSyncFail; walking = false; }
            }
            p = cut;
            first = false;
            blk = 0;
            wodd = wev = 0x80808080u;
            if (walking && p >= over_lim && p + w <= size - 1) { sync = kSyncFail; walking = false; }   // byte cap
            if (overflow) walking = false;
            if (nb == (len - 1) / 64 + 1) {                // the length fitted in the cut's block
                fin = true; fbs = bs; fci = ci;
            } else {                                       // the length-only block next step
                pend = true; pbs = bs; plen = len; pci = ci;
            }
        }
        if (fin) {
            if (real) put_digest<HW>(dseg + (size_t)fci * HW, st);
            if (fbs) put_digest<HW>(bdig + (size_t)(G + 1) * HW, st);
            set_iv<HW>(st);
            if (!walking && !pend) active = false;
        }
    }
    if (overflow && real) atomicOr(err, 64);
    if (real) {
        uint32_t *list = spec + (size_t)G * cap;
        for (int i = 0; i < n; i++) list[i] = (uint32_t)s + (uint32_t)vcuts[l * kLdsCutsF + i];
        if (n_main < 0) n_main = n;
        SegMeta mt;
        mt.n_main = n_main; mt.n_over = n - n_main; mt.sync = sync; mt.jmp = 0; mt.jj = 0; mt.n_ext = 0; mt.ext_dst = -1;
        mt.cp_from = 0; mt.cp_n = 0; mt.cp_dst = 0; mt.pad[0] = mt.pad[1] = mt.pad[2] = 0;
        meta[G] = mt;
        if (k < nseg - 1 && sync < 0) atomicOr(irr + (G >> 5), 1u << (G & 31));   // irregular boundary
        if (sync == kSyncFail) {
            const int q = atomicAdd(rq_count, 1);
            if (q < rq_cap) rq[q] = G;
            atomicOr(gm_need + bix, 1);                    // the repair walk reads the block's maxima
        }
    }
}

hipError_t launch_lane_hash(int hasher, const BlockDesc *d_blocks, int nblocks, int total_waves, int w, int maxlen,
                            uint32_t *spec, int cap, SegMeta *meta, int *rq, int *rq_count, int rq_cap, uint32_t *irr,
                            uint32_t *sdig, uint32_t *bdig, int *gm_need, int *err, hipStream_t st)
{
    const dim3 g((total_waves + 3) / 4);
    if (hasher == 0)
        hipLaunchKernelGGL(lane_hash_kernel<5>, g, dim3(256), 0, st, d_blocks, nblocks, total_waves, w, maxlen, spec, cap,
                           meta, rq, rq_count, rq_cap, irr, sdig, bdig, gm_need, err);
    else
        hipLaunchKernelGGL(lane_hash_kernel<7>, g, dim3(256), 0, st, d_blocks, nblocks, total_waves, w, maxlen, spec, cap,
                           meta, rq, rq_count, rq_cap, irr, sdig, bdig, gm_need, err);
    return hipGetLastError();
}

}  // namespace hdrf
