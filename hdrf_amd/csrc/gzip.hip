// gzip.hip — stream-mode compressor 5 (Hadoop GzipCodec = zlib 1.2.11 level 6), stage 1 of the
// GPU deflate: the position-parallel match pass.
//
// Reference: DN/BlockReceiver.java:858-873,887-894 stream every received block through
// GzipCodec; the arithmetic is zlib's deflate_slow/longest_match (restated and pinned against
// zlib in oracle/hdrf_gzip.c, which is the checker of this file).  At level 6 every position
// p <= n-3 is inserted into the hash chains, the 15-bit hash is a pure function of the 3 bytes at
// p, and the lookahead mid-stream never drops under 262 B.  Hence longest_match(p) depends only on
// p and on whether prev_length >= good_match (chain 128, else 32; nice 128): the chain at p is
// "earlier positions with the same hash, nearest first", the head at distance <= MAX_DIST and
// every later candidate at distance < MAX_DIST, position 0 never (zlib's NIL).  The lazy parse
// (stage 2) then only reads the two answers computed here.
//
// gz_prev_kernel: prev[p] = 1 + nearest q < p with hash(q) == hash(p), q >= 1 (0: none within
//   MAX_DIST).  One workgroup per 4096-position tile: a 32768-entry "last position" table in LDS
//   (128 KiB) is seeded from the MAX_DIST positions before the tile (atomicMax, order-free), then
//   the tile runs in rounds of 256 positions (nearest equal hash earlier in the round, else the
//   table; the round's positions are then max-inserted).
// gz_match_kernel: one lane per position walks prev[] and compares bytes; out128[p] / out32[p] =
//   (len << 16) | dist of the chain-128 / chain-32 answer (0 if no match of >= 3 bytes), bit 31
//   set when the head candidate sits at distance exactly MAX_DIST on a 32 KiB boundary — zlib's
//   window base after a slide is such a position and is NIL there, so stage 2 re-checks it.
#include "bytes.hpp"

namespace hdrf {

constexpr int kGzWsize = 32768;
constexpr int kGzMaxDist = kGzWsize - 262;       // MAX_DIST = WSIZE - MIN_LOOKAHEAD
constexpr int kGzTile = 4096;
constexpr int kGzHash = 1 << 15;

__device__ __forceinline__ uint32_t gz_hash(const uint8_t *s)
{
    return (((uint32_t)s[0] << 10) ^ ((uint32_t)s[1] << 5) ^ (uint32_t)s[2]) & (kGzHash - 1);
}

__global__ void __launch_bounds__(256) gz_prev_kernel(const uint8_t *__restrict__ src, int64_t n,
                                                      uint32_t *__restrict__ prev)
{
    extern __shared__ uint32_t last[];             // kGzHash entries: 1 + latest position (0 none)
    __shared__ uint32_t sh[256];
    const int tid = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * kGzTile;
    const int64_t nins = n - 2;                    // positions p <= n-3 are hashed/inserted
    for (int i = tid; i < kGzHash; i += 256) last[i] = 0;
    __syncthreads();
    int64_t w0 = t0 - kGzMaxDist;
    if (w0 < 1) w0 = 1;
    for (int64_t q = w0 + tid; q < t0 && q < nins; q += 256) atomicMax(&last[gz_hash(src + q)], (uint32_t)q + 1u);
    __syncthreads();
    for (int r = 0; r < kGzTile; r += 256) {
        const int64_t p = t0 + r + tid;
        const bool valid = p < nins;
        const uint32_t h = valid ? gz_hash(src + p) : 0xffffffffu;
        sh[tid] = (valid && p >= 1) ? h : 0xfffffffeu;
        __syncthreads();
        uint32_t pr = 0;
        if (valid) {
            int j = tid - 1;
            while (j >= 0 && sh[j] != h) j--;
            pr = j >= 0 ? (uint32_t)(t0 + r + j) + 1u : last[h];
            prev[p] = pr;
        }
        __syncthreads();
        if (valid && p >= 1) atomicMax(&last[h], (uint32_t)p + 1u);
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) gz_match_kernel(const uint8_t *__restrict__ src, int64_t n,
                                                       const uint32_t *__restrict__ prev, uint32_t *__restrict__ out128,
                                                       uint32_t *__restrict__ out32)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    uint32_t r128 = 0, r32 = 0;
    const uint32_t head = p < n - 2 ? prev[p] : 0u;
    if (head != 0 && p - (int64_t)(head - 1) <= kGzMaxDist) {
        const int64_t look = n - p;
        const int maxlen = look < 258 ? (int)look : 258;
        const int nice = look < 128 ? (int)look : 128;
        const uint8_t *scan = src + p;
        int best = 2, k = 0;
        int64_t bq = 0;
        uint32_t s32 = 0;
        bool snap = false;
        int64_t q = head - 1;
        uint32_t flag = (p - q == kGzMaxDist && (q & (kGzWsize - 1)) == 0) ? 0x80000000u : 0u;
        for (;;) {
            ++k;
            const uint8_t *m = src + q;
            int len = 0;
            while (len < maxlen && m[len] == scan[len]) len++;
            bool brk = false;
            if (len > best) {
                best = len;
                bq = q;
                brk = len >= nice;
            }
            if (k == 32) {
                s32 = best >= 3 ? ((uint32_t)best << 16) | (uint32_t)(p - bq) : 0u;
                snap = true;
            }
            if (brk || k == 128) break;
            const uint32_t nx = prev[q];
            if (nx == 0 || p - (int64_t)(nx - 1) >= kGzMaxDist) break;
            q = nx - 1;
        }
        r128 = best >= 3 ? ((uint32_t)best << 16) | (uint32_t)(p - bq) : 0u;
        r32 = snap ? s32 : r128;
        r128 |= flag;
        r32 |= flag;
    }
    out128[p] = r128;
    out32[p] = r32;
}

// ---- stage 2: zlib's lazy parse (deflate_slow) over the stage-1 answers, one lane per stream.
// The window base advances by WSIZE exactly when zlib's fill_window slides (strstart - base >=
// WSIZE + MAX_DIST once the lookahead is under MIN_LOOKAHEAD); it decides the window-base NIL
// corner flagged by stage 1 and the stored-block eligibility (block_start >= base) of stage 3.
// syms: (dist << 8) | lc per symbol; blks: per flushed block (symbol end, block_start, strstart,
// base, last); cnt = {symbols, blocks}.
__global__ void gz_parse_kernel(const uint8_t *__restrict__ src, int64_t n, const uint32_t *__restrict__ m128,
                                const uint32_t *__restrict__ m32, uint32_t *__restrict__ syms, int64_t *__restrict__ blks,
                                int64_t *__restrict__ cnt)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    constexpr int64_t kLook = 262, kLitbuf = 16384;
    int64_t strstart = 0, base = 0, end = 0, block_start = 0, match_start = 0, prev_match = 0;
    int64_t nsym = 0, nblk = 0, blk_sym = 0;
    uint32_t match_length = 2, prev_length = 2;
    bool match_available = false;
    auto flush = [&](int last) {
        int64_t *b = blks + 5 * nblk++;
        b[0] = nsym; b[1] = block_start; b[2] = strstart; b[3] = base; b[4] = last;
        blk_sym = nsym;
        block_start = strstart;
    };
    auto tally = [&](uint32_t dist, uint32_t lc) {
        syms[nsym++] = (dist << 8) | lc;
        return nsym - blk_sym == kLitbuf - 1;
    };
    for (;;) {
        if (end - strstart < kLook) {
            if (strstart - base >= kGzWsize + kGzMaxDist) base += kGzWsize;
            end = base + 2 * kGzWsize < n ? base + 2 * kGzWsize : n;
            if (end - strstart == 0) break;
        }
        prev_length = match_length;
        prev_match = match_start;
        match_length = 2;
        if (end - strstart >= 3 && prev_length < 16) {
            const uint32_t v = (prev_length >= 8 ? m32 : m128)[strstart];
            const int64_t dist = v & 0xffff;
            const uint32_t len = (v >> 16) & 0x7fff;
            const bool nil = (v >> 31) && strstart - dist == base;
            if (v && !nil && len > prev_length) {
                match_length = len;
                match_start = strstart - dist;
                if (len == 3 && dist > 4096) match_length = 2;
            }
        }
        if (prev_length >= 3 && match_length <= prev_length) {
            const bool bf = tally((uint32_t)(strstart - 1 - prev_match), prev_length - 3);
            strstart += prev_length - 1;
            match_available = false;
            match_length = 2;
            if (bf) flush(0);
        } else if (match_available) {
            if (tally(0, src[strstart - 1])) flush(0);
            strstart++;
        } else {
            match_available = true;
            strstart++;
        }
    }
    if (match_available) tally(0, src[strstart - 1]);
    flush(1);
    cnt[0] = nsym;
    cnt[1] = nblk;
}

hipError_t launch_gzip_parse(const uint8_t *src, int64_t n, const uint32_t *m128, const uint32_t *m32, uint32_t *syms,
                             int64_t *blks, int64_t *cnt, hipStream_t st)
{
    hipLaunchKernelGGL(gz_parse_kernel, dim3(1), dim3(64), 0, st, src, n, m128, m32, syms, blks, cnt);
    return hipGetLastError();
}

size_t gzip_match_lds() { return sizeof(uint32_t) * kGzHash; }

hipError_t launch_gzip_match(const uint8_t *src, int64_t n, uint32_t *prev, uint32_t *out128, uint32_t *out32,
                             hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    static const hipError_t attr = hipFuncSetAttribute((const void *)gz_prev_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)gzip_match_lds());
    if (attr != hipSuccess) return attr;
    const unsigned tiles = (unsigned)((n + kGzTile - 1) / kGzTile);
    hipLaunchKernelGGL(gz_prev_kernel, dim3(tiles), dim3(256), gzip_match_lds(), st, src, n, prev);
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(gz_match_kernel, dim3(g), dim3(256), 0, st, src, n, prev, out128, out32);
    return hipGetLastError();
}

}  // namespace hdrf
