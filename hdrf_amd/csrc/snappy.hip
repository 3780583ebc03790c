// snappy.hip — stream-mode compressor 0 (Hadoop SnappyCodec) on gfx950.
//
// Reference: DN/BlockReceiver.java:826-873,887-894,1238-1256 — with compressor == 0 a received
// block is streamed through SnappyCodec.createOutputStream(chunkDir + id), i.e. Hadoop's
// BlockCompressorStream (256 KiB buffer, overhead bufferSize/6 + 32, MAX_INPUT 218,422) around
// snappy::RawCompress calls made by the native SnappyCompressor.  The raw compressor is google/
// snappy's level-1 algorithm (restated in the test oracle; pinned against the
// snappy bundled in pyarrow, parity vs Hadoop's host libsnappy unpinned — DESIGN.md §12).
//
// A raw buffer is varint(n) followed by independent 64 KiB fragments (fresh hash table each), so
// one wave owns one fragment, table (2^15 u16 entries) in LDS, and sn_join concatenates a
// group's fragments.  The greedy parse is sequential; as in lz4.hip its search loop is made
// wave-parallel: the positions it visits depend only on the attempt count (step = skip++ >> 5),
// so batches of 16, 32, then 64 attempts are evaluated at once (positions from a constant table)
// with an exact replay of the table reads/writes in attempt order; match extension and literal
// copies are 64-lane operations.
#include "bytes.hpp"

namespace hdrf {

constexpr int kSnFrag = 65536;
constexpr int kSnFragStride = 76544;             // >= 32 + 65536 + 65536 / 6, 256-B multiple
constexpr int kSnMaxAttempts = 320;              // > 268: attempts past 64 KiB are never valid
constexpr uint32_t kSnTable = 1u << 15;

struct SnSteps {                                   // attempt k: position ip0 + off[k], stride step[k]
    uint32_t off[kSnMaxAttempts], step[kSnMaxAttempts];
    constexpr SnSteps() : off(), step()
    {
        uint32_t skip = 32, o = 0;
        for (int k = 0; k < kSnMaxAttempts; k++) {
            const uint32_t s = skip >> 5;
            off[k] = o;
            step[k] = s;
            skip += s;
            o += s;
        }
    }
};
__constant__ const SnSteps kSn = SnSteps();

__device__ __forceinline__ uint32_t snh(uint32_t v, uint32_t mask) { return ((v * 0x1e35a7bdu) >> 17) & mask; }

// literal: tag (+ 1..4 length bytes) + the bytes; returns the new output offset
__device__ __forceinline__ int sn_lit(uint8_t *out, int op, const uint8_t *lit, int len)
{
    const uint32_t n = (uint32_t)(len - 1);
    if (n < 60) {
        if (lane_id() == 0) wr8(out + op, n << 2);
        op += 1;
    } else {
        const int cnt = n < 256u ? 1 : n < 65536u ? 2 : n < (1u << 24) ? 3 : 4;
        const int l = lane_id();
        if (l == 0) wr8(out + op, (uint32_t)(59 + cnt) << 2);
        if (l < cnt) wr8(out + op + 1 + l, n >> (8 * l));
        op += 1 + cnt;
    }
    wave_copy(out + op, lit, len);
    return op + len;
}

// copy of len >= 4 bytes at distance off < 65536: 64-byte pieces while len >= 68, a 60-byte
// piece if still > 64, then the rest (1-byte-offset form when < 12 bytes and off < 2048)
__device__ __forceinline__ int sn_copy(uint8_t *out, int op, uint32_t off, int len)
{
    const int l = lane_id();
    const int k64 = len >= 68 ? (len - 68) / 64 + 1 : 0;
    for (int i = l; i < k64; i += 64) {
        wr8(out + op + 3 * i, 0xFE);                       // 2 | (63 << 2)
        wr8(out + op + 3 * i + 1, off);
        wr8(out + op + 3 * i + 2, off >> 8);
    }
    op += 3 * k64;
    len -= 64 * k64;
    if (len > 64) {
        if (l == 0) { wr8(out + op, 2u | (59u << 2)); wr8(out + op + 1, off); wr8(out + op + 2, off >> 8); }
        op += 3;
        len -= 60;
    }
    if (len < 12 && off < 2048) {
        if (l == 0) { wr8(out + op, 1u | ((uint32_t)(len - 4) << 2) | ((off >> 8) << 5)); wr8(out + op + 1, off); }
        op += 2;
    } else {
        if (l == 0) { wr8(out + op, 2u | ((uint32_t)(len - 1) << 2)); wr8(out + op + 1, off); wr8(out + op + 2, off >> 8); }
        op += 3;
    }
    return op;
}

// One fragment (n <= 64 KiB) -> snappy elements at out; returns their size.  Uniform control flow.
__device__ int sn_fragment(const uint8_t *src, int n, uint8_t *out, unsigned short *tab)
{
    const int l = lane_id();
    uint32_t ts = 256;
    while (ts < kSnTable && ts < (uint32_t)n) ts <<= 1;
    const uint32_t mask = ts - 1;
    uint4 *t4 = (uint4 *)tab;
    for (uint32_t i = l; i < ts / 8; i += 64) t4[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("" ::: "memory");
    int op = 0, ip = 0;
    if (n >= 15) {
        const int lim = n - 15;
        for (;;) {
            const int next_emit = ip, ip0 = ip + 1;
            int a0 = 0, m = 16, fpos = -1, fref = 0;
            for (;;) {
                // ---- a batch of m search attempts (lane l = attempt a0 + l) -----------------
                const int k = a0 + l;
                const bool inb = l < m && k < kSnMaxAttempts;
                const int pos = inb ? ip0 + (int)kSn.off[k] : 0;
                const bool valid = inb && pos + (int)kSn.step[k] <= lim;
                const uint32_t v = valid ? rd32u(src + pos) : 0u;
                const uint32_t h = snh(v, mask);
                const unsigned long long vmask = ballot64(valid);
                const int nv = vmask == ~0ull ? 64 : __builtin_ctzll(~vmask);   // valid lanes are a prefix
                // distinct hashes: every attempt reads the pre-batch entry (one gather, one
                // scatter); else a lane-by-lane replay.  Distinctness: scatter lane tags, read back
                int old = 0;
                if (valid) old = tab[h];
                asm volatile("" ::: "memory");
                if (valid) tab[h] = (unsigned short)l;
                asm volatile("" ::: "memory");
                const int t = valid ? (int)tab[h] : l;
                const bool slow = ballot64(valid && t != l) != 0;
                asm volatile("" ::: "memory");
                if (slow && valid) tab[h] = (unsigned short)old;            // equal hashes carry equal olds
                int ref = old;
                asm volatile("" ::: "memory");
                if (slow) {
                    for (int i = 0; i < nv; i++) {
                        if (l == i) { ref = tab[h]; tab[h] = (unsigned short)pos; }
                        asm volatile("" ::: "memory");
                    }
                }
                const bool ok = valid && rd32u(src + ref) == v;
                const unsigned long long okm = ballot64(ok);
                if (!slow) {                                   // commit attempts up to the first match
                    const int last = okm ? __builtin_ctzll(okm) : 63;
                    if (valid) tab[h] = (unsigned short)(l <= last ? pos : old);
                    asm volatile("" ::: "memory");
                }
                if (okm) {
                    const int istar = __builtin_ctzll(okm);
                    if (slow) {
                        for (int i = nv - 1; i > istar; i--) {   // undo the attempts after the match
                            if (l == i) tab[h] = (unsigned short)ref;
                            asm volatile("" ::: "memory");
                        }
                    }
                    fpos = (int)rdlane((uint32_t)pos, istar);
                    fref = (int)rdlane((uint32_t)ref, istar);
                    break;
                }
                if (nv < m) break;                             // the next attempt passes ip_limit
                a0 += m;
                m = min(64, 2 * m);
            }
            if (fpos < 0) { ip = next_emit; break; }
            ip = fpos;
            int cand = fref;
            op = sn_lit(out, op, src + next_emit, ip - next_emit);
            for (;;) {                                         // copies back to back
                const int base = ip;
                int p0 = ip + 4, c0 = cand + 4;
                for (;;) {                                     // match extension up to the fragment end
                    const int p = p0 + 4 * l;
                    uint32_t x;
                    if (p + 4 <= n) x = rd32u(src + p) ^ rd32u(src + c0 + 4 * l);
                    else if (p < n) x = (rd32u(src + p) ^ rd32u(src + c0 + 4 * l)) | (0xffffffffu << (8 * (n - p)));
                    else x = 0xffffffffu;
                    const unsigned long long mm = ballot64(x != 0u);
                    if (!mm) { p0 += 256; c0 += 256; continue; }
                    const int L = __builtin_ctzll(mm);
                    const uint32_t xl = rdlane(x, L);
                    p0 += 4 * L + (__builtin_ctz(xl) >> 3);
                    break;
                }
                ip = p0;
                op = sn_copy(out, op, (uint32_t)(base - cand), ip - base);
                if (ip >= lim) goto remainder;
                int r = 0;
                asm volatile("" ::: "memory");
                if (l == 0) {
                    tab[snh(rd32u(src + ip - 1), mask)] = (unsigned short)(ip - 1);
                    const uint32_t hh = snh(rd32u(src + ip), mask);
                    r = tab[hh];
                    tab[hh] = (unsigned short)ip;
                }
                asm volatile("" ::: "memory");
                cand = (int)rdlane((uint32_t)r, 0);
                if (rd32u(src + ip) != rd32u(src + cand)) break;
            }
        }
    }
remainder:
    if (ip < n) op = sn_lit(out, op, src + ip, n - ip);
    return op;
}

// grid nf x 64: fragment i -> scratch + i * kSnFragStride, size -> fclen[i]
__global__ void __launch_bounds__(64) sn_frag_kernel(const LzPiece *__restrict__ frags, int nf,
                                                     const uint8_t *__restrict__ base, uint8_t *__restrict__ scratch,
                                                     uint32_t *__restrict__ fclen)
{
    __shared__ unsigned short tab[kSnTable];
    const int i = blockIdx.x;
    if (i >= nf) return;
    const LzPiece f = frags[i];
    const int c = sn_fragment(base + f.src, (int)f.len, scratch + (size_t)i * kSnFragStride, tab);
    if (lane_id() == 0) fclen[i] = (uint32_t)c;
}

// grid n x 256: group i = varint(len) + its fragments (pieces[i].pad = first fragment) -> stage
__global__ void __launch_bounds__(256) sn_join_kernel(const LzPiece *__restrict__ pieces, int n,
                                                      const uint8_t *__restrict__ scratch,
                                                      const uint32_t *__restrict__ fclen, uint8_t *__restrict__ stage,
                                                      uint64_t stride, uint32_t *__restrict__ clen)
{
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzPiece pc = pieces[i];
    uint8_t *o = stage + (size_t)i * stride;
    int pos = 0;
    for (uint32_t v = pc.len;; v >>= 7) {
        if (threadIdx.x == 0) wr8(o + pos, v < 0x80 ? v : (v & 0x7f) | 0x80);
        pos++;
        if (v < 0x80) break;
    }
    const int nfr = (int)((pc.len + kSnFrag - 1) / kSnFrag);
    const int w = wave_id();
    for (int f = 0; f < nfr; f++) {
        const int c = (int)fclen[pc.pad + f];
        const int q = (c + 3) / 4;
        const int a = min(c, w * q), b = min(c, a + q);
        if (b > a) wave_copy(o + pos + a, scratch + (size_t)(pc.pad + f) * kSnFragStride + a, b - a);
        pos += c;
    }
    if (threadIdx.x == 0) clen[i] = (uint32_t)pos;
}

hipError_t launch_snappy_stream(const LzPiece *pieces, int n, const LzPiece *frags, int nf, const uint8_t *base,
                                uint8_t *scratch, uint32_t *fclen, uint8_t *stage, uint64_t stride, uint32_t *clen,
                                hipStream_t st)
{
    if (nf > 0) hipLaunchKernelGGL(sn_frag_kernel, dim3(nf), dim3(64), 0, st, frags, nf, base, scratch, fclen);
    if (n > 0)
        hipLaunchKernelGGL(sn_join_kernel, dim3(n), dim3(256), 0, st, pieces, n, scratch, fclen, stage, stride, clen);
    return hipGetLastError();
}

uint64_t snappy_frag_stride() { return kSnFragStride; }

// ---- decoder (read side: DataConstructor's SnappyCodec input stream, DN/DataConstructor.java:
//      102-220): one wave per raw buffer; element tags parsed from an LDS window of the input,
//      literals wave copies, each copy preceded by a fence (it may read output just written).
constexpr int kSnDecWin = 8192;

__global__ void __launch_bounds__(64) sn_decode_kernel(const LzDec *__restrict__ items, int n,
                                                       const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                       int *__restrict__ err)
{
    __shared__ uint8_t win[kSnDecWin];
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzDec d = items[i];
    const uint8_t *in = src + d.src;
    uint8_t *out = dst + d.dst;
    const int64_t iend = d.clen, oend = d.rawlen;
    const int l = lane_id();
    int64_t wbase = -kSnDecWin;
    auto byte = [&](int64_t pos) -> uint32_t {          // wave-uniform pos < iend
        if (pos >= wbase + kSnDecWin) {
            wbase = pos & ~(int64_t)15;
            __builtin_amdgcn_s_waitcnt(0);
            asm volatile("" ::: "memory");
            for (int k = l * 16; k < kSnDecWin; k += 64 * 16) {
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
    uint64_t raw = 0;
    for (int sh = 0;; sh += 7) {                         // varint32 raw length
        if (ip >= iend || sh > 28) { bad = true; break; }
        const uint32_t b = byte(ip++);
        raw |= (uint64_t)(b & 0x7f) << sh;
        if (!(b & 0x80)) break;
    }
    if (raw != (uint64_t)oend) bad = true;
    while (!bad && ip < iend) {
        const uint32_t tag = byte(ip++);
        int64_t len, off;
        if ((tag & 3) == 0) {
            len = (tag >> 2) + 1;
            if (len > 60) {
                const int cnt = (int)len - 60;
                if (ip + cnt > iend) { bad = true; break; }
                len = 0;
                for (int k = 0; k < cnt; k++) len |= (int64_t)byte(ip + k) << (8 * k);
                len += 1;
                ip += cnt;
            }
            if (ip + len > iend || op + len > oend) { bad = true; break; }
            wave_copy(out + op, in + ip, (int)len);
            ip += len;
            op += len;
            continue;
        }
        if ((tag & 3) == 1) {
            if (ip + 1 > iend) { bad = true; break; }
            len = 4 + ((tag >> 2) & 7);
            off = ((int64_t)(tag >> 5) << 8) | byte(ip);
            ip += 1;
        } else if ((tag & 3) == 2) {
            if (ip + 2 > iend) { bad = true; break; }
            len = (tag >> 2) + 1;
            off = (int64_t)byte(ip) | ((int64_t)byte(ip + 1) << 8);
            ip += 2;
        } else {
            if (ip + 4 > iend) { bad = true; break; }
            len = (tag >> 2) + 1;
            off = (int64_t)byte(ip) | ((int64_t)byte(ip + 1) << 8) | ((int64_t)byte(ip + 2) << 16) |
                  ((int64_t)byte(ip + 3) << 24);
            ip += 4;
        }
        if (off == 0 || off > op || op + len > oend) { bad = true; break; }
        __threadfence();
        if (l < len) wr8(out + op + l, rd8(out + op - off + (off >= len ? l : l % off)));   // len <= 64
        op += len;
    }
    __threadfence();
    if ((bad || op != oend) && l == 0) atomicOr(err, 1);
}

hipError_t launch_snappy_decode(const LzDec *items, int n, const uint8_t *src, uint8_t *dst, int *err, hipStream_t st)
{
    if (n > 0) hipLaunchKernelGGL(sn_decode_kernel, dim3(n), dim3(64), 0, st, items, n, src, dst, err);
    return hipGetLastError();
}

}  // namespace hdrf
