// lzo.hip — stream-mode compressor 3 on gfx950: the block through hadoop-lzo's LzopCodec
// (DN/BlockReceiver.java:836-845) and back through its input stream (DN/DataConstructor.java:
// 140-166).
//
// hadoop-lzo's LzopOutputStream cuts the stream into blocks like BlockCompressorStream (MAX_INPUT
// 245,693 B; a larger write is cut into slices, each its own block) and compresses each block with
// one lzo1x_1_compress call (LZO 2.10; deterministic build: a fresh 2^14-entry dictionary for
// every 49,152-B sub-block, the literal count carried across sub-blocks).  Blocks are independent,
// so one wave owns one block; the parse inside a block is LZO1X-1's greedy single-probe loop, run
// wave-uniformly (every lane holds the same parse state; the dictionary is in LDS, lane 0 stores
// the instruction bytes), with literal runs copied wave-wide.  The file framing (lzop header,
// [BE32 raw][BE32 stored] per block, BE32 0 at close) is planned on the host and written by
// lz4_emit_kernel (the same framing kernel as Lz4Codec).  The decoder is one wave per block.
// The oracle (oracle/hdrf_lzo.c) restates the same algorithm; parity vs hadoop-lzo / liblzo2 is
// unpinned.
#include "bytes.hpp"

namespace hdrf {

constexpr int kLzoDBits = 14;
// stage slot per block: the Lz4Codec piece stride (lz4_emit_kernel frames both), >= 245,693 + n/16 + 67
uint64_t lz4_piece_stride();

__device__ __forceinline__ uint64_t rd64u(const uint8_t *p) { return (uint64_t)rd32u(p) | ((uint64_t)rd32u(p + 4) << 32); }

struct LzoOut {                                    // wave-uniform output cursor (lane 0 stores)
    uint8_t *op;
    uint32_t p2 = 0, p1 = 0;                       // the last two instruction bytes put (op[-2], op[-1])
    __device__ __forceinline__ void put(uint32_t v)
    {
        if (lane_id() == 0) wr8(op, v);
        op++;
        p2 = p1;
        p1 = v & 0xffu;
    }
    // lzo's op[-2] |= t (1..3 literals after a match ride in its last instruction's low bits);
    // op[-2] is the previous match instruction's byte, kept in a register (no read-back)
    __device__ __forceinline__ void or_prev2(uint32_t t)
    {
        if (lane_id() == 0) wr8(op - 2, p2 | t);
    }
    __device__ __forceinline__ void zeros(int64_t n)   // n bytes of 0 (long length runs)
    {
        for (int64_t k = lane_id(); k < n; k += 64) wr8(op + k, 0);
        op += n;
    }
};

// lzo1x_c.ch do_compress (deterministic, unaligned-64 variant); returns the literals left
__device__ int64_t lzo_sub(const uint8_t *in, int64_t in_len, LzoOut &o, int64_t ti, unsigned short *dict)
{
    const uint8_t *ip = in, *ii = in;
    const uint8_t *const in_end = in + in_len, *const ip_end = in + in_len - 20;
    ip += ti < 4 ? 4 - ti : 0;
    ip += 1 + ((ip - ii) >> 5);                        // the loop's first step enters at `literal:`
    for (;;) {
        if (ip >= ip_end) break;
        const uint32_t dv = rd32u(ip);
        const uint32_t dindex = ((dv * 0x1824429du) >> (32 - kLzoDBits)) & ((1u << kLzoDBits) - 1);
        const uint8_t *m_pos = in + dict[dindex];
        __builtin_amdgcn_s_waitcnt(0);
        asm volatile("" ::: "memory");
        if (lane_id() == 0) dict[dindex] = (unsigned short)(ip - in);
        __builtin_amdgcn_s_waitcnt(0);
        asm volatile("" ::: "memory");
        if (dv != rd32u(m_pos)) {                      // literal
            ip += 1 + ((ip - ii) >> 5);
            continue;
        }
        ii -= ti;                                      // a match: its literals first
        ti = 0;
        {
            const int64_t t = ip - ii;
            if (t != 0) {
                if (t <= 3) {
                    o.or_prev2((uint32_t)t);
                } else if (t <= 18) {
                    o.put((uint32_t)(t - 3));
                } else {
                    int64_t tt = t - 18;
                    o.put(0);
                    const int64_t nz = tt > 255 ? (tt - 1) / 255 : 0;
                    o.zeros(nz);
                    tt -= 255 * nz;
                    o.put((uint32_t)tt);
                }
                wave_copy(o.op, ii, (int)t);
                o.op += t;
            }
        }
        int64_t m_len = 4;
        {
            uint64_t v = rd64u(ip + m_len) ^ rd64u(m_pos + m_len);
            bool done = false;
            while (v == 0) {
                m_len += 8;
                v = rd64u(ip + m_len) ^ rd64u(m_pos + m_len);
                if (ip + m_len >= ip_end) { done = true; break; }
            }
            if (!done) m_len += __builtin_ctzll(v) >> 3;
        }
        int64_t m_off = ip - m_pos;
        ip += m_len;
        ii = ip;
        if (m_len <= 8 && m_off <= 0x0800) {           // M2
            m_off -= 1;
            o.put((uint32_t)(((m_len - 1) << 5) | ((m_off & 7) << 2)));
            o.put((uint32_t)(m_off >> 3));
        } else if (m_off <= 0x4000) {                   // M3
            m_off -= 1;
            if (m_len <= 33) {
                o.put((uint32_t)(32 | (m_len - 2)));
            } else {
                m_len -= 33;
                o.put(32);
                const int64_t nz = m_len > 255 ? (m_len - 1) / 255 : 0;
                o.zeros(nz);
                m_len -= 255 * nz;
                o.put((uint32_t)m_len);
            }
            o.put((uint32_t)(m_off << 2));
            o.put((uint32_t)(m_off >> 6));
        } else {                                        // M4
            m_off -= 0x4000;
            if (m_len <= 9) {
                o.put((uint32_t)(16 | ((m_off >> 11) & 8) | (m_len - 2)));
            } else {
                m_len -= 9;
                o.put((uint32_t)(16 | ((m_off >> 11) & 8)));
                const int64_t nz = m_len > 255 ? (m_len - 1) / 255 : 0;
                o.zeros(nz);
                m_len -= 255 * nz;
                o.put((uint32_t)m_len);
            }
            o.put((uint32_t)(m_off << 2));
            o.put((uint32_t)(m_off >> 6));
        }
    }
    return in_end - (ii - ti);
}

// lzo1x_1_compress of one block into out; returns the compressed size
__device__ int64_t lzo1x_1_block(const uint8_t *in, int64_t in_len, uint8_t *out, unsigned short *dict)
{
    LzoOut o{out};
    const uint8_t *ip = in;
    int64_t l = in_len, t = 0;
    while (l > 20) {
        const int64_t ll = l < 49152 ? l : 49152;
        if (((t + ll) >> 5) == 0) break;               // lzo's pointer-overflow guard: t + ll < 32
        for (int k = lane_id(); k < (1 << kLzoDBits) / 2; k += 64) ((uint32_t *)dict)[k] = 0u;
        __builtin_amdgcn_s_waitcnt(0);
        asm volatile("" ::: "memory");
        t = lzo_sub(ip, ll, o, t, dict);
        ip += ll;
        l -= ll;
    }
    t += l;
    if (t > 0) {
        const uint8_t *ii = in + in_len - t;
        if (o.op == out && t <= 238) {
            o.put((uint32_t)(17 + t));
        } else if (t <= 3) {
            o.or_prev2((uint32_t)t);
        } else if (t <= 18) {
            o.put((uint32_t)(t - 3));
        } else {
            int64_t tt = t - 18;
            o.put(0);
            const int64_t nz = tt > 255 ? (tt - 1) / 255 : 0;
            o.zeros(nz);
            tt -= 255 * nz;
            o.put((uint32_t)tt);
        }
        wave_copy(o.op, ii, (int)t);
        o.op += t;
    }
    o.put(16 | 1);
    o.put(0);
    o.put(0);
    return o.op - out;
}

// grid n x 64: block i of the stream -> stage + i * stride; the stored size -> clen[i]
// (the raw bytes when LZO does not shrink them, as LzopOutputStream.compress writes them)
__global__ void __launch_bounds__(64) lzo_list_kernel(const LzPiece *__restrict__ pieces, int n,
                                                      const uint8_t *__restrict__ base, uint8_t *__restrict__ stage,
                                                      uint64_t stride, uint32_t *__restrict__ clen)
{
    __shared__ __attribute__((aligned(16))) unsigned short dict[1 << kLzoDBits];
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzPiece pc = pieces[i];
    uint8_t *out = stage + (size_t)i * stride;
    int64_t c = lzo1x_1_block(base + pc.src, (int64_t)pc.len, out, dict);
    if (c >= (int64_t)pc.len) {                        // not smaller: store the raw bytes
        __threadfence();
        wave_copy(out, base + pc.src, (int)pc.len);
        c = pc.len;
    }
    if (lane_id() == 0) clen[i] = (uint32_t)c;
}

// One LZO1X block per wave (LzopInputStream): raw blocks (stored == raw length) are copied; errors
// (bounds, bad distance, wrong length) set *err.  Wave-uniform parse, wave-wide copies.
__global__ void __launch_bounds__(64) lzo_decode_kernel(const LzDec *__restrict__ items, int n,
                                                        const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                        int *__restrict__ err)
{
    const int i = blockIdx.x;
    if (i >= n) return;
    const LzDec d = items[i];
    const uint8_t *in = src + d.src;
    uint8_t *out = dst + d.dst;
    const int l = lane_id();
    if (d.clen == d.rawlen) {
        wave_copy(out, in, (int)d.rawlen);
        return;
    }
    const int64_t iend = d.clen, oend = d.rawlen;
    int64_t ip = 0, op = 0;
    bool bad = false;
    auto B = [&](int64_t p) -> uint32_t { return p < iend ? rd8(in + p) : 0u; };
    auto lits = [&](int64_t t) {                       // t literals
        if (ip + t > iend || op + t > oend) { bad = true; return; }
        wave_copy(out + op, in + ip, (int)t);
        ip += t;
        op += t;
    };
    auto copy_match = [&](int64_t dist, int64_t len) {
        if (dist <= 0 || dist > op || op + len > oend) { bad = true; return; }
        __threadfence();
        if (dist >= len) {
            wave_copy(out + op, out + op - dist, (int)len);
        } else {
            for (int64_t k = l; k < len; k += 64) wr8(out + op + k, rd8(out + op - dist + (k % dist)));
        }
        __threadfence();
        op += len;
    };
    auto runlen = [&](int64_t t, int64_t add) -> int64_t {   // t == 0: 255-runs then a byte
        if (t != 0) return t;
        while (ip < iend && B(ip) == 0) { t += 255; ip++; }
        if (ip >= iend) { bad = true; return 0; }
        return t + add + (int64_t)B(ip++);
    };
    int64_t t = 0;
    int state;                                          // 0 literal run, 1 first literal run, 2 match, 3 match_next
    if (iend < 1) bad = true;
    if (!bad && B(0) > 17) {
        t = (int64_t)B(ip++) - 17;
        state = t < 4 ? 3 : 4;
    } else {
        state = 0;
    }
    while (!bad) {
        if (state == 4) {                               // first literal run of > 3 bytes
            lits(t);
            if (bad) break;
            if (ip >= iend) { bad = true; break; }
            t = B(ip++);
            if (t >= 16) { state = 2; continue; }
            const int64_t dist = 1 + 0x0800 + (t >> 2) + ((int64_t)B(ip++) << 2);
            copy_match(dist, 3);
            state = 5;
            continue;
        }
        if (state == 0) {
            if (ip >= iend) { bad = true; break; }
            t = B(ip++);
            if (t >= 16) { state = 2; continue; }
            t = runlen(t, 15);
            if (bad) break;
            t += 3;
            state = 4;
            continue;
        }
        if (state == 2) {                               // match with instruction byte t
            int64_t dist, len;
            if (t >= 64) {
                dist = 1 + ((t >> 2) & 7) + ((int64_t)B(ip++) << 3);
                len = (t >> 5) + 1;
            } else if (t >= 32) {
                len = runlen(t & 31, 31) + 2;
                if (bad || ip + 2 > iend) { bad = true; break; }
                dist = 1 + (B(ip) >> 2) + ((int64_t)B(ip + 1) << 6);
                ip += 2;
            } else if (t >= 16) {
                const int64_t hi = (t & 8) << 11;
                len = runlen(t & 7, 7) + 2;
                if (bad || ip + 2 > iend) { bad = true; break; }
                dist = hi + (B(ip) >> 2) + ((int64_t)B(ip + 1) << 6);
                ip += 2;
                if (dist == 0) {                        // end of stream
                    if (len != 3 || ip != iend || op != oend) bad = true;
                    break;
                }
                dist += 0x4000;
            } else {                                    // 2-byte match after a match
                dist = 1 + (t >> 2) + ((int64_t)B(ip++) << 2);
                len = 2;
            }
            copy_match(dist, len);
            state = 5;
            continue;
        }
        if (state == 5) {                               // match_done: trailing literals of the last instruction
            if (ip < 2) { bad = true; break; }
            t = B(ip - 2) & 3;
            if (t == 0) { state = 0; continue; }
            state = 3;
            continue;
        }
        if (state == 3) {                               // match_next: t (1..3) literals, then an instruction
            lits(t);
            if (bad) break;
            if (ip >= iend) { bad = true; break; }
            t = B(ip++);
            state = 2;
            continue;
        }
        bad = true;
    }
    if (bad && l == 0) atomicOr(err, 1);
}

hipError_t launch_lzo_stream(const LzPiece *pieces, int n, const uint8_t *base, uint8_t *stage, uint32_t *clen,
                             hipStream_t st)
{
    if (n > 0)
        hipLaunchKernelGGL(lzo_list_kernel, dim3(n), dim3(64), 0, st, pieces, n, base, stage, lz4_piece_stride(), clen);
    return hipGetLastError();
}

hipError_t launch_lzo_decode(const LzDec *items, int n, const uint8_t *src, uint8_t *dst, int *err, hipStream_t st)
{
    if (n > 0) hipLaunchKernelGGL(lzo_decode_kernel, dim3(n), dim3(64), 0, st, items, n, src, dst, err);
    return hipGetLastError();
}

uint64_t lzo_piece_stride() { return lz4_piece_stride(); }

}  // namespace hdrf
