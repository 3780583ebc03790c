/* hdrf_lzo.c — TEST INFRASTRUCTURE ONLY (the checker for the GPU LZOP path; never linked into
 * libhdrf).  Stream-mode compressor 3 of the reference: the received block written through
 * hadoop-lzo's LzopCodec (DN/BlockReceiver.java:836-845) and read back through its input stream
 * (DN/DataConstructor.java:140-166).
 *
 * Third-party algorithms restated here (neither is in /root/reference nor in this image):
 *   - LZO1X-1, lzo1x_1_compress of LZO 2.10 (lzo1x_1.c + lzo1x_c.ch) as built for x86-64:
 *     LZO_DETERMINISTIC (dictionary of 2^14 u16 offsets cleared for every 49,152-B sub-block,
 *     the carried literal count t), LZO_OPT_UNALIGNED64 match extension (8 bytes at a time,
 *     cut at ip_end = sub-block end - 20), multiplicative hash 0x1824429d >> 18, literal-run
 *     skip ip += 1 + ((ip - ii) >> 5); and the LZO1X decompressor (lzo1x_d.ch) for reading.
 *   - hadoop-lzo 0.4.21-SNAPSHOT (hadoop-hdfs/pom.xml:229) LzopOutputStream: lzop magic,
 *     header {version 0x1010, LZO library version, compat 0x0940, method 1 / level 5 (LZO1X_1),
 *     flags 0, mode 0x81a4, mtime, gmtdiff 0, no file name} + its Adler-32, then per block
 *     [BE32 raw length][BE32 compressed length][bytes] (the raw bytes when LZO does not shrink
 *     them), blocks cut like BlockCompressorStream (MAX_INPUT = 256 KiB - (256 KiB/16 + 67) =
 *     245,693; a write larger than that is cut into MAX_INPUT slices, each its own block), and
 *     close() writes BE32 0.
 * Parity against hadoop-lzo / liblzo2 is UNPINNED (no JDK, no hadoop-lzo jar, no liblzo2 here):
 * the restatement is checked by its own decoder, by the LZO1X format rules, and the GPU output is
 * compared with it byte for byte (tests/test_lzop.py).  The header's mtime (the reference writes
 * the wall clock) is a parameter. */
#include <stdint.h>
#include <string.h>

#define LZO_D_BITS 14
#define LZO_M2_MAX_LEN 8
#define LZO_M2_MAX_OFFSET 0x0800
#define LZO_M3_MAX_OFFSET 0x4000
#define LZO_M3_MAX_LEN 33
#define LZO_M4_MAX_LEN 9
#define LZO_M3_MARKER 32
#define LZO_M4_MARKER 16
#define LZOP_MAX_INPUT 245693
#define LZOP_LIB_VERSION 0x20a0   /* LZO 2.10, the library hadoop-lzo's native code links */

static uint32_t le32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t le64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* lzo1x_c.ch do_compress (deterministic, unaligned-64 variant); returns the literals left */
static size_t lzo_do_compress(const uint8_t *in, size_t in_len, uint8_t *out, size_t *out_len, size_t ti,
                              uint16_t *dict)
{
    const uint8_t *ip = in, *ii = in;
    const uint8_t *const in_end = in + in_len, *const ip_end = in + in_len - 20;
    uint8_t *op = out;
    ip += ti < 4 ? 4 - ti : 0;
    for (;;) {
        const uint8_t *m_pos;
        size_t m_off, m_len;
        {
            uint32_t dv;
            size_t dindex;
        literal:
            ip += 1 + ((size_t)(ip - ii) >> 5);
        next:
            if (ip >= ip_end) break;
            dv = le32(ip);
            dindex = ((uint32_t)(dv * 0x1824429du) >> (32 - LZO_D_BITS)) & ((1u << LZO_D_BITS) - 1);
            m_pos = in + dict[dindex];
            dict[dindex] = (uint16_t)(ip - in);
            if (dv != le32(m_pos)) goto literal;
        }
        ii -= ti;                                        /* a match: literals first */
        ti = 0;
        {
            size_t t = (size_t)(ip - ii);
            if (t != 0) {
                if (t <= 3) {
                    op[-2] = (uint8_t)(op[-2] | t);
                } else if (t <= 18) {
                    *op++ = (uint8_t)(t - 3);
                } else {
                    size_t tt = t - 18;
                    *op++ = 0;
                    while (tt > 255) { tt -= 255; *op++ = 0; }
                    *op++ = (uint8_t)tt;
                }
                memcpy(op, ii, t);
                op += t;
            }
        }
        m_len = 4;
        {
            uint64_t v = le64(ip + m_len) ^ le64(m_pos + m_len);
            if (v == 0) {
                do {
                    m_len += 8;
                    v = le64(ip + m_len) ^ le64(m_pos + m_len);
                    if (ip + m_len >= ip_end) goto m_len_done;
                } while (v == 0);
            }
            m_len += (size_t)__builtin_ctzll(v) / 8;
        }
    m_len_done:
        m_off = (size_t)(ip - m_pos);
        ip += m_len;
        ii = ip;
        if (m_len <= LZO_M2_MAX_LEN && m_off <= LZO_M2_MAX_OFFSET) {
            m_off -= 1;
            *op++ = (uint8_t)(((m_len - 1) << 5) | ((m_off & 7) << 2));
            *op++ = (uint8_t)(m_off >> 3);
        } else if (m_off <= LZO_M3_MAX_OFFSET) {
            m_off -= 1;
            if (m_len <= LZO_M3_MAX_LEN) {
                *op++ = (uint8_t)(LZO_M3_MARKER | (m_len - 2));
            } else {
                m_len -= LZO_M3_MAX_LEN;
                *op++ = LZO_M3_MARKER | 0;
                while (m_len > 255) { m_len -= 255; *op++ = 0; }
                *op++ = (uint8_t)m_len;
            }
            *op++ = (uint8_t)(m_off << 2);
            *op++ = (uint8_t)(m_off >> 6);
        } else {
            m_off -= 0x4000;
            if (m_len <= LZO_M4_MAX_LEN) {
                *op++ = (uint8_t)(LZO_M4_MARKER | ((m_off >> 11) & 8) | (m_len - 2));
            } else {
                m_len -= LZO_M4_MAX_LEN;
                *op++ = (uint8_t)(LZO_M4_MARKER | ((m_off >> 11) & 8));
                while (m_len > 255) { m_len -= 255; *op++ = 0; }
                *op++ = (uint8_t)m_len;
            }
            *op++ = (uint8_t)(m_off << 2);
            *op++ = (uint8_t)(m_off >> 6);
        }
        goto next;
    }
    *out_len = (size_t)(op - out);
    return (size_t)(in_end - (ii - ti));
}

/* lzo1x_1_compress: worst case n + n/16 + 64 + 3 bytes */
int64_t hdrf_oracle_lzo1x_1_compress(const uint8_t *in, int64_t in_len, uint8_t *out)
{
    static __thread uint16_t dict[1u << LZO_D_BITS];
    const uint8_t *ip = in;
    uint8_t *op = out;
    size_t l = (size_t)in_len, t = 0;
    while (l > 20) {
        const size_t ll = l < 49152 ? l : 49152;
        if (((t + ll) >> 5) == 0) break;                 /* lzo's pointer-overflow guard, true iff t + ll < 32 */
        memset(dict, 0, sizeof dict);
        size_t ol = 0;
        t = lzo_do_compress(ip, ll, op, &ol, t, dict);
        ip += ll;
        op += ol;
        l -= ll;
    }
    t += l;
    if (t > 0) {
        const uint8_t *ii = in + in_len - t;
        if (op == out && t <= 238) {
            *op++ = (uint8_t)(17 + t);
        } else if (t <= 3) {
            op[-2] = (uint8_t)(op[-2] | t);
        } else if (t <= 18) {
            *op++ = (uint8_t)(t - 3);
        } else {
            size_t tt = t - 18;
            *op++ = 0;
            while (tt > 255) { tt -= 255; *op++ = 0; }
            *op++ = (uint8_t)tt;
        }
        memcpy(op, ii, t);
        op += t;
    }
    *op++ = LZO_M4_MARKER | 1;
    *op++ = 0;
    *op++ = 0;
    return (int64_t)(op - out);
}

/* lzo1x_decompress_safe: returns the decoded length, or -1 on malformed input / overrun */
int64_t hdrf_oracle_lzo1x_decompress(const uint8_t *in, int64_t in_len, uint8_t *out, int64_t cap)
{
    const uint8_t *ip = in, *const ip_end = in + in_len;
    uint8_t *op = out, *const op_end = out + cap;
    size_t t;
    const uint8_t *m_pos;
#define NEED_IP(x) do { if ((size_t)(ip_end - ip) < (size_t)(x)) return -1; } while (0)
#define NEED_OP(x) do { if ((size_t)(op_end - op) < (size_t)(x)) return -1; } while (0)
#define LB_CHECK() do { if (m_pos < out || m_pos >= op) return -1; } while (0)
    NEED_IP(1);
    if (*ip > 17) {
        t = (size_t)(*ip++ - 17);
        if (t < 4) goto match_next;
        NEED_OP(t); NEED_IP(t + 3);
        do *op++ = *ip++; while (--t > 0);
        goto first_literal_run;
    }
    for (;;) {
        NEED_IP(3);
        t = *ip++;
        if (t >= 16) goto match;
        if (t == 0) {
            while (*ip == 0) { t += 255; ip++; NEED_IP(1); }
            t += 15 + *ip++;
        }
        NEED_OP(t + 3); NEED_IP(t + 6);
        for (size_t k = 0; k < t + 3; k++) *op++ = *ip++;
    first_literal_run:
        t = *ip++;
        if (t >= 16) goto match;
        m_pos = op - (1 + LZO_M2_MAX_OFFSET);
        m_pos -= t >> 2;
        m_pos -= *ip++ << 2;
        LB_CHECK(); NEED_OP(3);
        *op++ = *m_pos++; *op++ = *m_pos++; *op++ = *m_pos;
        goto match_done;
        for (;;) {
        match:
            if (t >= 64) {
                m_pos = op - 1;
                m_pos -= (t >> 2) & 7;
                m_pos -= *ip++ << 3;
                t = (t >> 5) - 1;
                LB_CHECK(); NEED_OP(t + 2);
                goto copy_match;
            } else if (t >= 32) {
                t &= 31;
                if (t == 0) {
                    while (*ip == 0) { t += 255; ip++; NEED_IP(1); }
                    t += 31 + *ip++;
                    NEED_IP(2);
                }
                m_pos = op - 1;
                m_pos -= (ip[0] >> 2) + (ip[1] << 6);
                ip += 2;
            } else if (t >= 16) {
                m_pos = op;
                m_pos -= (t & 8) << 11;
                t &= 7;
                if (t == 0) {
                    while (*ip == 0) { t += 255; ip++; NEED_IP(1); }
                    t += 7 + *ip++;
                    NEED_IP(2);
                }
                m_pos -= (ip[0] >> 2) + (ip[1] << 6);
                ip += 2;
                if (m_pos == op) goto eof_found;
                m_pos -= 0x4000;
            } else {
                m_pos = op - 1;
                m_pos -= t >> 2;
                m_pos -= *ip++ << 2;
                LB_CHECK(); NEED_OP(2);
                *op++ = *m_pos++; *op++ = *m_pos;
                goto match_done;
            }
            LB_CHECK(); NEED_OP(t + 2);
        copy_match:
            for (size_t k = 0; k < t + 2; k++) *op++ = *m_pos++;
        match_done:
            t = ip[-2] & 3;
            if (t == 0) break;
        match_next:
            NEED_OP(t); NEED_IP(t + 3);
            do *op++ = *ip++; while (--t > 0);
            t = *ip++;
        }
    }
eof_found:
    if (t != 1 || ip != ip_end) return -1;
    return (int64_t)(op - out);
#undef NEED_IP
#undef NEED_OP
#undef LB_CHECK
}

static uint32_t adler32(const uint8_t *p, size_t n)
{
    uint32_t a = 1, b = 0;
    for (size_t i = 0; i < n; i++) { a = (a + p[i]) % 65521u; b = (b + a) % 65521u; }
    return (b << 16) | a;
}
static uint8_t *be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
    return p + 4;
}

/* LzopOutputStream.writeLzopHeader (34 bytes + 4 B checksum after the 9-B magic = 47 bytes) */
int64_t hdrf_oracle_lzop_header(uint32_t mtime, uint8_t *dst)
{
    static const uint8_t magic[9] = {0x89, 'L', 'Z', 'O', 0x00, 0x0d, 0x0a, 0x1a, 0x0a};
    uint8_t h[64], *p = h;
    *p++ = 0x10; *p++ = 0x10;                                        /* LZOP_VERSION 0x1010 */
    *p++ = (uint8_t)(LZOP_LIB_VERSION >> 8); *p++ = (uint8_t)LZOP_LIB_VERSION;
    *p++ = 0x09; *p++ = 0x40;                                        /* LZOP_COMPAT_VERSION 0x0940 */
    *p++ = 1; *p++ = 5;                                              /* LZO1X_1: method 1, level 5 */
    p = be32(p, 0);                                                  /* flags */
    p = be32(p, 0x81a4);                                             /* mode */
    p = be32(p, mtime);
    p = be32(p, 0);                                                  /* gmtdiff */
    *p++ = 0;                                                        /* no file name */
    p = be32(p, adler32(h, (size_t)(p - h)));
    memcpy(dst, magic, 9);
    memcpy(dst + 9, h, (size_t)(p - h));
    return 9 + (int64_t)(p - h);
}

int64_t hdrf_oracle_lzop_stream_bound(int64_t n, int64_t nwrites)
{
    return 64 + n + n / 16 + (n / LZOP_MAX_INPUT + nwrites + 2) * (8 + 64 + 3) + 4;
}

static uint8_t *lzop_block(const uint8_t *src, int64_t n, uint8_t *dst)
{
    uint8_t *p = be32(dst, (uint32_t)n);
    const int64_t c = hdrf_oracle_lzo1x_1_compress(src, n, p + 4);
    if (n <= c) {                                                    /* not smaller: the raw bytes */
        p = be32(p, (uint32_t)n);
        memcpy(p, src, (size_t)n);
        return p + n;
    }
    p = be32(p, (uint32_t)c);
    return p + c;
}

/* The LzopCodec output stream of one block written as writes[0..nwrites) then closed */
int64_t hdrf_oracle_lzop_stream(const uint8_t *src, const int64_t *writes, int64_t nwrites, uint32_t mtime,
                                uint8_t *dst)
{
    uint8_t *p = dst + hdrf_oracle_lzop_header(mtime, dst);
    int64_t off = 0, gs = 0, lim = 0;
    for (int64_t w = 0; w < nwrites; w++) {
        int64_t n = writes[w];
        if (n == 0) continue;
        if (lim > 0 && n + lim > LZOP_MAX_INPUT) { p = lzop_block(src + gs, lim, p); lim = 0; }   /* finish() */
        if (n > LZOP_MAX_INPUT) {                                    /* sliced write, a block per slice */
            for (int64_t o = 0; o < n; o += LZOP_MAX_INPUT)
                p = lzop_block(src + off + o, n - o < LZOP_MAX_INPUT ? n - o : LZOP_MAX_INPUT, p);
            off += n;
            continue;
        }
        if (lim == 0) gs = off;
        lim += n;
        off += n;
    }
    if (lim > 0) p = lzop_block(src + gs, lim, p);
    p = be32(p, 0);                                                  /* close() */
    return (int64_t)(p - dst);
}

/* LzopInputStream: header checks, then the blocks; returns the decoded length or -1 */
int64_t hdrf_oracle_lzop_decode(const uint8_t *f, int64_t n, uint8_t *dst, int64_t cap)
{
    static const uint8_t magic[9] = {0x89, 'L', 'Z', 'O', 0x00, 0x0d, 0x0a, 0x1a, 0x0a};
    if (n < 9 + 38 || memcmp(f, magic, 9) != 0) return -1;
    const uint8_t *h = f + 9;
    const uint32_t flags = ((uint32_t)h[8] << 24) | ((uint32_t)h[9] << 16) | ((uint32_t)h[10] << 8) | h[11];
    if (h[6] != 1 && h[6] != 2 && h[6] != 3) return -1;
    const int fname = h[24];
    int64_t pos = 9 + 25 + fname;
    if (pos + 4 > n) return -1;
    const uint32_t hc = ((uint32_t)f[pos] << 24) | ((uint32_t)f[pos + 1] << 16) | ((uint32_t)f[pos + 2] << 8) | f[pos + 3];
    if (hc != adler32(h, (size_t)(25 + fname))) return -1;
    pos += 4;
    if (flags & 0x40) return -1;                                     /* F_H_EXTRA_FIELD: not written by hadoop-lzo */
    const int dck = ((flags & 1) != 0) + ((flags & 0x100) != 0), cck = ((flags & 2) != 0) + ((flags & 0x200) != 0);
    int64_t out = 0;
    for (;;) {
        if (pos + 4 > n) return -1;
        const uint32_t ul = ((uint32_t)f[pos] << 24) | ((uint32_t)f[pos + 1] << 16) | ((uint32_t)f[pos + 2] << 8) | f[pos + 3];
        pos += 4;
        if (ul == 0) break;
        if (pos + 4 > n) return -1;
        const uint32_t cl = ((uint32_t)f[pos] << 24) | ((uint32_t)f[pos + 1] << 16) | ((uint32_t)f[pos + 2] << 8) | f[pos + 3];
        pos += 4 + 4 * (int64_t)dck + (cl < ul ? 4 * (int64_t)cck : 0);
        if (cl > ul || pos + cl > n || out + ul > cap) return -1;
        if (cl == ul) {
            memcpy(dst + out, f + pos, ul);
        } else if (hdrf_oracle_lzo1x_decompress(f + pos, cl, dst + out, ul) != (int64_t)ul) {
            return -1;
        }
        pos += cl;
        out += ul;
    }
    return pos == n ? out : -1;
}
