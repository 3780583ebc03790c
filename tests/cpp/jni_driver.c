/* jni_driver.c — runs integration/jni/hdrf_jni.c (the binding a DataNode's HipReductionScheme loads)
 * through a working JNIEnv function table, the way the DataNode hooks of INTEGRATION.md §2 call it,
 * and checks everything it hands back against the CPU oracle.  Test infrastructure (links the oracle).
 *
 *   jni_driver <compressor 1|2> <chunkDir prefix, e.g. /tmp/x/> [block MiB] [blocks]
 *
 * The context is the JNI's own (open0: 256 arena slots, retain_containers, 16-block batches).
 *   phase A  BlockReceiver + DDRunner (DN/BlockReceiver.java:1258-1261, DN/DDRunner.java:26-36): a ticket
 *            per block at arrival (arrive0), the reductions on one thread per block started in
 *            REVERSE order (reduceTicket0): the FIFO of DN/DataDeduplicator.java:124-158 decides
 *   phase B  packet receive (DN/BlockReceiver.java:877-896): rxBegin0 / packet0 (64,512-B payloads at
 *            an offset into the packet buffer) / submitSlots0 per round of three, wait0
 *   phase C  reduceAsync (submit0 from allocPinned0 buffers, three in flight), wait0
 *   drain0 into chunkDir after every completed batch (the storers' file writes, :748-818)
 * Checks: every chunkDir file equals the oracle's container file (raw, or Lz4Codec when closed under
 * compressor 2), recipe0 / length0 / reconstruct0 of every block, stream0 + streamDecode0 for codecs 4
 * and 0, and the argument checks (a packet range outside its buffer, a too-long submitBlocks list, an
 * unknown block) raise the mock's IOException. */
#define _GNU_SOURCE
#include <jni.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hdrf.h"
#include "hdrf_oracle.h"

/* ---- the mock VM: objects, arrays, strings, one pending exception per thread -------------- */
enum { K_CLASS = 1, K_DIRECT, K_BYTES, K_INTS, K_LONGS, K_STRING };
struct _jobject {
    int kind;
    void *p;
    jlong len;          /* capacity (direct buffer) or element count (arrays) */
    int owned;
};
static _Thread_local int t_exc;
static _Thread_local char t_msg[600];
static int g_fail;

static jobject mk(int kind, void *p, jlong len, int owned)
{
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof *o);
    o->kind = kind; o->p = p; o->len = len; o->owned = owned;
    return o;
}
static void rel(jobject o)
{
    if (!o) return;
    if (o->owned) free(o->p);
    free(o);
}

static jclass m_FindClass(JNIEnv *e, const char *n) { (void)e; static struct _jobject c = {K_CLASS, 0, 0, 0}; c.p = (void *)n; return &c; }
static jint m_ThrowNew(JNIEnv *e, jclass c, const char *msg)
{
    (void)e;
    t_exc = 1;
    snprintf(t_msg, sizeof t_msg, "%s: %s", c && c->p ? (const char *)c->p : "?", msg);
    return 0;
}
static void *m_GetDirectBufferAddress(JNIEnv *e, jobject b) { (void)e; return b && b->kind == K_DIRECT ? b->p : NULL; }
static jlong m_GetDirectBufferCapacity(JNIEnv *e, jobject b) { (void)e; return b && b->kind == K_DIRECT ? b->len : -1; }
static jsize m_GetArrayLength(JNIEnv *e, jarray a) { (void)e; return (jsize)a->len; }
static jlong *m_GetLongArrayElements(JNIEnv *e, jlongArray a, unsigned char *c) { (void)e; if (c) *c = 0; return (jlong *)a->p; }
static void m_ReleaseLongArrayElements(JNIEnv *e, jlongArray a, jlong *x, jint m) { (void)e; (void)a; (void)x; (void)m; }
static jint *m_GetIntArrayElements(JNIEnv *e, jintArray a, jboolean *c) { (void)e; if (c) *c = 0; return (jint *)a->p; }
static void m_ReleaseIntArrayElements(JNIEnv *e, jintArray a, jint *x, jint m) { (void)e; (void)a; (void)x; (void)m; }
static jbyteArray m_NewByteArray(JNIEnv *e, jsize n) { (void)e; return mk(K_BYTES, calloc(1, (size_t)n + 1), n, 1); }
static void m_SetByteArrayRegion(JNIEnv *e, jbyteArray a, jsize s, jsize n, const jbyte *b)
{
    (void)e;
    if (s < 0 || n < 0 || (jlong)s + n > a->len) { t_exc = 1; snprintf(t_msg, sizeof t_msg, "ArrayIndexOutOfBounds"); return; }
    memcpy((jbyte *)a->p + s, b, (size_t)n);
}
static const char *m_GetStringUTFChars(JNIEnv *e, jstring s, jboolean *c) { (void)e; if (c) *c = 0; return (const char *)s->p; }
static void m_ReleaseStringUTFChars(JNIEnv *e, jstring s, const char *u) { (void)e; (void)s; (void)u; }
static jobject m_NewDirectByteBuffer(JNIEnv *e, void *a, jlong cap) { (void)e; return mk(K_DIRECT, a, cap, 0); }
static jbyte *m_GetByteArrayElements(JNIEnv *e, jbyteArray a, jboolean *c) { (void)e; if (c) *c = 0; return (jbyte *)a->p; }
static void m_ReleaseByteArrayElements(JNIEnv *e, jbyteArray a, jbyte *x, jint m) { (void)e; (void)a; (void)x; (void)m; }

static const struct JNINativeInterface_ g_table = {
    m_FindClass, m_ThrowNew, m_GetDirectBufferAddress, m_GetDirectBufferCapacity, m_GetArrayLength,
    m_GetLongArrayElements, m_ReleaseLongArrayElements, m_GetIntArrayElements, m_ReleaseIntArrayElements,
    m_NewByteArray, m_SetByteArrayRegion, m_GetStringUTFChars, m_ReleaseStringUTFChars, m_NewDirectByteBuffer,
    m_GetByteArrayElements, m_ReleaseByteArrayElements,
};
static const struct JNINativeInterface_ *g_envp = &g_table;
#define ENV ((JNIEnv *)&g_envp)

/* ---- the shim's entry points (integration/jni/hdrf_jni.c) --------------------------------- */
#define JFN(name) Java_org_apache_hadoop_hdfs_server_datanode_HipReductionScheme_##name
jlong JFN(open0)(JNIEnv *, jclass, jint, jint, jint, jlong, jint);
jlong JFN(arrive0)(JNIEnv *, jclass, jlong);
void JFN(reduceTicket0)(JNIEnv *, jclass, jlong, jlong, jobject, jint, jlong);
jint JFN(drain0)(JNIEnv *, jclass, jlong, jstring);
jobject JFN(allocPinned0)(JNIEnv *, jclass, jlong, jlong);
void JFN(freePinned0)(JNIEnv *, jclass, jlong, jobject);
jint JFN(rxBegin0)(JNIEnv *, jclass, jlong, jlong);
void JFN(packet0)(JNIEnv *, jclass, jlong, jint, jobject, jint, jint);
void JFN(submitSlots0)(JNIEnv *, jclass, jlong, jintArray);
void JFN(submit0)(JNIEnv *, jclass, jlong, jobject, jint, jlong);
void JFN(wait0)(JNIEnv *, jclass, jlong);
jlong JFN(length0)(JNIEnv *, jclass, jlong, jlong);
jbyteArray JFN(recipe0)(JNIEnv *, jclass, jlong, jlong);
jbyteArray JFN(reconstruct0)(JNIEnv *, jclass, jlong, jlong);
jbyteArray JFN(stream0)(JNIEnv *, jclass, jlong, jint, jobject, jint, jlong, jlongArray);
jbyteArray JFN(streamDecode0)(JNIEnv *, jclass, jlong, jint, jbyteArray, jlong);
void JFN(close0)(JNIEnv *, jclass, jlong);

#define CHECK_OK(what)                                                                  \
    do {                                                                                \
        if (t_exc) { printf("unexpected exception in %s: %s\n", what, t_msg); g_fail++; t_exc = 0; } \
    } while (0)
#define EXPECT_THROW(what)                                                              \
    do {                                                                                \
        if (!t_exc) { printf("no exception from %s\n", what); g_fail++; }               \
        else printf("%s -> %s\n", what, t_msg);                                         \
        t_exc = 0;                                                                      \
    } while (0)

/* ---- blocks: 1 MiB segments, half of them copies of an earlier block's (the bench corpus), every
 * third block mapped onto a text alphabet so compressor 2's LZ4 finds matches ------------------- */
static uint8_t **g_blk;
static int64_t *g_len;
static void make_blocks(int nblk, int64_t S)
{
    const int64_t seg = 1 << 20, spb = S / seg;
    uint32_t *roots = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(nblk * spb));
    hdrf_oracle_corpus_roots(91, 500000, nblk, spb, roots);
    static const char alpha[] = "etaoinshrdlucmfwypvbgkjqxz ETAOIN.,\n0123456789";
    g_blk = (uint8_t **)calloc((size_t)nblk, sizeof *g_blk);
    g_len = (int64_t *)calloc((size_t)nblk, sizeof *g_len);
    for (int b = 0; b < nblk; b++) {
        g_blk[b] = (uint8_t *)malloc((size_t)S);
        hdrf_oracle_corpus_fill(91, roots, b, spb, seg, g_blk[b]);
        if (b % 3 == 2)
            for (int64_t i = 0; i < S; i++) g_blk[b][i] = (uint8_t)alpha[g_blk[b][i] % (sizeof alpha - 1)];
        g_len[b] = b % 4 == 1 ? S - 1000 * b - 7 : S;            /* ragged lengths too */
    }
    free(roots);
}

/* ---- phase A: DDRunner threads ----------------------------------------------------------- */
struct Job { jlong h, ticket, id; int b; };
static void *ddrunner(void *arg)
{
    struct Job *j = (struct Job *)arg;
    jobject buf = mk(K_DIRECT, g_blk[j->b], g_len[j->b], 0);
    JFN(reduceTicket0)(ENV, NULL, j->h, j->ticket, buf, (jint)g_len[j->b], j->id);
    CHECK_OK("reduceTicket0");
    rel(buf);
    return NULL;
}

static int drain(jlong h, const char *dir)
{
    jobject s = mk(K_STRING, (void *)dir, 0, 0);
    jint n = JFN(drain0)(ENV, NULL, h, s);
    CHECK_OK("drain0");
    rel(s);
    return n;
}

static uint8_t *read_file(const char *path, int64_t *n)
{
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *p = (uint8_t *)malloc((size_t)*n + 1);
    if (fread(p, 1, (size_t)*n, f) != (size_t)*n) *n = -1;
    fclose(f);
    return p;
}

int main(int argc, char **argv)
{
    if (argc < 3) { fprintf(stderr, "usage: %s compressor chunkDir/ [block_mib] [blocks]\n", argv[0]); return 2; }
    const int compressor = atoi(argv[1]);
    const char *dir = argv[2];
    const int64_t S = (argc > 3 ? atoll(argv[3]) : 16) << 20;
    const int nblk = argc > 4 ? atoi(argv[4]) : 18;
    const int nA = nblk / 3, nB = nblk / 3;
    make_blocks(nblk, S);
    const jlong h = JFN(open0)(ENV, NULL, 0, compressor, 0, S, 16);
    CHECK_OK("open0");
    if (!h) { printf("FAIL open\n"); return 1; }
    int *order = (int *)malloc(sizeof(int) * (size_t)nblk), no = 0, nev = 0;
    jlong *ids = (jlong *)malloc(sizeof(jlong) * (size_t)nblk);
    for (int b = 0; b < nblk; b++) ids[b] = 0x7000 + 11 * b;

    /* phase A: tickets in arrival order, reductions on threads started in reverse order */
    struct Job *jobs = (struct Job *)calloc((size_t)nA, sizeof *jobs);
    for (int b = 0; b < nA; b++) {
        jobs[b] = (struct Job){h, JFN(arrive0)(ENV, NULL, h), ids[b], b};
        CHECK_OK("arrive0");
        order[no++] = b;
    }
    pthread_t *th = (pthread_t *)calloc((size_t)nA, sizeof *th);
    for (int b = nA - 1; b >= 0; b--) pthread_create(&th[b], NULL, ddrunner, &jobs[b]);
    for (int b = 0; b < nA; b++) pthread_join(th[b], NULL);
    nev += drain(h, dir);

    /* phase B: packets, a receive round of up to three blocks per submitBlocks() */
    const jint P = 64512;                                         /* an HDFS packet's data payload */
    uint8_t *pkt = (uint8_t *)malloc((size_t)P + 4096);
    jobject pbuf = mk(K_DIRECT, pkt, P + 4096, 0);
    int pend = 0;
    for (int b0 = nA; b0 < nA + nB; b0 += 3) {
        const int k = nA + nB - b0 < 3 ? nA + nB - b0 : 3;
        jint rx[3];
        for (int i = 0; i < k; i++) { rx[i] = JFN(rxBegin0)(ENV, NULL, h, ids[b0 + i]); CHECK_OK("rxBegin0"); }
        for (int64_t o = 0;; o += P) {                            /* the blocks' packets interleaved */
            int any = 0;
            for (int i = 0; i < k; i++) {
                const int b = b0 + i;
                if (o >= g_len[b]) continue;
                const jint n = (jint)(g_len[b] - o < P ? g_len[b] - o : P);
                const jint off = (jint)((o / P) % 7) * 512;       /* the payload sits at an offset */
                memcpy(pkt + off, g_blk[b] + o, (size_t)n);
                JFN(packet0)(ENV, NULL, h, rx[i], pbuf, off, n);
                CHECK_OK("packet0");
                memset(pkt + off, 0xA5, (size_t)n);               /* the buffer is reused at once */
                any = 1;
            }
            if (!any) break;
        }
        if (b0 == nA) {                                           /* argument checks on a live receive */
            JFN(packet0)(ENV, NULL, h, rx[0], pbuf, 4000, P);     /* off + len past the buffer */
            EXPECT_THROW("packet0(range past the direct buffer)");
            JFN(packet0)(ENV, NULL, h, rx[0], pbuf, 0, -5);
            EXPECT_THROW("packet0(negative length)");
            jint big[17];
            for (int i = 0; i < 17; i++) big[i] = rx[0];
            jobject a17 = mk(K_INTS, big, 17, 0);
            JFN(submitSlots0)(ENV, NULL, h, a17);
            EXPECT_THROW("submitSlots0(17 buffers)");
            rel(a17);
        }
        jobject arr = mk(K_INTS, rx, k, 0);
        JFN(submitSlots0)(ENV, NULL, h, arr);
        CHECK_OK("submitSlots0");
        rel(arr);
        for (int i = 0; i < k; i++) order[no++] = b0 + i;
        if (++pend == 2) { JFN(wait0)(ENV, NULL, h); CHECK_OK("wait0"); pend--; nev += drain(h, dir); }
    }
    while (pend) { JFN(wait0)(ENV, NULL, h); CHECK_OK("wait0"); pend--; nev += drain(h, dir); }

    /* phase C: reduceAsync from pinned buffers, three in flight */
    jobject *pin = (jobject *)calloc((size_t)nblk, sizeof *pin);
    for (int b = nA + nB; b < nblk; b++) {
        pin[b] = JFN(allocPinned0)(ENV, NULL, h, S);
        CHECK_OK("allocPinned0");
        memcpy(pin[b]->p, g_blk[b], (size_t)g_len[b]);
        JFN(submit0)(ENV, NULL, h, pin[b], (jint)g_len[b], ids[b]);
        CHECK_OK("submit0");
        order[no++] = b;
        if (++pend == 3) { JFN(wait0)(ENV, NULL, h); CHECK_OK("wait0"); pend--; nev += drain(h, dir); }
    }
    while (pend) { JFN(wait0)(ENV, NULL, h); CHECK_OK("wait0"); pend--; nev += drain(h, dir); }
    nev += drain(h, dir);
    printf("reduced %d blocks (%d ticketed, %d packet-received, %d async); %d chunkDir writes\n", no, nA, nB,
           nblk - nA - nB, nev);

    /* the oracle in the same order */
    hdrf_oracle *ora = hdrf_oracle_new(0, compressor, 1u << 25);
    for (int i = 0; i < no; i++) {
        const int b = order[i];
        int64_t ss = 0;
        if (hdrf_oracle_reduce(ora, g_blk[b], g_len[b], ids[b], g_len[b] / 702 + 2, NULL, NULL, NULL, NULL, &ss) < 0) g_fail++;
    }
    /* every container file of chunkDir == the oracle's */
    uint8_t alloc[24];
    int nfiles = 0, closed_files = 0;
    if (hdrf_oracle_allocator(ora, alloc) == 1)
        for (int t = 0; t < 3; t++) {
            const uint32_t last = (uint32_t)alloc[3 * t] << 16 | (uint32_t)alloc[3 * t + 1] << 8 | alloc[3 * t + 2];
            for (uint32_t cid = (uint32_t)t << 22; cid <= last; cid++) {
                int closed = 0;
                const int64_t r0 = hdrf_oracle_container(ora, cid, NULL, 0, &closed);
                if (r0 == -1) continue;                           /* never written */
                const int64_t cap = r0 >= 0 ? r0 : -r0 - 2;
                uint8_t *od = (uint8_t *)malloc((size_t)cap + 1);
                (void)cap;
                const int64_t on = hdrf_oracle_container(ora, cid, od, cap, &closed);
                char path[4200];
                snprintf(path, sizeof path, "%s%u", dir, cid);
                int64_t gn = -1;
                uint8_t *gd = read_file(path, &gn);
                const int ok = gd && gn == on && memcmp(gd, od, (size_t)on) == 0;
                if (!ok) {
                    printf("container %#x: file %s (%lld B) vs oracle %lld B%s\n", cid, gd ? "differs" : "missing",
                           (long long)gn, (long long)on, closed ? " (closed)" : "");
                    g_fail++;
                }
                nfiles++;
                closed_files += closed;
                free(gd);
                free(od);
            }
        }
    printf("chunkDir: %d container files equal the oracle's (%d closed)\n", nfiles, closed_files);
    if (closed_files == 0) { printf("no container closed: the test does not reach the close path\n"); g_fail++; }

    /* recipe0 / length0 / reconstruct0 of every block */
    for (int b = 0; b < nblk; b++) {
        const jlong n = JFN(length0)(ENV, NULL, h, ids[b]);
        CHECK_OK("length0");
        jbyteArray r = JFN(recipe0)(ENV, NULL, h, ids[b]);
        CHECK_OK("recipe0");
        const int64_t rn = hdrf_oracle_recipe(ora, ids[b], NULL, 0);
        uint8_t *orc = (uint8_t *)malloc((size_t)(rn < 0 ? -rn : rn) + 1);
        const int64_t rl = hdrf_oracle_recipe(ora, ids[b], orc, rn < 0 ? -rn : rn);
        const int rok = r && r->len == rl && memcmp(r->p, orc, (size_t)rl) == 0;
        jbyteArray d = JFN(reconstruct0)(ENV, NULL, h, ids[b]);
        CHECK_OK("reconstruct0");
        const int dok = d && d->len == g_len[b] && memcmp(d->p, g_blk[b], (size_t)g_len[b]) == 0;
        if (n != g_len[b] || !rok || !dok) {
            printf("block %d: length %lld/%lld recipe %s reconstruct %s\n", b, (long long)n, (long long)g_len[b],
                   rok ? "ok" : "DIFFERS", dok ? "ok" : "DIFFERS");
            g_fail++;
        }
        free(orc);
        rel(r);
        rel(d);
    }
    JFN(length0)(ENV, NULL, h, 0x7fffffff);
    EXPECT_THROW("length0(unknown block)");
    jbyteArray none = JFN(reconstruct0)(ENV, NULL, h, 0x7fffffff);
    EXPECT_THROW("reconstruct0(unknown block)");
    rel(none);
    jbyteArray nor = JFN(recipe0)(ENV, NULL, h, 0x7fffffff);
    EXPECT_THROW("recipe0(unknown block)");
    if (nor) { printf("recipe0(unknown block) returned an array\n"); g_fail++; }

    /* stream mode (compressor 4 / 0): the block file for 64,512-B packet writes, and its GPU decode */
    const int codecs[2] = {4, 0};
    for (int ci = 0; ci < 2; ci++) {
        const int b = 2, codec = codecs[ci];
        const int64_t L = g_len[b], nw = (L + P - 1) / P;
        jlong *w = (jlong *)malloc(sizeof(jlong) * (size_t)nw);
        int64_t *w64 = (int64_t *)malloc(sizeof(int64_t) * (size_t)nw);
        for (int64_t i = 0; i < nw; i++) w[i] = w64[i] = (i + 1) * P <= L ? P : L - i * P;
        jobject buf = mk(K_DIRECT, g_blk[b], L, 0);
        jlongArray wa = mk(K_LONGS, w, nw, 0);
        const jlong sid = 0x9000 + codec;
        jbyteArray f = JFN(stream0)(ENV, NULL, h, codec, buf, (jint)L, sid, wa);
        CHECK_OK("stream0");
        const int64_t ob = hdrf_oracle_hadoop_stream_bound(codec, L, nw);
        uint8_t *of = (uint8_t *)malloc((size_t)ob);
        const int64_t on = hdrf_oracle_hadoop_stream(codec, g_blk[b], w64, nw, of);
        const int fok = f && f->len == on && memcmp(f->p, of, (size_t)on) == 0;
        jbyteArray d = f ? JFN(streamDecode0)(ENV, NULL, h, codec, f, sid) : NULL;
        CHECK_OK("streamDecode0");
        const int dok = d && d->len == L && memcmp(d->p, g_blk[b], (size_t)L) == 0;
        printf("stream codec %d: file %lld B %s, decode %s\n", codec, (long long)(f ? f->len : -1),
               fok ? "= oracle" : "DIFFERS", dok ? "ok" : "DIFFERS");
        g_fail += !fok + !dok;
        free(w); free(w64); free(of);
        rel(buf); rel(wa); rel(f); rel(d);
    }

    for (int b = nA + nB; b < nblk; b++) {
        JFN(freePinned0)(ENV, NULL, h, pin[b]);
        CHECK_OK("freePinned0");
        rel(pin[b]);
    }
    JFN(close0)(ENV, NULL, h);
    hdrf_oracle_free(ora);
    rel(pbuf);
    printf(g_fail ? "FAIL (%d)\n" : "PASS\n", g_fail);
    return g_fail ? 1 : 0;
}
