/* hdrf_jni.c — JNI shim for HipReductionScheme over libhdrf.so (C-ABI in include/hdrf.h).
 * Build (on a host with a JDK):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      integration/jni/hdrf_jni.c -Lhdrf_amd/_build -lhdrf -o libhdrf_jni.so
 * Errors become IOException; DDRunner-style callers may log and continue (DDRunner.java:27-31). */
#define _FILE_OFFSET_BITS 64
#define _POSIX_C_SOURCE 200809L
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "hdrf.h"

static void throw_io(JNIEnv *env, hdrf_ctx *ctx, int rc)
{
    char msg[512];
    snprintf(msg, sizeof msg, "hdrf error %d: %s", rc, ctx ? hdrf_last_error(ctx) : "open failed");
    jclass c = (*env)->FindClass(env, "java/io/IOException");
    if (c) (*env)->ThrowNew(env, c, msg);
}

#define JFN(name) Java_org_apache_hadoop_hdfs_server_datanode_HipReductionScheme_##name

JNIEXPORT jlong JNICALL JFN(open0)(JNIEnv *env, jclass cls, jint hasher, jint compressor, jint device,
                                   jlong max_block, jint max_batch)
{
    (void)cls;
    hdrf_cfg cfg;
    hdrf_default_cfg(&cfg);
    cfg.hasher = hasher;              /* DataNode.hasher  (DataNode.java:446) */
    cfg.compressor = compressor;      /* 1 dedup, 2 dedup + Lz4Codec (DataNode.java:438) */
    cfg.arena_slots = 256;            /* 64 containers per storer range resident (8 GiB of HBM) */
    cfg.retain_containers = 1;        /* durable: nothing leaves HBM before drain0 wrote its file */
    cfg.device = device;
    cfg.max_block_bytes = max_block;  /* dfs.blocksize */
    cfg.max_batch_blocks = max_batch; /* blocks per submitBlocks() batch (1..64; 16 receive buffers) */
    hdrf_ctx *ctx = NULL;
    int rc = hdrf_open(&cfg, &ctx);
    if (rc) { throw_io(env, NULL, rc); return 0; }
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL JFN(reduce0)(JNIEnv *env, jclass cls, jlong h, jobject buf, jint len, jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const uint8_t *p = (const uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    if (!p) { throw_io(env, ctx, HDRF_E_INVAL); return; }
    int rc = hdrf_reduce_block(ctx, (uint64_t)id, p, (uint64_t)len, NULL);
    if (rc) throw_io(env, ctx, rc);
}

/* BlockReceiver, at block arrival: the block's place in the FIFO (AIWriteQueue,
 * DataDeduplicator.java:124-158) */
JNIEXPORT jlong JNICALL JFN(arrive0)(JNIEnv *env, jclass cls, jlong h)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    uint64_t t = 0;
    int rc = hdrf_ticket_take(ctx, &t);
    if (rc) throw_io(env, ctx, rc);
    return (jlong)t;
}

/* DDRunner.run on any thread: waits for the earlier tickets, then reduces */
JNIEXPORT void JNICALL JFN(reduceTicket0)(JNIEnv *env, jclass cls, jlong h, jlong ticket, jobject buf, jint len,
                                          jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const uint8_t *p = (const uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    if (!p && len) {
        hdrf_ticket_cancel(ctx, (uint64_t)ticket);
        throw_io(env, ctx, HDRF_E_INVAL);
        return;
    }
    int rc = hdrf_reduce_block_ticketed(ctx, (uint64_t)ticket, (uint64_t)id, p, (uint64_t)len, NULL);
    if (rc) throw_io(env, ctx, rc);
}

JNIEXPORT void JNICALL JFN(cancel0)(JNIEnv *env, jclass cls, jlong h, jlong ticket)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int rc = hdrf_ticket_cancel(ctx, (uint64_t)ticket);
    if (rc) throw_io(env, ctx, rc);
}

/* The storers' chunkDir writes (DataDeduplicator.java:748-818): every container closed since the
 * last call is (re)written whole to chunkDir + id, every open container's new bytes are written at
 * the file's end.  Returns the number of file operations. */
static int write_event(const char *dir, const hdrf_container_event *e, const uint8_t *data)
{
    char path[4096];
    snprintf(path, sizeof path, "%s%u", dir, e->id);   /* DataNode.chunkDir + id (:754, :811) */
    /* file_off == 0: (re)write the file (a new container, or a closed Lz4Codec file); otherwise the
     * bytes go at the file's end (an open container's growth, or a raw container's closing tail) */
    FILE *f = fopen(path, e->file_off == 0 ? "wb" : "r+b");
    if (!f) return -1;
    int ok = fseeko(f, (off_t)e->file_off, SEEK_SET) == 0 &&
             fwrite(data, 1, (size_t)e->nbytes, f) == (size_t)e->nbytes;
    ok = (fclose(f) == 0) && ok;
    return ok ? 0 : -1;
}

JNIEXPORT jint JNICALL JFN(drain0)(JNIEnv *env, jclass cls, jlong h, jstring chunkDir)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const char *dir = (*env)->GetStringUTFChars(env, chunkDir, NULL);
    int64_t cap = 64ll << 20, need = 0, total = 0;
    uint8_t *buf = (uint8_t *)malloc((size_t)cap);
    hdrf_container_event ev[256];
    int rc = buf ? 0 : HDRF_E_NOMEM;
    while (!rc) {
        int64_t n = hdrf_drain_containers(ctx, ev, 256, buf, cap, &need);
        if (n == HDRF_E_CAPACITY && need > cap) {          /* one event larger than the buffer */
            uint8_t *nb = (uint8_t *)realloc(buf, (size_t)need);
            if (!nb) { rc = HDRF_E_NOMEM; break; }
            buf = nb;
            cap = need;
            continue;
        }
        if (n < 0) { rc = (int)n; break; }
        if (n == 0) break;
        for (int64_t i = 0; i < n && !rc; i++)
            if (write_event(dir, &ev[i], buf + ev[i].data_off)) rc = HDRF_E_INVAL;
        total += n;
    }
    free(buf);
    (*env)->ReleaseStringUTFChars(env, chunkDir, dir);
    if (rc) { throw_io(env, ctx, rc); return -1; }
    return (jint)total;
}

/* page-locked receive buffers: hdrf_submit_host copies from them on a side stream */
JNIEXPORT jobject JNICALL JFN(allocPinned0)(JNIEnv *env, jclass cls, jlong h, jlong bytes)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    void *p = NULL;
    int rc = hdrf_host_alloc(ctx, (uint64_t)bytes, &p);
    if (rc) { throw_io(env, ctx, rc); return NULL; }
    return (*env)->NewDirectByteBuffer(env, p, bytes);
}

JNIEXPORT void JNICALL JFN(freePinned0)(JNIEnv *env, jclass cls, jlong h, jobject buf)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    void *p = (*env)->GetDirectBufferAddress(env, buf);
    int rc = p ? hdrf_host_free(ctx, p) : HDRF_E_INVAL;
    if (rc) throw_io(env, ctx, rc);
}

/* Packet-granular receive (BlockReceiver.java:877-896): each received packet goes to the GPU as it
 * arrives; submitSlot hands the finished block to the pipeline (pair with wait0). */
JNIEXPORT jint JNICALL JFN(rxBegin0)(JNIEnv *env, jclass cls, jlong h, jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int32_t rx = -1;
    int rc = hdrf_rx_begin(ctx, (uint64_t)id, &rx);
    if (rc) throw_io(env, ctx, rc);
    return rx;
}

JNIEXPORT void JNICALL JFN(packet0)(JNIEnv *env, jclass cls, jlong h, jint rx, jobject buf, jint off, jint len)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const uint8_t *p = (const uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    const jlong cap = p ? (*env)->GetDirectBufferCapacity(env, buf) : 0;
    /* a negative jint would become a huge uint64_t length: check the range before the library */
    if (off < 0 || len < 0 || (jlong)off + (jlong)len > cap || (!p && len)) { throw_io(env, ctx, HDRF_E_INVAL); return; }
    int rc = hdrf_append_packet(ctx, rx, p + off, (uint64_t)len);   /* copied before return */
    if (rc) throw_io(env, ctx, rc);
}

JNIEXPORT void JNICALL JFN(submitSlot0)(JNIEnv *env, jclass cls, jlong h, jint rx)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int rc = hdrf_submit_slot(ctx, rx);
    if (rc) throw_io(env, ctx, rc);
}

/* every block whose last packet arrived since the previous submit, as ONE batch (FIFO = array order) */
JNIEXPORT void JNICALL JFN(submitSlots0)(JNIEnv *env, jclass cls, jlong h, jintArray rxs)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const jsize n = (*env)->GetArrayLength(env, rxs);
    jint *r = (*env)->GetIntArrayElements(env, rxs, NULL);
    if (!r) { throw_io(env, ctx, HDRF_E_NOMEM); return; }
    int32_t tmp[16];
    int rc = (n < 1 || n > 16) ? HDRF_E_INVAL : 0;
    for (jsize i = 0; !rc && i < n; i++) tmp[i] = (int32_t)r[i];
    (*env)->ReleaseIntArrayElements(env, rxs, r, JNI_ABORT);
    if (!rc) rc = hdrf_submit_slots(ctx, (int32_t)n, tmp);
    if (rc) throw_io(env, ctx, rc);
}

JNIEXPORT void JNICALL JFN(rxCancel0)(JNIEnv *env, jclass cls, jlong h, jint rx)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int rc = hdrf_rx_cancel(ctx, rx);
    if (rc) throw_io(env, ctx, rc);
}

/* reduceAsync: hdrf_submit_host on the direct buffer (copied H2D on a side stream) */
JNIEXPORT void JNICALL JFN(submit0)(JNIEnv *env, jclass cls, jlong h, jobject buf, jint len, jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const uint8_t *p = (const uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    const uint64_t n = (uint64_t)len, bid = (uint64_t)id;
    int rc = hdrf_submit_host(ctx, 1, &p, &n, &bid);
    if (rc) throw_io(env, ctx, rc);
}

JNIEXPORT void JNICALL JFN(wait0)(JNIEnv *env, jclass cls, jlong h)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int rc = hdrf_wait_batch(ctx);
    if (rc) throw_io(env, ctx, rc);
}

JNIEXPORT jlong JNICALL JFN(length0)(JNIEnv *env, jclass cls, jlong h, jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int64_t n = hdrf_block_length(ctx, (uint64_t)id);
    if (n < 0) throw_io(env, ctx, (int)n);
    return (jlong)n;
}

JNIEXPORT jbyteArray JNICALL JFN(recipe0)(JNIEnv *env, jclass cls, jlong h, jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    /* an unknown block throws, as length0 does (the recipe GET of DN/DataConstructor.java:46-72
     * has nothing to rebuild from) */
    int64_t len = hdrf_block_length(ctx, (uint64_t)id);
    if (len < 0) { throw_io(env, ctx, (int)len); return NULL; }
    int64_t cap = 4 + (int64_t)hdrf_digest_len(ctx) * (len / 702 + 2);
    uint8_t *tmp = (uint8_t *)malloc((size_t)cap);
    if (!tmp) { throw_io(env, ctx, HDRF_E_NOMEM); return NULL; }
    int64_t n = hdrf_recipe_get(ctx, (uint64_t)id, tmp, cap);
    if (n <= 0) { free(tmp); throw_io(env, ctx, n < 0 ? (int)n : HDRF_E_NOTFOUND); return NULL; }
    jbyteArray out = (*env)->NewByteArray(env, (jsize)n);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)n, (const jbyte *)tmp);
    free(tmp);
    return out;                                      /* NULL: OutOfMemoryError is pending */
}

/* DataConstructor(blkID, recipe).data, served by BlockSender (DN/BlockSender.java:612-619) */
JNIEXPORT jbyteArray JNICALL JFN(reconstruct0)(JNIEnv *env, jclass cls, jlong h, jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int64_t len = hdrf_block_length(ctx, (uint64_t)id);
    if (len < 0) { throw_io(env, ctx, (int)len); return NULL; }
    uint8_t *tmp = (uint8_t *)malloc((size_t)(len ? len : 1));
    if (!tmp) { throw_io(env, ctx, HDRF_E_NOMEM); return NULL; }
    int64_t n = hdrf_reconstruct_block(ctx, (uint64_t)id, tmp, len);
    if (n < 0) { free(tmp); throw_io(env, ctx, (int)n); return NULL; }
    jbyteArray out = (*env)->NewByteArray(env, (jsize)n);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)n, (const jbyte *)tmp);
    free(tmp);
    return out;
}

/* stream mode (compressor 0 SnappyCodec / 3 LzopCodec / 4 Lz4Codec / 5 GzipCodec): the block's chunkDir
 * file for packet writes.  LzopCodec headers carry the wall clock, as LzopOutputStream writes
 * System.currentTimeMillis() / 1000. */
JNIEXPORT jbyteArray JNICALL JFN(stream0)(JNIEnv *env, jclass cls, jlong h, jint codec, jobject buf, jint len,
                                          jlong id, jlongArray writes)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    const uint8_t *p = (const uint8_t *)(*env)->GetDirectBufferAddress(env, buf);
    const jsize nw = (*env)->GetArrayLength(env, writes);
    if (!p && len) { throw_io(env, ctx, HDRF_E_INVAL); return NULL; }
    jlong *w = (*env)->GetLongArrayElements(env, writes, NULL);
    if (codec == 3) hdrf_set_lzop_mtime(ctx, (uint32_t)time(NULL));
    const int64_t cap = 64 + (int64_t)len + len / 6 + 48 * ((int64_t)nw + len / 218422 + 2);
    uint8_t *out = (uint8_t *)malloc((size_t)cap);
    int64_t n = out ? hdrf_stream_block_host(ctx, codec, (uint64_t)id, p, (uint64_t)len, (const uint64_t *)w, nw, out,
                                             cap)
                    : HDRF_E_INVAL;
    (*env)->ReleaseLongArrayElements(env, writes, w, JNI_ABORT);
    jbyteArray r = NULL;
    if (n < 0) throw_io(env, ctx, (int)n);
    else if ((r = (*env)->NewByteArray(env, (jsize)n)) != NULL)
        (*env)->SetByteArrayRegion(env, r, 0, (jsize)n, (const jbyte *)out);
    free(out);
    return r;
}

JNIEXPORT void JNICALL JFN(close0)(JNIEnv *env, jclass cls, jlong h)
{
    (void)env; (void)cls;
    hdrf_close((hdrf_ctx *)(intptr_t)h);
}

/* stream-mode read (DataConstructor's codec input stream over chunkDir + blkID,
 * DN/DataConstructor.java:102-220): the block file decoded on the GPU (codec 0 SnappyCodec,
 * 3 LzopCodec, 4 Lz4Codec, 5 GzipCodec); the raw length is the one streamBlock recorded for blockId. */
JNIEXPORT jbyteArray JNICALL JFN(streamDecode0)(JNIEnv *env, jclass cls, jlong h, jint codec, jbyteArray file,
                                                jlong id)
{
    (void)cls;
    hdrf_ctx *ctx = (hdrf_ctx *)(intptr_t)h;
    int64_t len = hdrf_block_length(ctx, (uint64_t)id);
    if (len < 0) { throw_io(env, ctx, (int)len); return NULL; }
    const jsize flen = (*env)->GetArrayLength(env, file);
    void *dev = NULL;
    uint8_t *tmp = (uint8_t *)malloc((size_t)(len ? len : 1));
    int rc = tmp ? hdrf_dev_alloc(ctx, (uint64_t)(len ? len : 1), &dev) : HDRF_E_NOMEM;
    int64_t n = rc;
    if (!rc) {
        jbyte *f = (*env)->GetByteArrayElements(env, file, NULL);
        n = f ? hdrf_stream_file_decode(ctx, codec, (const uint8_t *)f, flen, (uint8_t *)dev, len) : HDRF_E_INVAL;
        if (f) (*env)->ReleaseByteArrayElements(env, file, f, JNI_ABORT);
        if (n >= 0 && n != len) n = HDRF_E_INVAL;          /* the file must hold the recorded length */
        if (n > 0 && (rc = hdrf_memcpy_d2h(ctx, tmp, dev, (uint64_t)n)) != 0) n = rc;
        hdrf_dev_free(ctx, dev);
    }
    jbyteArray r = NULL;
    if (n < 0) throw_io(env, ctx, (int)n);
    else if ((r = (*env)->NewByteArray(env, (jsize)n)) != NULL)
        (*env)->SetByteArrayRegion(env, r, 0, (jsize)n, (const jbyte *)tmp);
    free(tmp);
    return r;
}
