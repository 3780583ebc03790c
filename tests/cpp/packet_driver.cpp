// packet_driver.cpp — the DataNode's packet-granular write path driven from native threads
// through the C-ABI the JNI binding calls (BASELINE config 5; VERDICT r2 "no native driver of the
// 64 KiB-packet path").
//
// Reference shape: BlockReceiver.receivePacket appends every received packet to bf1
// (DN/BlockReceiver.java:877-896; dfs.client-write-packet-size 64 KiB, hdfs-default.xml:1079-1080),
// one DataXceiver thread per block, and the finished block is handed to the reducer
// (:1258-1261).  Here T receiver threads each own one block at a time and call
// hdrf_append_packet once per packet from pinned host memory; the main thread opens receive
// buffers (hdrf_rx_begin) in block order, submits the received blocks in that order
// (hdrf_submit_slot: the FIFO); a completer thread completes them (hdrf_wait_batch, which blocks
// without the context lock) and drains the durable containers after every completed block
// (hdrf_drain_containers, as hdrf_jni.c does) while the receivers take the next blocks.
//
// usage: packet_driver BLOCKS BLOCK_MIB PACKET_KIB THREADS STEPS [OUT_FILE]
//   The corpus is BASELINE config 2's (1 MiB segments, 50 % cross-block duplicates, seed
//   20251015), generated on the device and copied to pinned host memory before the timed steps.
//   Prints one JSON line; OUT_FILE (optional) receives "block n_chunks store_size" per block of
//   the last step (the parity test compares them with the oracle).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "hdrf.h"

static uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// hdrf_amd/corpus.py corpus_roots (the segment each (block, segment) carries)
static std::vector<uint32_t> corpus_roots(uint64_t seed, uint32_t dup_ppm, int64_t nb, int64_t spb)
{
    std::vector<uint32_t> roots((size_t)(nb * spb));
    for (int64_t g = 0; g < nb * spb; g++) roots[(size_t)g] = (uint32_t)g;
    for (int64_t b = 1; b < nb; b++)
        for (int64_t s = 0; s < spb; s++) {
            const uint64_t g = (uint64_t)(b * spb + s);
            const uint64_t coin = mix64(seed ^ 0xD1B54A32D192ED03ull ^ mix64(g));
            if (coin % 1000000ull >= dup_ppm) continue;
            const uint64_t r1 = mix64(coin);
            const uint64_t ss = mix64(r1) % (uint64_t)spb;
            const uint64_t sb = r1 % (uint64_t)b;
            roots[(size_t)g] = roots[(size_t)(sb * spb + ss)];
        }
    return roots;
}

#define CK(x)                                                                                  \
    do {                                                                                       \
        int rc_ = (x);                                                                         \
        if (rc_) {                                                                             \
            std::fprintf(stderr, "%s failed: %d %s\n", #x, rc_, hdrf_last_error(ctx));         \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

int main(int argc, char **argv)
{
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s BLOCKS BLOCK_MIB PACKET_KIB THREADS STEPS [OUT_FILE]\n", argv[0]);
        return 2;
    }
    const int64_t nb = std::atoll(argv[1]);
    const int64_t S = std::atoll(argv[2]) << 20;
    const int64_t P = std::atoll(argv[3]) << 10;
    const int T = std::atoi(argv[4]);
    const int steps = std::atoi(argv[5]);
    const char *out_file = argc > 6 ? argv[6] : nullptr;
    const int64_t seg = 1 << 20, spb = S / seg;
    if (nb < 1 || S < seg || P < 1 || T < 1 || T > 16 || steps < 1) return 2;

    hdrf_ctx *ctx = nullptr;
    hdrf_cfg cfg;
    hdrf_default_cfg(&cfg);
    cfg.max_block_bytes = S;
    cfg.max_batch_blocks = 1;
    cfg.index_log2 = 27;
    cfg.arena_slots = 512;
    cfg.retain_containers = std::getenv("HDRF_DRIVER_NODRAIN") ? 0 : 1;
    if (int rc = hdrf_open(&cfg, &ctx)) {
        std::fprintf(stderr, "hdrf_open: %d\n", rc);
        return 1;
    }
    // corpus on the device, then into pinned host memory (the received blocks)
    std::vector<uint32_t> roots = corpus_roots(20251015ull, 500000, nb, spb);
    void *dev = nullptr, *host = nullptr, *dbuf = nullptr;
    const int64_t dcap = 256ll << 20;
    CK(hdrf_dev_alloc(ctx, (uint64_t)(nb * S), &dev));
    CK(hdrf_corpus_fill(ctx, (uint8_t *)dev, roots.data(), nb, spb, seg, 20251015ull));
    CK(hdrf_host_alloc(ctx, (uint64_t)(nb * S), &host));
    CK(hdrf_host_alloc(ctx, (uint64_t)dcap, &dbuf));
    CK(hdrf_memcpy_d2h(ctx, host, dev, (uint64_t)(nb * S)));
    CK(hdrf_dev_free(ctx, dev));

    std::vector<int64_t> n_chunks((size_t)nb), store((size_t)nb);
    std::vector<hdrf_container_event> ev(4096);
    int64_t drained_bytes = 0, done = 0;
    auto drain = [&]() {
        for (;;) {
            int64_t need = 0;
            const int64_t n = hdrf_drain_containers(ctx, ev.data(), (int64_t)ev.size(), (uint8_t *)dbuf, dcap, &need);
            if (n < 0) {
                std::fprintf(stderr, "drain: %lld %s\n", (long long)n, hdrf_last_error(ctx));
                std::exit(1);
            }
            if (n == 0) return;
            for (int64_t i = 0; i < n; i++) drained_bytes += ev[(size_t)i].nbytes;
        }
    };
    const bool no_drain = std::getenv("HDRF_DRIVER_NODRAIN") != nullptr;      // A/B only
    // HDRF_DRIVER_SERIAL (A/B only): the main thread completes and drains between receive rounds
    // (round-3 c1 shape); default: a completer thread does it while the receivers run, as the
    // reference's reducer/storer runs apart from the DataXceiver threads.
    const bool serial = std::getenv("HDRF_DRIVER_SERIAL") != nullptr;
    auto complete = [&]() {
        CK(hdrf_wait_batch(ctx));
        CK(hdrf_batch_info(ctx, 0, &n_chunks[(size_t)done], &store[(size_t)done]));
        done++;
        if (!no_drain) drain();
    };
    const int kDepth = 5, kRx = 16;                // HDRF_PIPELINE_DEPTH, receive buffers (hdrf.h)
    double best = 0, total_s = 0;
    for (int step = 0; step <= steps; step++) {    // step 0: warm-up
        CK(hdrf_reset(ctx));
        done = 0;
        drained_bytes = 0;
        std::mutex mu;
        std::condition_variable cv;
        int64_t submitted = 0, completed = 0;      // guarded by mu
        std::thread completer;
        if (!serial)
            completer = std::thread([&]() {
                for (int64_t c = 0; c < nb; c++) {
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return submitted > c; });
                    }
                    complete();
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        completed = c + 1;
                    }
                    cv.notify_all();
                }
            });
        auto in_flight = [&]() { std::lock_guard<std::mutex> lk(mu); return submitted - completed; };
        auto wait_until = [&](int64_t max_in_flight) {          // completer frees slots / buffers
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return submitted - completed <= max_in_flight; });
        };
        const auto t0 = std::chrono::steady_clock::now();
        for (int64_t g = 0; g < nb; g += T) {
            const int k = (int)std::min<int64_t>(T, nb - g);
            if (serial) {
                while (in_flight() + k > kRx || in_flight() >= kDepth) {
                    complete();
                    std::lock_guard<std::mutex> lk(mu);
                    completed++;
                }
            } else {
                wait_until(kRx - k);
            }
            std::vector<int32_t> rx((size_t)k);
            for (int i = 0; i < k; i++) CK(hdrf_rx_begin(ctx, (uint64_t)(g + i), &rx[(size_t)i]));
            std::vector<std::thread> th;
            std::atomic<int> bad{0};
            for (int i = 0; i < k; i++)
                th.emplace_back([&, i]() {
                    const uint8_t *b = (const uint8_t *)host + (g + i) * S;
                    for (int64_t o = 0; o < S; o += P)
                        if (hdrf_append_packet(ctx, rx[(size_t)i], b + o, (uint64_t)std::min(P, S - o))) bad++;
                });
            for (auto &t : th) t.join();
            if (bad) {
                std::fprintf(stderr, "append failed: %s\n", hdrf_last_error(ctx));
                return 1;
            }
            for (int i = 0; i < k; i++) {
                if (serial) {
                    if (in_flight() >= kDepth) {
                        complete();
                        std::lock_guard<std::mutex> lk(mu);
                        completed++;
                    }
                } else {
                    wait_until(kDepth - 1);
                }
                CK(hdrf_submit_slot(ctx, rx[(size_t)i]));
                {
                    std::lock_guard<std::mutex> lk(mu);
                    submitted++;
                }
                cv.notify_all();
            }
        }
        if (serial)
            while (in_flight()) {
                complete();
                std::lock_guard<std::mutex> lk(mu);
                completed++;
            }
        else
            completer.join();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (step > 0) {
            total_s += s;
            best = std::max(best, nb * S / s / 1e9);
        }
    }
    int64_t stored = 0, chunks = 0;
    for (int64_t b = 0; b < nb; b++) { stored += store[(size_t)b]; chunks += n_chunks[(size_t)b]; }
    std::printf("{\"driver\": \"tests/cpp/packet_driver.cpp\", \"blocks\": %lld, \"block_bytes\": %lld, "
                "\"packet_bytes\": %lld, \"threads\": %d, \"steps\": %d, \"GB_s\": %.3f, \"best_GB_s\": %.3f, "
                "\"packets_per_step\": %lld, \"stored_bytes\": %lld, \"chunks\": %lld, "
                "\"drained_bytes_last_step\": %lld}\n",
                (long long)nb, (long long)S, (long long)P, T, steps, nb * S * steps / total_s / 1e9, best,
                (long long)(nb * ((S + P - 1) / P)), (long long)stored, (long long)chunks, (long long)drained_bytes);
    if (out_file) {
        FILE *f = std::fopen(out_file, "w");
        for (int64_t b = 0; b < nb; b++)
            std::fprintf(f, "%lld %lld %lld\n", (long long)b, (long long)n_chunks[(size_t)b], (long long)store[(size_t)b]);
        std::fclose(f);
    }
    hdrf_host_free(ctx, host);
    hdrf_host_free(ctx, dbuf);
    hdrf_close(ctx);
    return 0;
}
