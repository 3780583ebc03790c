// packet_driver.cpp — the DataNode's packet-granular write path driven from native threads
// through the C-ABI the JNI binding calls (BASELINE config 5: "JNI-backed GPU ReductionScheme with
// overlapped H2D copies under concurrent block writes incl. block mirroring").
//
// Reference shape: BlockReceiver.receivePacket forwards every received packet to the next DataNode
// of the write pipeline FIRST (packetReceiver.mirrorPacketTo(mirrorOut), DN/BlockReceiver.java:
// 635-641) and then appends it to bf1 (:877-896; dfs.client-write-packet-size 64 KiB,
// hdfs-default.xml:1079-1080), one DataXceiver thread per block; the finished block is handed to
// the reducer (:1258-1261).  Here T receiver threads (DataXceivers) each take the next block as soon
// as they finished the last one, open a receive buffer for it (hdrf_rx_begin), and per packet forward
// it to their mirror (below) and then call hdrf_append_packet from pinned host memory.  The main
// thread submits the received blocks in block order (the FIFO): one block per submit
// (hdrf_submit_slot, the reference's per-block DDRunner) or every block received in order since the
// last submit as one batch (--batch: hdrf_submit_slots).  A completer thread completes the batches
// (hdrf_wait_batch, which blocks without the context lock) and drains the durable containers after
// every completed batch (hdrf_drain_containers, as hdrf_jni.c does) while the receivers go on.
//
// Mirror (the downstream DataNode's end of mirrorOut), one consumer thread per receiver:
//   ring    the packet is copied into a 32 MiB byte ring the consumer drains (mirrorOut as a
//           buffered stream whose reader keeps up; the default)
//   socket  the packet is written to an AF_UNIX stream socket the consumer reads (a loopback link)
//   none    no mirroring (a single-replica write)
// The consumer checksums every block it receives; after the run each block's mirrored checksum
// must equal the checksum of the block's bytes ("mirror_ok").
//
// usage: packet_driver BLOCKS BLOCK_MIB PACKET_KIB THREADS STEPS [OUT_DIR] [--compressor C]
//          [--mirror ring|socket|none] [--batch] [--mixed] [--container-kib K] [--arena-slots N]
//          [--index-log2 L] [--out-blocks K] [--out-containers M]
//   The corpus is BASELINE config 2's (1 MiB segments, 50 % cross-block duplicates, seed
//   20251015; --mixed: config 4's mixed-entropy segments), generated on the device and copied to
//   pinned host memory before the timed steps.  Prints one JSON line.  OUT_DIR (optional) receives
//   the last step's results: blocks.txt ("block n_chunks store_size"), blk_<b>.bin per block
//   (offsets u32[n], digests u8[n*H], is_new u8[n]) and containers.bin (the chunkDir the drained
//   events built: records [u32 id][u32 closed][u64 len][bytes]); the parity test compares them
//   with the oracle.  With OUT_DIR the results come from one more, untimed step after the timed
//   ones; --out-blocks K keeps blk_<b>.bin of blocks b < K only, --out-containers M the containers
//   whose per-range index (id & 0x3FFFFF) is below M (bench.py's sample check).
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
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

// Position-keyed checksum of a byte stream fed in arbitrary pieces (the mirror's check that every
// packet arrived downstream once, in order): sum over 8-byte words w_i of w_i * (2i + 1).
struct StreamSum {
    uint64_t sum = 0, word = 0, pos = 0;       // pos: bytes consumed
    void feed(const uint8_t *p, uint64_t n)
    {
        while (n && (pos & 7)) {               // finish a partial word
            word |= (uint64_t)*p++ << (8 * (pos & 7));
            if ((++pos & 7) == 0) { sum += word * (2 * (pos / 8 - 1) + 1); word = 0; }
            n--;
        }
        uint64_t i = pos / 8, s = 0;
        const uint64_t nw = n / 8;
        for (uint64_t k = 0; k < nw; k++) {
            uint64_t w;
            std::memcpy(&w, p + 8 * k, 8);
            s += w * (2 * (i + k) + 1);
        }
        sum += s;
        pos += 8 * nw;
        p += 8 * nw;
        n -= 8 * nw;
        while (n) {
            word |= (uint64_t)*p++ << (8 * (pos & 7));
            if ((++pos & 7) == 0) { sum += word * (2 * (pos / 8 - 1) + 1); word = 0; }
            n--;
        }
    }
    uint64_t finish() const { return (pos & 7) ? sum + word * (2 * (pos / 8) + 1) : sum; }
};

// spin briefly, then sleep: an idle mirror consumer must not hold a core the receivers need
static void backoff(int &spins)
{
    if (++spins < 64) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
}

// One receiver's mirror: the packets of the blocks it receives (each S bytes) go downstream in order;
// the consumer checksums each block until the stream ends.
struct Mirror {
    static constexpr uint64_t kRing = 32ull << 20;
    int mode = 0;                                 // 1 ring, 2 socket
    std::vector<uint8_t> ring;
    alignas(64) std::atomic<uint64_t> head{0};    // bytes produced
    alignas(64) std::atomic<uint64_t> tail{0};    // bytes consumed
    int fd[2] = {-1, -1};
    std::thread th;

    void push(const uint8_t *p, uint64_t n)
    {
        if (mode == 2) {
            while (n) {
                const ssize_t w = write(fd[0], p, n);
                if (w <= 0) { std::perror("mirror write"); std::exit(1); }
                p += w;
                n -= (uint64_t)w;
            }
            return;
        }
        while (n) {
            const uint64_t h = head.load(std::memory_order_relaxed);
            uint64_t room;
            int spins = 0;
            while ((room = kRing - (h - tail.load(std::memory_order_acquire))) == 0) backoff(spins);
            const uint64_t off = h % kRing, m = std::min({n, room, kRing - off});
            std::memcpy(ring.data() + off, p, m);
            head.store(h + m, std::memory_order_release);
            p += m;
            n -= m;
        }
    }
    // the consumer: checksums of consecutive S-byte blocks until the stream ends (socket: EOF; ring:
    // `done` set once every producer has stopped)
    void consume(int64_t S, std::vector<uint64_t> &sums, const std::atomic<bool> &done)
    {
        std::vector<uint8_t> buf(mode == 2 ? (1u << 20) : 0);
        StreamSum cs;
        int64_t left = S;
        auto got = [&](const uint8_t *p, uint64_t m) {
            while (m) {
                const uint64_t k = std::min<uint64_t>(m, (uint64_t)left);
                cs.feed(p, k);
                p += k;
                m -= k;
                left -= (int64_t)k;
                if (left == 0) {
                    sums.push_back(cs.finish());
                    cs = StreamSum();
                    left = S;
                }
            }
        };
        for (;;) {
            if (mode == 2) {
                const ssize_t r = read(fd[1], buf.data(), buf.size());
                if (r < 0) { std::perror("mirror read"); std::exit(1); }
                if (r == 0) return;                      // the receiver closed its end
                got(buf.data(), (uint64_t)r);
                continue;
            }
            const uint64_t t = tail.load(std::memory_order_relaxed);
            const uint64_t avail = head.load(std::memory_order_acquire) - t;
            if (avail == 0) {
                if (done.load(std::memory_order_acquire) && head.load(std::memory_order_acquire) == t) return;
                int spins = 0;
                backoff(spins);
                continue;
            }
            const uint64_t off = t % kRing, m = std::min<uint64_t>(avail, kRing - off);
            got(ring.data() + off, m);
            tail.store(t + m, std::memory_order_release);
        }
    }
};

int main(int argc, char **argv)
{
    if (argc < 6) {
        std::fprintf(stderr,
                     "usage: %s BLOCKS BLOCK_MIB PACKET_KIB THREADS STEPS [OUT_DIR] [--compressor C] "
                     "[--mirror ring|socket|none] [--batch] [--mixed] [--container-kib K] [--arena-slots N] "
                     "[--index-log2 L] [--out-blocks K] [--out-containers M]\n",
                     argv[0]);
        return 2;
    }
    const int64_t nb = std::atoll(argv[1]);
    const int64_t S = std::atoll(argv[2]) << 20;
    const int64_t P = std::atoll(argv[3]) << 10;
    const int T = std::atoi(argv[4]);
    const int steps = std::atoi(argv[5]);
    const char *out_dir = nullptr;
    int compressor = 1, mirror_mode = 1, mixed = 0, index_log2 = 27;
    bool batch = false;
    int64_t container = 1ll << 25, arena = 512, out_blocks = -1, out_conts = -1;
    for (int i = 6; i < argc; i++) {
        const std::string a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : "";
        if (a == "--compressor") compressor = std::atoi(v), i++;
        else if (a == "--mirror") {
            const std::string m = v;
            mirror_mode = m == "none" ? 0 : m == "socket" ? 2 : m == "ring" ? 1 : -1;
            i++;
        } else if (a == "--batch") batch = true;
        else if (a == "--mixed") mixed = 1;
        else if (a == "--container-kib") container = std::atoll(v) << 10, i++;
        else if (a == "--arena-slots") arena = std::atoll(v), i++;
        else if (a == "--index-log2") index_log2 = std::atoi(v), i++;
        else if (a == "--out-blocks") out_blocks = std::atoll(v), i++;
        else if (a == "--out-containers") out_conts = std::atoll(v), i++;
        else if (a.size() && a[0] != '-' && !out_dir) out_dir = argv[i];
        else {
            std::fprintf(stderr, "bad argument %s\n", a.c_str());
            return 2;
        }
    }
    const int64_t seg = 1 << 20, spb = S / seg;
    if (nb < 1 || S < seg || P < 1 || T < 1 || T > 16 || steps < 1 || mirror_mode < 0 ||
        (compressor != 1 && compressor != 2))
        return 2;

    hdrf_ctx *ctx = nullptr;
    hdrf_cfg cfg;
    hdrf_default_cfg(&cfg);
    cfg.max_block_bytes = S;
    cfg.max_batch_blocks = batch ? 16 : 1;
    cfg.index_log2 = index_log2;
    cfg.arena_slots = arena;
    cfg.container_max = (uint32_t)container;
    cfg.compressor = compressor;
    cfg.retain_containers = std::getenv("HDRF_DRIVER_NODRAIN") ? 0 : 1;
    if (int rc = hdrf_open(&cfg, &ctx)) {
        std::fprintf(stderr, "hdrf_open: %d\n", rc);
        return 1;
    }
    const int H = hdrf_digest_len(ctx);
    // corpus on the device, then into pinned host memory (the received blocks)
    std::vector<uint32_t> roots = corpus_roots(20251015ull, 500000, nb, spb);
    void *dev = nullptr, *host = nullptr, *dbuf = nullptr;
    const int64_t dcap = 256ll << 20;
    CK(hdrf_dev_alloc(ctx, (uint64_t)(nb * S), &dev));
    CK(hdrf_corpus_fill_kind(ctx, (uint8_t *)dev, roots.data(), nb, spb, seg, 20251015ull, mixed));
    CK(hdrf_host_alloc(ctx, (uint64_t)(nb * S), &host));
    CK(hdrf_host_alloc(ctx, (uint64_t)dcap, &dbuf));
    CK(hdrf_memcpy_d2h(ctx, host, dev, (uint64_t)(nb * S)));
    CK(hdrf_dev_free(ctx, dev));

    // mirrors: one per receiver index, alive over all steps
    std::vector<Mirror> mirrors(mirror_mode ? T : 0);
    std::vector<std::vector<uint64_t>> msum(mirrors.size());        // per receiver: mirrored block sums
    std::vector<std::vector<int64_t>> mids(mirrors.size());         // per receiver: the blocks it received
    std::atomic<bool> mirror_done{false};
    for (int r = 0; r < (int)mirrors.size(); r++) {
        Mirror &m = mirrors[(size_t)r];
        m.mode = mirror_mode;
        if (mirror_mode == 1) m.ring.resize(Mirror::kRing);
        else {
            if (socketpair(AF_UNIX, SOCK_STREAM, 0, m.fd)) { std::perror("socketpair"); return 1; }
            int sz = 4 << 20;
            setsockopt(m.fd[0], SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
            setsockopt(m.fd[1], SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
        }
        m.th = std::thread([&m, &msum, &mirror_done, r, S]() { m.consume(S, msum[(size_t)r], mirror_done); });
    }

    std::vector<int64_t> n_chunks((size_t)nb), store((size_t)nb);
    struct BlockOut {
        std::vector<uint32_t> off;
        std::vector<uint8_t> dig, isnew;
    };
    std::vector<BlockOut> bout(out_dir ? (size_t)nb : 0);
    std::map<uint32_t, std::pair<std::vector<uint8_t>, uint32_t>> disk;      // the last step's chunkDir
    bool capture = false;
    std::vector<hdrf_container_event> ev(4096);
    int64_t drained_bytes = 0, drained_events = 0, done = 0, batches = 0;
    auto drain = [&]() {
        for (;;) {
            int64_t need = 0;
            const int64_t n = hdrf_drain_containers(ctx, ev.data(), (int64_t)ev.size(), (uint8_t *)dbuf, dcap, &need);
            if (n < 0) {
                std::fprintf(stderr, "drain: %lld %s\n", (long long)n, hdrf_last_error(ctx));
                std::exit(1);
            }
            if (n == 0) return;
            for (int64_t i = 0; i < n; i++) {
                const hdrf_container_event &e = ev[(size_t)i];
                drained_bytes += e.nbytes;
                if (!capture || (out_conts >= 0 && (int64_t)(e.id & 0x3FFFFFu) >= out_conts)) continue;
                auto &f = disk[e.id];
                const uint8_t *src = (const uint8_t *)dbuf + e.data_off;
                if (e.file_off == 0) f.first.assign(src, src + e.nbytes);   // (re)write
                else {                                                       // the file grows
                    if ((int64_t)f.first.size() != e.file_off) {
                        std::fprintf(stderr, "append to %u at %lld, file has %zu\n", e.id, (long long)e.file_off,
                                     f.first.size());
                        std::exit(1);
                    }
                    f.first.insert(f.first.end(), src, src + e.nbytes);
                }
                f.second = (uint32_t)e.closed;
            }
            drained_events += n;
        }
    };
    const bool no_drain = std::getenv("HDRF_DRIVER_NODRAIN") != nullptr;      // A/B only
    // HDRF_DRIVER_SERIAL (A/B only): the main thread completes and drains between receive rounds
    // (round-3 c1 shape); default: a completer thread does it while the receivers run, as the
    // reference's reducer/storer runs apart from the DataXceiver threads.
    const bool serial = std::getenv("HDRF_DRIVER_SERIAL") != nullptr;
    std::vector<int64_t> batch_len;                 // blocks per submitted batch, in order
    auto complete = [&](int64_t bi) {
        CK(hdrf_wait_batch(ctx));
        const int64_t k = batch_len[(size_t)bi];
        for (int64_t i = 0; i < k; i++) {
            const int64_t b = done + i;
            CK(hdrf_batch_info(ctx, (int32_t)i, &n_chunks[(size_t)b], &store[(size_t)b]));
            if (capture && (out_blocks < 0 || b < out_blocks)) {
                BlockOut &o = bout[(size_t)b];
                const int64_t n = n_chunks[(size_t)b];
                o.off.resize((size_t)n);
                o.dig.resize((size_t)(n * H));
                o.isnew.resize((size_t)n);
                CK(hdrf_batch_offsets(ctx, (int32_t)i, o.off.data(), n));
                CK(hdrf_batch_digests(ctx, (int32_t)i, o.dig.data(), n * H));
                CK(hdrf_batch_is_new(ctx, (int32_t)i, o.isnew.data(), n));
            }
        }
        done += k;
        if (!no_drain) drain();
    };
    const int kDepth = 5, kRx = 16;                // HDRF_PIPELINE_DEPTH, receive buffers (hdrf.h)
    double best = 0, total_s = 0;
    std::vector<double> step_rate;                 // GB/s of every timed step
    // step 0: warm-up; steps 1..steps timed; OUT_DIR: one more, untimed step keeps the results
    const int last = steps + (out_dir ? 1 : 0);
    int64_t timed_drained_bytes = 0, timed_drained_events = 0;
    for (int step = 0; step <= last; step++) {
        CK(hdrf_reset(ctx));
        done = 0;
        drained_bytes = drained_events = 0;
        capture = out_dir && step == last;
        if (capture) disk.clear();
        std::mutex mu;
        std::condition_variable cv;
        int64_t submitted = 0, completed = 0;      // batches, guarded by mu
        int64_t sub_blocks = 0;                    // blocks submitted, guarded by mu
        std::vector<int32_t> rxof((size_t)nb, -1); // receive buffer of each fully received block (mu)
        batch_len.clear();
        batch_len.reserve((size_t)nb);
        std::thread completer;
        auto on_complete = [&](int64_t c) {
            {
                std::lock_guard<std::mutex> lk(mu);
                completed = c + 1;
            }
            cv.notify_all();                        // receive buffers and a pipeline slot are free again
        };
        int64_t nbatch = -1;                       // known once the submitter has finished (mu)
        if (!serial)
            completer = std::thread([&]() {
                for (int64_t c = 0;; c++) {
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return submitted > c || (nbatch >= 0 && c >= nbatch); });
                        if (nbatch >= 0 && c >= nbatch) return;
                    }
                    complete(c);
                    on_complete(c);
                }
            });
        auto serial_complete_one = [&]() {
            int64_t c;
            {
                std::lock_guard<std::mutex> lk(mu);
                c = completed;
            }
            complete(c);
            on_complete(c);
        };
        std::atomic<int64_t> next_block{0};
        std::atomic<int> bad{0};
        const auto t0 = std::chrono::steady_clock::now();
        // receivers: each takes the next block as soon as its last one is received; a block may start
        // only kRx blocks ahead of the submit order, so the lowest unsubmitted block always finds a
        // receive buffer once the batches in flight complete
        std::vector<std::thread> th;
        for (int i = 0; i < T; i++)
            th.emplace_back([&, i]() {
                Mirror *m = mirrors.empty() ? nullptr : &mirrors[(size_t)i];
                for (;;) {
                    const int64_t b = next_block.fetch_add(1);
                    if (b >= nb) return;
                    int32_t rx = -1;
                    for (;;) {
                        {
                            std::unique_lock<std::mutex> lk(mu);
                            cv.wait(lk, [&] { return b < sub_blocks + kRx; });
                        }
                        const int rc = hdrf_rx_begin(ctx, (uint64_t)b, &rx);
                        if (rc == 0) break;
                        if (rc != HDRF_E_CAPACITY) { bad++; return; }
                        std::unique_lock<std::mutex> lk(mu);       // all sixteen in use: wait for a completion
                        const int64_t c0 = completed;
                        cv.wait_for(lk, std::chrono::milliseconds(5), [&] { return completed != c0; });
                    }
                    if (m) mids[(size_t)i].push_back(b);
                    const uint8_t *src = (const uint8_t *)host + b * S;
                    for (int64_t o = 0; o < S; o += P) {
                        const uint64_t n = (uint64_t)std::min(P, S - o);
                        if (m) m->push(src + o, n);                 // mirrorPacketTo before bf1.put (:635-641)
                        if (hdrf_append_packet(ctx, rx, src + o, n)) { bad++; return; }
                    }
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        rxof[(size_t)b] = rx;
                    }
                    cv.notify_all();
                }
            });
        // submitter: blocks in order; --batch hands over every block received in order so far (<= 16)
        int64_t nb_done = 0, nbt = 0;
        while (nb_done < nb && !bad) {
            std::vector<int32_t> rxs;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return rxof[(size_t)nb_done] >= 0 || bad; });
                if (bad) break;
                const int64_t lim = batch ? 16 : 1;
                for (int64_t b = nb_done; b < nb && (int64_t)rxs.size() < lim && rxof[(size_t)b] >= 0; b++)
                    rxs.push_back(rxof[(size_t)b]);
            }
            if (serial) {
                for (;;) {
                    bool full;
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        full = submitted - completed >= kDepth;
                    }
                    if (!full) break;
                    serial_complete_one();
                }
            } else {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return submitted - completed <= kDepth - 1; });
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                batch_len.push_back((int64_t)rxs.size());
            }
            if (rxs.size() == 1) CK(hdrf_submit_slot(ctx, rxs[0]));
            else CK(hdrf_submit_slots(ctx, (int32_t)rxs.size(), rxs.data()));
            {
                std::lock_guard<std::mutex> lk(mu);
                submitted++;
                sub_blocks += (int64_t)rxs.size();
            }
            cv.notify_all();
            nb_done += (int64_t)rxs.size();
            nbt++;
        }
        for (auto &t : th) t.join();
        if (bad) {
            std::fprintf(stderr, "receive failed: %s\n", hdrf_last_error(ctx));
            return 1;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            nbatch = nbt;
        }
        cv.notify_all();
        if (serial)
            while (true) {
                bool left;
                {
                    std::lock_guard<std::mutex> lk(mu);
                    left = completed < submitted;
                }
                if (!left) break;
                serial_complete_one();
            }
        else
            completer.join();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (step > 0 && step <= steps) {
            batches = nbt;
            total_s += s;
            best = std::max(best, nb * S / s / 1e9);
            step_rate.push_back(nb * S / s / 1e9);
            timed_drained_bytes = drained_bytes;
            timed_drained_events = drained_events;
        }
    }
    // the mirror received every block of every step once, in the order its receiver took them
    bool mirror_ok = true;
    int64_t mirrored = 0;
    mirror_done.store(true, std::memory_order_release);
    for (auto &m : mirrors)
        if (m.mode == 2) close(m.fd[0]);                       // EOF for the socket consumers
    for (auto &m : mirrors) m.th.join();
    if (!mirrors.empty()) {
        std::vector<uint64_t> want((size_t)nb);
        for (int64_t b = 0; b < nb; b++) {
            StreamSum cs;
            cs.feed((const uint8_t *)host + b * S, (uint64_t)S);
            want[(size_t)b] = cs.finish();
        }
        int64_t nmir = 0;
        for (int r = 0; r < T; r++) {
            mirror_ok &= msum[(size_t)r].size() == mids[(size_t)r].size();
            for (size_t k = 0; k < msum[(size_t)r].size() && k < mids[(size_t)r].size(); k++) {
                mirror_ok &= msum[(size_t)r][k] == want[(size_t)mids[(size_t)r][k]];
                mirrored += S;
            }
            nmir += (int64_t)mids[(size_t)r].size();
        }
        mirror_ok &= nmir == nb * (last + 1);
        for (auto &m : mirrors)
            if (m.mode == 2) close(m.fd[1]);
    }
    int64_t stored = 0, chunks = 0;
    for (int64_t b = 0; b < nb; b++) { stored += store[(size_t)b]; chunks += n_chunks[(size_t)b]; }
    std::vector<double> sorted_rate = step_rate;
    std::sort(sorted_rate.begin(), sorted_rate.end());
    const double median = sorted_rate.empty() ? 0.0 : sorted_rate[sorted_rate.size() / 2];
    std::string rates = "[";
    for (size_t i = 0; i < step_rate.size(); i++) {
        char b[32];
        std::snprintf(b, sizeof b, "%s%.3f", i ? ", " : "", step_rate[i]);
        rates += b;
    }
    rates += "]";
    std::printf("{\"driver\": \"tests/cpp/packet_driver.cpp\", \"blocks\": %lld, \"block_bytes\": %lld, "
                "\"packet_bytes\": %lld, \"threads\": %d, \"steps\": %d, \"GB_s\": %.3f, \"best_GB_s\": %.3f, "
                "\"median_GB_s\": %.3f, \"step_GB_s\": %s, "
                "\"packets_per_step\": %lld, \"stored_bytes\": %lld, \"chunks\": %lld, \"compressor\": %d, "
                "\"corpus\": \"%s\", \"mirror\": \"%s\", \"mirror_ok\": %s, \"mirrored_bytes\": %lld, "
                "\"submit\": \"%s\", \"batches_per_step\": %lld, \"container_bytes\": %lld, "
                "\"drained_bytes_last_step\": %lld, \"drained_events_last_step\": %lld}\n",
                (long long)nb, (long long)S, (long long)P, T, steps, nb * S * steps / total_s / 1e9, best, median,
                rates.c_str(),
                (long long)(nb * ((S + P - 1) / P)), (long long)stored, (long long)chunks, compressor,
                mixed ? "mixed" : "config2", mirror_mode == 0 ? "none" : mirror_mode == 1 ? "ring" : "socket",
                mirror_ok ? "true" : "false", (long long)mirrored,
                batch ? "hdrf_submit_slots (the blocks received in order since the last submit, <= 16)"
                      : "hdrf_submit_slot (one block per batch)",
                (long long)batches, (long long)container, (long long)timed_drained_bytes,
                (long long)timed_drained_events);
    if (out_dir) {
        const std::string d = out_dir;
        FILE *f = std::fopen((d + "/blocks.txt").c_str(), "w");
        for (int64_t b = 0; b < nb; b++)
            std::fprintf(f, "%lld %lld %lld\n", (long long)b, (long long)n_chunks[(size_t)b], (long long)store[(size_t)b]);
        std::fclose(f);
        for (int64_t b = 0; b < nb && (out_blocks < 0 || b < out_blocks); b++) {
            FILE *g = std::fopen((d + "/blk_" + std::to_string(b) + ".bin").c_str(), "wb");
            const BlockOut &o = bout[(size_t)b];
            std::fwrite(o.off.data(), 4, o.off.size(), g);
            std::fwrite(o.dig.data(), 1, o.dig.size(), g);
            std::fwrite(o.isnew.data(), 1, o.isnew.size(), g);
            std::fclose(g);
        }
        FILE *c = std::fopen((d + "/containers.bin").c_str(), "wb");
        for (auto &kv : disk) {
            const uint32_t id = kv.first, closed = kv.second.second;
            const uint64_t n = kv.second.first.size();
            std::fwrite(&id, 4, 1, c);
            std::fwrite(&closed, 4, 1, c);
            std::fwrite(&n, 8, 1, c);
            std::fwrite(kv.second.first.data(), 1, n, c);
        }
        std::fclose(c);
    }
    hdrf_host_free(ctx, host);
    hdrf_host_free(ctx, dbuf);
    hdrf_close(ctx);
    return mirror_ok ? 0 : 3;
}
