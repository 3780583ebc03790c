// hdrf_scheme.hpp — C++ host-side mirror of HDRF's reduction-scheme plugin interface.
//
// HDRF's README promises an abstract `ReductionScheme` (README.md:3); the de-facto API in the
// reference is
//   write:  new DataDeduplicator(ByteBuffer block, long blockId)     DN/DataDeduplicator.java:108
//           started per block by DDRunner                             DN/DDRunner.java:20-36
//   read:   new DataConstructor(long blkID, byte[] recipe).data       DN/DataConstructor.java:46-73
//   length: FsDatasetImpl.getLength via Redis GET id                  DN/fsdataset/impl/FsDatasetImpl.java:736-763
// The Java toolchain is absent in this image, so the interface is mirrored here (and in
// hdrf_amd/scheme.py); INTEGRATION.md shows the Java class and JNI stub over the same C-ABI.
// Header-only; link with libhdrf.so.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "hdrf.h"

namespace hdrf {

struct ReduceResult {
    std::vector<uint32_t> offsets;
    std::vector<uint8_t> digests;
    std::vector<uint8_t> is_new;
    std::vector<uint32_t> container_id, container_pos;
    int64_t store_size = 0;
};

class Error : public std::runtime_error {
  public:
    Error(int code, const std::string &m) : std::runtime_error(m + " (code " + std::to_string(code) + ")"), code(code) {}
    int code;
};

// Abstract scheme: one instance per DataNode; reduce() is called once per received block in
// arrival order (the FIFO of DN/DataDeduplicator.java:124-158).
class ReductionScheme {
  public:
    virtual ~ReductionScheme() = default;
    virtual ReduceResult reduce(const uint8_t *block, uint64_t len, uint64_t block_id) = 0;
    virtual std::vector<uint8_t> reconstruct(uint64_t block_id) = 0;
    virtual int64_t length(uint64_t block_id) = 0;
};

// MI355X backend (compressor 1 = dedup, 2 = dedup + Lz4Codec containers).
class HipReductionScheme final : public ReductionScheme {
  public:
    explicit HipReductionScheme(const hdrf_cfg *cfg = nullptr)
    {
        hdrf_cfg c;
        hdrf_default_cfg(&c);
        if (cfg) c = *cfg;
        int rc = hdrf_open(&c, &ctx_);
        if (rc) throw Error(rc, "hdrf_open failed");
        window_ = c.window;
        H_ = hdrf_digest_len(ctx_);
    }
    ~HipReductionScheme() override
    {
        if (ctx_) hdrf_close(ctx_);
    }
    HipReductionScheme(const HipReductionScheme &) = delete;
    HipReductionScheme &operator=(const HipReductionScheme &) = delete;

    ReduceResult reduce(const uint8_t *block, uint64_t len, uint64_t block_id) override
    {
        const int64_t cap = (int64_t)(len / (uint64_t)(window_ + 2) + 2);
        ReduceResult r;
        r.offsets.resize(cap);
        r.digests.resize((size_t)cap * H_);
        r.is_new.resize(cap);
        r.container_id.resize(cap);
        r.container_pos.resize(cap);
        hdrf_block_result out{};
        out.capacity = cap;
        out.offsets = r.offsets.data();
        out.digests = r.digests.data();
        out.is_new = r.is_new.data();
        out.container_id = r.container_id.data();
        out.container_pos = r.container_pos.data();
        check(hdrf_reduce_block(ctx_, block_id, block, len, &out));
        const size_t n = (size_t)out.n_chunks;
        r.offsets.resize(n);
        r.digests.resize(n * H_);
        r.is_new.resize(n);
        r.container_id.resize(n);
        r.container_pos.resize(n);
        r.store_size = out.store_size;
        return r;
    }

    std::vector<uint8_t> reconstruct(uint64_t block_id) override
    {
        const int64_t len = hdrf_block_length(ctx_, block_id);
        if (len < 0) check((int)len);
        std::vector<uint8_t> out((size_t)len);
        const int64_t n = hdrf_reconstruct_block(ctx_, block_id, out.data(), len);
        if (n < 0) check((int)n);
        out.resize((size_t)n);
        return out;
    }

    int64_t length(uint64_t block_id) override
    {
        int64_t n = hdrf_block_length(ctx_, block_id);
        if (n < 0) check((int)n);
        return n;
    }

    std::vector<uint8_t> recipe(uint64_t block_id)
    {
        const int64_t len = hdrf_block_length(ctx_, block_id);
        if (len < 0) return {};
        std::vector<uint8_t> out(4 + (size_t)H_ * (size_t)(len / (window_ + 2) + 2));
        int64_t n = hdrf_recipe_get(ctx_, block_id, out.data(), (int64_t)out.size());
        if (n < 0) check((int)n);
        out.resize((size_t)n);
        return out;
    }

    bool index_get(const uint8_t *digest, uint8_t out11[11])
    {
        int rc = hdrf_index_get(ctx_, digest, out11);
        if (rc < 0) check(rc);
        return rc == 1;
    }

    hdrf_ctx *handle() { return ctx_; }

  private:
    void check(int rc)
    {
        if (rc < 0) throw Error(rc, hdrf_last_error(ctx_));
    }
    hdrf_ctx *ctx_ = nullptr;
    int window_ = 700;
    int H_ = 20;
};

}  // namespace hdrf
