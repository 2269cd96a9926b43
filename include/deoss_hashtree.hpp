// deoss_hashtree.hpp -- C++ host-side mirror of DeOSS common/hashtree over the C ABI.
//
// Same names, argument meaning and error behaviour as the reference Go package:
//   NewHashTree(chunkPath) -> (tree, error)          common/hashtree/types.go:19-39
//   HashTreeContent{CalculateHash, Equals}           common/hashtree/hashtree.go:18-35
//   MerkleTree{Leafs, MerkleRoot()}                  cbergoon/merkletree v0.2.0 (go.mod:10)
// Leafs has n entries, n+1 when n is odd (last leaf duplicated, dup = true), as merkletree's
// buildWithContent makes it.  Interior nodes are not materialised (the GPU reduces the tree).
// Also the Go package's additions: Init / DEOSS_GPUS (every GPU by default), NewHashTreeFromBuffer,
// PinnedBuffer (zero-copy host memory) and the hash-while-receiving Stream.  Header-only; link with -ldeoss_merkle.
#pragma once

#include <array>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "deoss_merkle.h"

namespace hashtree {

using Digest = std::array<uint8_t, 32>;

struct Error {
    int code;
    std::string message;   // "Empty data", "open <path>: no such file or directory", ...
};

struct HashTreeContent {
    std::string x;          // chunk bytes (empty when not kept)
    Digest digest{};        // SHA-256(x) from the GPU leaf kernel
    std::pair<Digest, std::optional<Error>> CalculateHash() const { return {digest, std::nullopt}; }
    std::pair<bool, std::optional<Error>> Equals(const HashTreeContent& o) const {
        if (!x.empty() || !o.x.empty()) return {x == o.x, std::nullopt};
        return {digest == o.digest, std::nullopt};
    }
};

struct Node {
    Digest Hash{};
    HashTreeContent C;
    bool leaf = false;
    bool dup = false;
};

struct MerkleTree {
    std::vector<Node> Leafs;
    Node Root;
    const Digest& MerkleRoot() const { return Root.Hash; }
};

// GPUs of the process-wide context, as the Go package chooses them (go/hashtree/types_hip.go):
// Init(devs) before first use, else DEOSS_GPUS ("0,1,2,3" or "all"), else every visible GPU.
// With more than one, NewHashTree / NewHashTreeFromBuffer shard by aligned chunk ranges.
inline std::vector<int>& selected_devices() {
    static std::vector<int> devs;
    return devs;
}

inline std::vector<int> device_list() {
    if (!selected_devices().empty()) return selected_devices();
    std::vector<int> out;
    const char* env = std::getenv("DEOSS_GPUS");
    std::string spec = env ? env : "";
    if (!spec.empty() && spec != "all") {
        size_t pos = 0;
        while (pos <= spec.size()) {
            const size_t comma = spec.find(',', pos);
            const std::string f = spec.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
            if (!f.empty()) out.push_back(std::atoi(f.c_str()));
            if (comma == std::string::npos) break;
            pos = comma + 1;
        }
        return out;
    }
    for (int i = 0; i < dm_gpu_count(); i++) out.push_back(i);
    return out;
}

// Process-wide GPU context, created on first use.
class Context {
  public:
    static Context& instance() {
        static Context c;
        return c;
    }
    dm_ctx* get() const { return ctx_; }
    int status() const { return rc_; }
    ~Context() {
        if (ctx_) dm_destroy(ctx_);
    }

  private:
    Context() {
        const std::vector<int> devs = device_list();
        rc_ = devs.empty() ? DM_ERR_NODEV : dm_create(&ctx_, devs.data(), (int)devs.size());
    }
    dm_ctx* ctx_ = nullptr;
    int rc_ = DM_OK;
};

// Init(devs) of the Go package: must run before the first call that creates the context.
inline std::optional<Error> Init(const std::vector<int>& devs) {
    if (devs.empty()) return Error{DM_ERR_INVALID, "hashtree: Init needs at least one device"};
    selected_devices() = devs;
    return std::nullopt;
}

// dm_last_error is the calling thread's message: read it right after the failing call.
inline Error make_error(dm_ctx* c, int rc) {
    if (rc == DM_ERR_EMPTY) return {rc, "Empty data"};
    std::string m = dm_last_error(c);
    return {rc, m.empty() ? std::string(dm_strerror(rc)) : m};
}

inline std::unique_ptr<MerkleTree> build(const std::vector<uint8_t>& leaves, const Digest& root) {
    auto t = std::make_unique<MerkleTree>();
    const size_t n = leaves.size() / 32;
    for (size_t i = 0; i < n; i++) {
        Node nd;
        std::copy(leaves.begin() + 32 * i, leaves.begin() + 32 * i + 32, nd.Hash.begin());
        nd.C.digest = nd.Hash;
        nd.leaf = true;
        t->Leafs.push_back(nd);
    }
    if (n % 2 == 1) {   // merkletree v0.2.0 buildWithContent: duplicate the last leaf
        Node d = t->Leafs.back();
        d.dup = true;
        t->Leafs.push_back(d);
    }
    t->Root.Hash = root;
    return t;
}

// types.go:19-39 -- one leaf per file, each read whole.
inline std::pair<std::unique_ptr<MerkleTree>, std::optional<Error>> NewHashTree(
    const std::vector<std::string>& chunkPath) {
    if (chunkPath.empty()) return {nullptr, Error{DM_ERR_EMPTY, "Empty data"}};
    Context& cx = Context::instance();
    if (cx.status() != DM_OK) return {nullptr, Error{cx.status(), dm_strerror(cx.status())}};
    std::vector<const char*> p;
    for (const auto& s : chunkPath) p.push_back(s.c_str());
    std::vector<uint8_t> leaves(32 * chunkPath.size());
    Digest root{};
    int rc = dm_new_hash_tree(cx.get(), p.data(), p.size(), leaves.data(), root.data());
    if (rc != DM_OK) return {nullptr, make_error(cx.get(), rc)};
    return {build(leaves, root), std::nullopt};
}

// Objects up to kBatchLimit bytes go through a process-wide coalescing dm_batcher per chunk size,
// as the Go package does: concurrent callers share GPU passes.  Larger ones take
// dm_root_buffer on the context (ramped striped H2D, zero-copy when pinned, sharded over its GPUs).
constexpr uint64_t kBatchLimit = 256ull << 20;

class Batchers {
  public:
    static Batchers& instance() {
        static Batchers b;
        return b;
    }
    // The batcher for `chunk` (created on first use over the context's GPUs), or an error.
    std::pair<dm_batcher*, std::optional<Error>> get(uint64_t chunk) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = m_.find(chunk);
        if (it != m_.end()) return {it->second, std::nullopt};
        const std::vector<int> devs = device_list();
        dm_batcher* b = nullptr;
        // 2 worker slots per GPU, 4,096 leaves per batch, 2 ms linger
        const int rc = dm_batcher_create(devs.data(), (int)devs.size(), DM_BATCH_ROOT, chunk, 0, 0, 0, 0, 0, 2000, &b);
        if (rc != DM_OK) return {nullptr, Error{rc, dm_batcher_last_error()}};
        m_[chunk] = b;
        return {b, std::nullopt};
    }
    ~Batchers() {
        for (auto& kv : m_) dm_batcher_destroy(kv.second);
    }

  private:
    Batchers() { (void)Context::instance(); }   // fixes the device list; destroyed before it
    std::mutex mu_;
    std::map<uint64_t, dm_batcher*> m_;
};

// Additive: one in-memory object split into chunkSize chunks (the upload-handler buffer).
inline std::pair<std::unique_ptr<MerkleTree>, std::optional<Error>> NewHashTreeFromBuffer(
    const void* buf, uint64_t len, int64_t chunkSize) {
    if (chunkSize <= 0) return {nullptr, Error{DM_ERR_INVALID, "hashtree: chunk size must be positive"}};
    if (len == 0) return {nullptr, Error{DM_ERR_EMPTY, "Empty data"}};
    Context& cx = Context::instance();
    if (cx.status() != DM_OK) return {nullptr, Error{cx.status(), dm_strerror(cx.status())}};
    const uint64_t n = (len + (uint64_t)chunkSize - 1) / (uint64_t)chunkSize;
    std::vector<uint8_t> leaves(32 * n);
    Digest root{};
    if (len <= kBatchLimit) {
        auto [b, err] = Batchers::instance().get((uint64_t)chunkSize);
        if (err) return {nullptr, err};
        const int rc = dm_batcher_root(b, buf, len, leaves.data(), root.data());
        if (rc == DM_ERR_EMPTY) return {nullptr, Error{rc, "Empty data"}};
        if (rc != DM_OK) return {nullptr, Error{rc, dm_batcher_last_error()}};
        return {build(leaves, root), std::nullopt};
    }
    int rc = dm_root_buffer(cx.get(), buf, len, (uint64_t)chunkSize, leaves.data(), root.data());
    if (rc != DM_OK) return {nullptr, make_error(cx.get(), rc)};
    return {build(leaves, root), std::nullopt};
}

// Page-locked host memory (dm_host_alloc), as the Go PinnedBuffer: an object read into it is hashed
// in place by NewHashTreeFromBuffer (zero-copy: the leaf kernel reads it over PCIe).
class PinnedBuffer {
  public:
    static std::pair<std::unique_ptr<PinnedBuffer>, std::optional<Error>> New(uint64_t n) {
        void* p = nullptr;
        const int rc = dm_host_alloc(n, &p);
        if (rc != DM_OK) return {nullptr, make_error(nullptr, rc)};
        return {std::unique_ptr<PinnedBuffer>(new PinnedBuffer(p, n)), std::nullopt};
    }
    uint8_t* data() const { return static_cast<uint8_t*>(p_); }
    uint64_t size() const { return n_; }
    ~PinnedBuffer() { dm_host_free(p_); }
    PinnedBuffer(const PinnedBuffer&) = delete;
    PinnedBuffer& operator=(const PinnedBuffer&) = delete;

  private:
    PinnedBuffer(void* p, uint64_t n) : p_(p), n_(n) {}
    void* p_;
    uint64_t n_;
};

// Hash-while-receiving, as the Go Stream (go/hashtree/stream_hip.go): Write pieces of any size,
// Close() returns the tree NewHashTreeFromBuffer builds over the concatenated bytes, Abort()
// drops it.  One thread at a time per Stream.
class Stream {
  public:
    static std::pair<std::unique_ptr<Stream>, std::optional<Error>> New(int64_t chunkSize) {
        if (chunkSize <= 0 || chunkSize % 16)
            return {nullptr, Error{DM_ERR_INVALID, "hashtree: stream chunk size must be a positive multiple of 16"}};
        Context& cx = Context::instance();
        if (cx.status() != DM_OK) return {nullptr, Error{cx.status(), dm_strerror(cx.status())}};
        std::unique_ptr<Stream> s(new Stream((uint64_t)chunkSize));
        const int rc = dm_stream_open(cx.get(), (uint64_t)chunkSize, &s->st_);
        if (rc != DM_OK) return {nullptr, make_error(cx.get(), rc)};
        return {std::move(s), std::nullopt};
    }
    std::optional<Error> Write(const void* p, uint64_t len) {
        if (!st_) return Error{DM_ERR_INVALID, "hashtree: write on a closed stream"};
        if (err_) return err_;
        if (len == 0) return std::nullopt;
        const int rc = dm_stream_write(st_, p, len);
        if (rc != DM_OK) {
            err_ = make_error(Context::instance().get(), rc);
            return err_;
        }
        received_ += len;
        return std::nullopt;
    }
    std::pair<std::unique_ptr<MerkleTree>, std::optional<Error>> Close() {
        if (!st_) return {nullptr, Error{DM_ERR_INVALID, "hashtree: stream already closed"}};
        dm_stream* st = st_;
        st_ = nullptr;
        if (err_) {
            dm_stream_abort(st);
            return {nullptr, err_};
        }
        const uint64_t n = (received_ + chunk_ - 1) / chunk_;
        std::vector<uint8_t> leaves(32 * (n ? n : 1));
        Digest root{};
        uint64_t got = 0;
        const int rc = dm_stream_close(st, leaves.data(), n, &got, root.data());
        if (rc != DM_OK) return {nullptr, make_error(Context::instance().get(), rc)};
        leaves.resize(32 * n);
        return {build(leaves, root), std::nullopt};
    }
    void Abort() {
        if (st_) dm_stream_abort(st_);
        st_ = nullptr;
    }
    ~Stream() { Abort(); }

  private:
    explicit Stream(uint64_t chunk) : chunk_(chunk) {}
    dm_stream* st_ = nullptr;
    uint64_t chunk_ = 0, received_ = 0;
    std::optional<Error> err_;
};

}  // namespace hashtree
