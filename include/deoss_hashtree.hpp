// deoss_hashtree.hpp -- C++ host-side mirror of DeOSS common/hashtree over the C ABI.
//
// Same names, argument meaning and error behaviour as the reference Go package:
//   NewHashTree(chunkPath) -> (tree, error)          common/hashtree/types.go:19-39
//   HashTreeContent{CalculateHash, Equals}           common/hashtree/hashtree.go:18-35
//   MerkleTree{Leafs, MerkleRoot()}                  cbergoon/merkletree v0.2.0 (go.mod:10)
// Leafs has n entries, n+1 when n is odd (last leaf duplicated, dup = true), as merkletree's
// buildWithContent makes it.  Interior nodes are not materialised (the GPU reduces the tree).
// Header-only; link with -ldeoss_merkle.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
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

// Process-wide GPU context (device 0), created on first use.
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
    Context() { rc_ = dm_create(&ctx_, nullptr, 0); }
    dm_ctx* ctx_ = nullptr;
    int rc_ = DM_OK;
};

inline Error make_error(dm_ctx* c, int rc) {
    if (rc == DM_ERR_EMPTY) return {rc, "Empty data"};
    std::string m = c ? dm_last_error(c) : "";
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

// Additive: one in-memory object split into chunkSize chunks (the upload-handler buffer).
inline std::pair<std::unique_ptr<MerkleTree>, std::optional<Error>> NewHashTreeFromBuffer(
    const void* buf, uint64_t len, uint64_t chunkSize) {
    if (len == 0) return {nullptr, Error{DM_ERR_EMPTY, "Empty data"}};
    Context& cx = Context::instance();
    if (cx.status() != DM_OK) return {nullptr, Error{cx.status(), dm_strerror(cx.status())}};
    const uint64_t n = chunkSize ? (len + chunkSize - 1) / chunkSize : 0;
    std::vector<uint8_t> leaves(32 * n);
    Digest root{};
    int rc = dm_root_buffer(cx.get(), buf, len, chunkSize, leaves.data(), root.data());
    if (rc != DM_OK) return {nullptr, make_error(cx.get(), rc)};
    return {build(leaves, root), std::nullopt};
}

}  // namespace hashtree
