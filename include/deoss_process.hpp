// deoss_process.hpp -- C++ host mirror of the Go process shim (go/process): cess-go-sdk
// process.FullProcessing(file, cipher, savedir) (go.mod:8; node/objectHandler.go:168,
// node/fileHandler.go:771, node/filesHandler.go:201, node/resumeHandler.go:326,
// node/tracker.go:767-769) and the streaming Writer (go/process/stream_hip.go), over the C ABI
// (include/deoss_merkle.h: dm_full_processing, dm_pstream_*).  Same result shape: segment and
// fragment path names under savedir (every one exists as a file), the hex fid, an error.
// Deviation (as in Go): a non-empty cipher is an error.  Header-only; link -ldeoss_merkle.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <memory>
#include <optional>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "deoss_merkle.h"

namespace process {

constexpr uint64_t SegmentSize = 32ull << 20;   // chain.SegmentSize
constexpr int DataShards = 4, ParShards = 8;    // chain.DataShards / chain.ParShards

struct Error {
    int code;
    std::string message;
};

struct SegmentDataInfo {   // chain.SegmentDataInfo
    std::string SegmentHash;
    std::vector<std::string> FragmentHash;
};

using Result = std::tuple<std::vector<SegmentDataInfo>, std::string, std::optional<Error>>;

// One coder per visible GPU, created on first use; calls pick one round robin (each call holds
// its coder's context for its duration, so concurrent calls spread over the GPUs).
class Pipelines {
  public:
    static Pipelines& instance() {
        static Pipelines p;
        return p;
    }
    dm_rs* pick() { return rs_.empty() ? nullptr : rs_[next_++ % rs_.size()]; }
    int status() const { return rc_; }
    ~Pipelines() {
        for (dm_rs* r : rs_) dm_rs_destroy(r);
        for (dm_ctx* c : ctx_) dm_destroy(c);
    }

  private:
    Pipelines() {
        const int n = dm_gpu_count();
        if (n <= 0) rc_ = DM_ERR_NODEV;
        for (int g = 0; g < n && rc_ == DM_OK; g++) {
            dm_ctx* c = nullptr;
            dm_rs* r = nullptr;
            if ((rc_ = dm_create(&c, &g, 1)) != DM_OK) break;
            ctx_.push_back(c);
            if ((rc_ = dm_rs_create(c, DataShards, ParShards, &r)) != DM_OK) break;
            rs_.push_back(r);
        }
    }
    std::vector<dm_ctx*> ctx_;
    std::vector<dm_rs*> rs_;
    std::atomic<uint64_t> next_{0};
    int rc_ = DM_OK;
};

inline bool write_segments() {
    const char* v = std::getenv("DEOSS_SKIP_SEGMENT_FILES");
    return !(v && v[0] == '1' && v[1] == 0);
}

inline Error last_error(int rc) {   // dm_last_error is the calling thread's message
    if (rc == DM_ERR_EMPTY) return {rc, "Empty data"};
    std::string m = dm_last_error(nullptr);
    return {rc, m.empty() ? std::string(dm_strerror(rc)) : m};
}

inline std::string hex32(const uint8_t* d) {
    static const char* x = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; i++) {
        s[2 * i] = x[d[i] >> 4];
        s[2 * i + 1] = x[d[i] & 15];
    }
    return s;
}

inline std::string join(const std::string& dir, const std::string& name) {
    return dir.empty() || dir.back() == '/' ? dir + name : dir + "/" + name;
}

inline std::vector<SegmentDataInfo> infos(const std::string& savedir, const std::vector<uint8_t>& segd,
                                          const std::vector<uint8_t>& fragd, uint64_t nseg) {
    const int total = DataShards + ParShards;
    std::vector<SegmentDataInfo> out(nseg);
    for (uint64_t s = 0; s < nseg; s++) {
        out[s].SegmentHash = join(savedir, hex32(segd.data() + 32 * s));
        for (int j = 0; j < total; j++) out[s].FragmentHash.push_back(join(savedir, hex32(fragd.data() + 32 * (s * total + j))));
    }
    return out;
}

// FullProcessing(file, cipher, savedir): one dm_full_processing call (the library reads the file
// and writes every fragment and segment file to savedir/<hex SHA-256>).
inline Result FullProcessing(const std::string& file, const std::string& cipher, const std::string& savedir) {
    if (!cipher.empty()) return {{}, "", Error{DM_ERR_INVALID, "process: cipher is not supported by the GPU pipeline"}};
    auto& p = Pipelines::instance();
    dm_rs* rs = p.pick();
    if (!rs) return {{}, "", Error{p.status(), dm_strerror(p.status())}};
    const int flags = write_segments() ? DM_FP_SEGMENT_FILES : 0;
    uint64_t cap = 1;
    for (int attempt = 0; attempt < 3; attempt++) {   // cap from the library's count when too small
        std::vector<uint8_t> segd(32 * cap), fragd(32 * cap * (DataShards + ParShards));
        uint8_t fid[32];
        uint64_t nseg = 0;
        const int rc = dm_full_processing(rs, file.c_str(), savedir.c_str(), SegmentSize, flags, segd.data(),
                                          fragd.data(), cap, &nseg, fid);
        if (rc == DM_ERR_INVALID && nseg > cap) {
            cap = nseg;
            continue;
        }
        if (rc != DM_OK) return {{}, "", last_error(rc)};
        return {infos(savedir, segd, fragd, nseg), hex32(fid), std::nullopt};
    }
    return {{}, "", Error{DM_ERR_INVALID, "process: file size changed during the call"}};
}

// FindFragment(fpath, fragmentHash) (go/process: the download handler's one fragment,
// node/fileHandler.go:962-979): the fragment bytes, an empty vector when the file has no fragment
// of that name, or an error.  dm_fragment_lookup: nothing is written to disk.
inline std::pair<std::vector<uint8_t>, std::optional<Error>> FindFragment(const std::string& fpath,
                                                                          const std::string& fragment_hash) {
    // fragment files are named by lower-case hex SHA-256 and the handler compares strings
    // (node/fileHandler.go:968): any other spelling names no fragment (not found, no error)
    uint8_t want[32];
    auto nib = [](char ch) -> int { return ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10 : -1; };
    bool ok = fragment_hash.size() == 64;
    for (int i = 0; ok && i < 32; i++) {
        const int hi = nib(fragment_hash[2 * i]), lo = nib(fragment_hash[2 * i + 1]);
        ok = hi >= 0 && lo >= 0;
        want[i] = (uint8_t)(hi * 16 + lo);
    }
    if (!ok) return {{}, std::nullopt};
    auto& p = Pipelines::instance();
    dm_rs* rs = p.pick();
    if (!rs) return {{}, Error{p.status(), dm_strerror(p.status())}};
    std::vector<uint8_t> out(SegmentSize / DataShards);
    int found = 0, idx = 0;
    uint64_t seg = 0;
    const int rc = dm_fragment_lookup(rs, fpath.c_str(), SegmentSize, want, out.data(), out.size(), &found, &seg, &idx);
    if (rc != DM_OK) return {{}, last_error(rc)};
    if (!found) out.clear();
    return {std::move(out), std::nullopt};
}

// FullProcessing while the body arrives (dm_pstream_*): Write the pieces, then Close.
class Writer {
  public:
    static std::pair<std::unique_ptr<Writer>, std::optional<Error>> New(const std::string& savedir) {
        auto& p = Pipelines::instance();
        dm_rs* rs = p.pick();
        if (!rs) return {nullptr, Error{p.status(), dm_strerror(p.status())}};
        std::unique_ptr<Writer> w(new Writer(savedir));
        const int rc = dm_pstream_open(rs, SegmentSize, savedir.c_str(), write_segments() ? DM_FP_SEGMENT_FILES : 0, &w->st_);
        if (rc != DM_OK) return {nullptr, last_error(rc)};
        return {std::move(w), std::nullopt};
    }
    std::optional<Error> Write(const void* p, uint64_t len) {
        if (!st_) return Error{DM_ERR_INVALID, "process: write on a closed Writer"};
        const int rc = dm_pstream_write(st_, p, len);
        if (rc != DM_OK) {
            Error e = last_error(rc);
            Abort();
            return e;
        }
        n_ += len;
        return std::nullopt;
    }
    Result Close() {
        if (!st_) return {{}, "", Error{DM_ERR_INVALID, "process: Writer already closed"}};
        const uint64_t cap = std::max<uint64_t>(1, (n_ + SegmentSize - 1) / SegmentSize);
        std::vector<uint8_t> segd(32 * cap), fragd(32 * cap * (DataShards + ParShards));
        uint8_t fid[32];
        uint64_t nseg = 0;
        dm_pstream* st = st_;
        st_ = nullptr;
        const int rc = dm_pstream_close(st, segd.data(), fragd.data(), cap, &nseg, fid);
        if (rc != DM_OK) return {{}, "", last_error(rc)};
        return {infos(savedir_, segd, fragd, nseg), hex32(fid), std::nullopt};
    }
    void Abort() {
        if (st_) dm_pstream_abort(st_);
        st_ = nullptr;
    }
    ~Writer() { Abort(); }

  private:
    explicit Writer(std::string savedir) : savedir_(std::move(savedir)) {}
    std::string savedir_;
    dm_pstream* st_ = nullptr;
    uint64_t n_ = 0;
};

}  // namespace process
