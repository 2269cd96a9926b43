// Exercise every C-ABI entry point of libdeoss_merkle (include/deoss_merkle.h) from C++, checked
// against the CPU oracle (oracle/liboracle_merkle.so, linked as the checker only).  Built twice
// by tests/cpp/run_host_tests.sh: plain, and with the library's HOST code compiled under
// AddressSanitizer + UBSan (-Xarch_host -fsanitize=...; device code is not instrumented).
// Prints PASS and exits 0 when everything matches.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <fstream>
#include <iterator>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "deoss_merkle.h"

extern "C" {
int or_root_buffer(const void* buf, uint64_t len, uint64_t chunk, uint8_t* leaf_out, uint8_t root[32], int nthreads);
int or_root_chunks(const void* const* ptrs, const uint64_t* lens, uint64_t n, uint8_t* leaf_out, uint8_t root[32],
                   int nthreads);
void or_fill_splitmix(void* dst, uint64_t off, uint64_t nbytes, uint64_t seed);
int or_rs_encode(int data, int parity, const uint8_t* const* dshards, uint8_t* const* pshards, size_t shard,
                 int nthreads);
int64_t or_full_processing(const void* buf, uint64_t len, uint64_t segment, int data, int parity,
                           uint8_t* seg_hashes, uint8_t* frag_hashes, uint8_t fid[32], uint8_t* frags, int nthreads);
uint64_t or_reduce(const uint8_t* digests, uint64_t n, int levels, uint8_t* out);
void or_sha256(const void* data, uint64_t len, uint8_t out[32]);
}

static std::atomic<int> fails{0};
#define EXPECT(c)                                                                     \
    do {                                                                              \
        if (!(c)) {                                                                   \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);         \
            fails++;                                                                  \
        }                                                                             \
    } while (0)

static std::vector<uint8_t> bytes(uint64_t n, uint64_t seed) {
    std::vector<uint8_t> v((n + 7) / 8 * 8 + 8);
    or_fill_splitmix(v.data(), 0, v.size() - 8, seed);
    v.resize(n);
    return v;
}

static void check_buffer(dm_ctx* c, uint64_t len, uint64_t chunk, uint64_t seed) {
    auto b = bytes(len, seed);
    const uint64_t n = (len + chunk - 1) / chunk;
    std::vector<uint8_t> lw(32 * n), lg(32 * n);
    uint8_t rw[32], rg[32];
    EXPECT(or_root_buffer(b.data(), len, chunk, lw.data(), rw, 4) == 0);
    EXPECT(dm_root_buffer(c, b.data(), len, chunk, lg.data(), rg) == DM_OK);
    EXPECT(std::memcmp(rw, rg, 32) == 0);
    EXPECT(lw == lg);
    // device-resident forms
    void* dev = nullptr;
    EXPECT(hipMalloc(&dev, len + 64) == hipSuccess);
    EXPECT(hipMemcpy(dev, b.data(), len, hipMemcpyHostToDevice) == hipSuccess);
    uint8_t rd[32];
    EXPECT(dm_root_device(c, dev, len, chunk, rd) == DM_OK);
    EXPECT(std::memcmp(rw, rd, 32) == 0);
    void* droot = nullptr;
    EXPECT(hipMalloc(&droot, 32) == hipSuccess);
    EXPECT(dm_root_device_async(c, dev, len, chunk, droot, nullptr, nullptr) == DM_OK);
    EXPECT(hipDeviceSynchronize() == hipSuccess);
    EXPECT(hipMemcpy(rd, droot, 32, hipMemcpyDeviceToHost) == hipSuccess);
    EXPECT(std::memcmp(rw, rd, 32) == 0);
    // subtree + finish over two halves at a block boundary
    if (n >= 4) {
        uint32_t k = 0;
        while ((2ull << k) * 2 <= n) k++;
        const uint64_t split = (n / (1ull << k) / 2) * (1ull << k) * chunk;
        if (split > 0 && split < len) {
            void* nodes = nullptr;
            EXPECT(hipMalloc(&nodes, 32 * (n + 2)) == hipSuccess);
            uint64_t c1 = 0, c2 = 0;
            EXPECT(dm_subtree_device_async(c, dev, split, chunk, k, nodes, &c1, nullptr) == DM_OK);
            EXPECT(dm_subtree_device_async(c, (uint8_t*)dev + split, len - split, chunk, k, (uint8_t*)nodes + 32 * c1,
                                           &c2, nullptr) == DM_OK);
            EXPECT(dm_finish_device_async(c, nodes, c1 + c2, k == 0, droot, nullptr) == DM_OK);
            EXPECT(hipDeviceSynchronize() == hipSuccess);
            EXPECT(hipMemcpy(rd, droot, 32, hipMemcpyDeviceToHost) == hipSuccess);
            EXPECT(std::memcmp(rw, rd, 32) == 0);
            (void)hipFree(nodes);
        }
    }
    (void)hipFree(droot);
    (void)hipFree(dev);
    // streaming with random piece sizes
    dm_stream* st = nullptr;
    if (chunk % 16 == 0) {
        EXPECT(dm_stream_open(c, chunk, &st) == DM_OK);
        std::mt19937_64 rng(seed);
        uint64_t pos = 0;
        while (pos < len) {
            uint64_t m = std::min<uint64_t>(len - pos, 1 + rng() % (3u << 20));
            EXPECT(dm_stream_write(st, b.data() + pos, m) == DM_OK);
            pos += m;
        }
        uint64_t nl = 0;
        std::vector<uint8_t> ls(32 * n);
        uint8_t rs[32];
        EXPECT(dm_stream_close(st, ls.data(), n, &nl, rs) == DM_OK);
        EXPECT(nl == n && std::memcmp(rw, rs, 32) == 0 && ls == lw);
    }
}

// Write files under dir, return their paths (the NewHashTree inputs).
static std::vector<std::string> write_files(const std::string& dir, const std::vector<std::vector<uint8_t>>& data,
                                            const char* tag) {
    std::vector<std::string> paths;
    for (size_t i = 0; i < data.size(); i++) {
        paths.push_back(dir + "/" + tag + std::to_string(i));
        std::ofstream f(paths.back(), std::ios::binary);
        f.write(reinterpret_cast<const char*>(data[i].data()), (std::streamsize)data[i].size());
    }
    return paths;
}

// dm_new_hash_tree over files vs or_root_chunks over the same bytes (leaves and root).
static void check_files(dm_ctx* c, const std::string& dir, const std::vector<std::vector<uint8_t>>& data,
                        const char* tag) {
    auto paths = write_files(dir, data, tag);
    std::vector<const char*> cp;
    std::vector<const void*> ptrs;
    std::vector<uint64_t> lens;
    for (size_t i = 0; i < data.size(); i++) {
        cp.push_back(paths[i].c_str());
        ptrs.push_back(data[i].data());
        lens.push_back(data[i].size());
    }
    const uint64_t n = data.size();
    std::vector<uint8_t> lw(32 * n), lg(32 * n);
    uint8_t rw[32], rg[32];
    EXPECT(or_root_chunks(ptrs.data(), lens.data(), n, lw.data(), rw, 4) == 0);
    EXPECT(dm_new_hash_tree(c, cp.data(), n, lg.data(), rg) == DM_OK);
    EXPECT(std::memcmp(rw, rg, 32) == 0 && lw == lg);
    for (auto& p : paths) std::remove(p.c_str());
}

// The Go Stream call sequence (go/hashtree/stream_hip.go): NewStream, Write pieces of random
// sizes, Close with leaf_cap = ceil(received / chunk); or Abort mid-body.
static void go_stream_sequence(dm_ctx* c, uint64_t len, uint64_t chunk, uint64_t seed, bool abort_midway) {
    auto b = bytes(len, seed);
    dm_stream* st = nullptr;
    EXPECT(dm_stream_open(c, chunk, &st) == DM_OK);
    std::mt19937_64 rng(seed * 31 + 7);
    uint64_t pos = 0;
    while (pos < len) {
        const uint64_t m = std::min<uint64_t>(len - pos, 1 + rng() % (2u << 20));
        EXPECT(dm_stream_write(st, b.data() + pos, m) == DM_OK);
        pos += m;
        if (abort_midway && pos > len / 2) {
            dm_stream_abort(st);
            return;
        }
    }
    const uint64_t n = (len + chunk - 1) / chunk;
    std::vector<uint8_t> lw(32 * n), lg(32 * n);
    uint8_t rw[32], rg[32];
    uint64_t got = 0;
    EXPECT(or_root_buffer(b.data(), len, chunk, lw.data(), rw, 2) == 0);
    EXPECT(dm_stream_close(st, lg.data(), n, &got, rg) == DM_OK);
    EXPECT(got == n && std::memcmp(rw, rg, 32) == 0 && lw == lg);
}

// One thread's mix of host-memory calls (buffers, streams -- some aborted --, batches), each
// checked against the oracle: the concurrent-routing workload of the multi-device / lanes blocks.
static void mixed_calls(dm_ctx* cv, int t) {
    for (int i = 0; i < 3; i++) {
        switch ((t + i) % 3) {
            case 0: check_buffer(cv, 150000 + 4099 * (3 * t + i), 8192, 1300 + 3 * t + i); break;
            case 1: go_stream_sequence(cv, 2000000 + 777 * t, 65536, 1400 + t, (t + i) % 5 == 0); break;
            default: {
                std::vector<std::vector<uint8_t>> objs;
                for (int o = 0; o < 5; o++) objs.push_back(bytes(30000 + 1000 * o + t, 1500 + 10 * t + o));
                std::vector<const void*> op;
                std::vector<uint64_t> ol;
                for (auto& o : objs) {
                    op.push_back(o.data());
                    ol.push_back(o.size());
                }
                std::vector<uint8_t> roots(32 * objs.size());
                EXPECT(dm_root_batch(cv, op.data(), ol.data(), objs.size(), 4096, roots.data()) == DM_OK);
                for (size_t o = 0; o < objs.size(); o++) {
                    uint8_t r[32];
                    EXPECT(or_root_buffer(objs[o].data(), objs[o].size(), 4096, nullptr, r, 1) == 0);
                    EXPECT(std::memcmp(r, roots.data() + 32 * o, 32) == 0);
                }
            }
        }
    }
}

int main(int argc, char** argv) {
    const std::string tmpdir = argc > 1 ? argv[1] : "/tmp";
    dm_ctx* c = nullptr;
    int rc = dm_create(&c, nullptr, 0);
    if (rc != DM_OK) {
        std::fprintf(stderr, "dm_create: %s\n", dm_strerror(rc));
        return 1;
    }
    // argument errors
    uint8_t root[32];
    EXPECT(dm_root_buffer(c, nullptr, 0, 64, nullptr, root) == DM_ERR_EMPTY);
    EXPECT(std::string(dm_last_error(c)) == "Empty data");
    EXPECT(dm_root_buffer(c, root, 1, 0, nullptr, root) == DM_ERR_INVALID);
    EXPECT(dm_root_chunks(c, nullptr, nullptr, 0, nullptr, root) == DM_ERR_EMPTY);
    EXPECT(dm_set_leaf_kernel(c, 9) == DM_ERR_INVALID);
    EXPECT(dm_set_leaf_kernel(c, 5) == DM_ERR_INVALID);
    EXPECT(std::string(dm_strerror(DM_ERR_EMPTY)) == "Empty data");
    dm_stream* bad = nullptr;
    EXPECT(dm_stream_open(c, 100, &bad) == DM_ERR_INVALID && bad == nullptr);
    const char* missing[] = {"/nonexistent/deoss/chunk"};
    EXPECT(dm_new_hash_tree(c, missing, 1, nullptr, root) == DM_ERR_IO);
    EXPECT(std::string(dm_last_error(c)).find("no such file or directory") != std::string::npos);

    for (int mode : {DM_LEAF_AUTO, DM_LEAF_WIDE, DM_LEAF_LATENCY, DM_LEAF_PAIR, DM_LEAF_QUAD}) {
        EXPECT(dm_set_leaf_kernel(c, mode) == DM_OK);
        check_buffer(c, 1, 64, 1);
        check_buffer(c, 100000, 1000, 2);
        check_buffer(c, (3u << 20) + 5, 4096, 3);
        check_buffer(c, (5u << 20) + 17, 1u << 20, 4);
    }
    EXPECT(dm_set_leaf_kernel(c, DM_LEAF_AUTO) == DM_OK);
    check_buffer(c, (300ull << 20) + 3, 64ull << 20, 5);   // striped host path

    // where the last call ran (round 4): one device, a valid lane; no exchange without sharding
    {
        int devs[4] = {-1, -1, -1, -1}, ids[4] = {-1, -1, -1, -1}, lane = -9;
        EXPECT(dm_last_call_devices(c, devs, ids, 4, &lane) == 1);
        EXPECT(devs[0] == 0 && ids[0] == 0 && lane >= 0 && lane < dm_lane_count(c));
        EXPECT(dm_last_call_devices(nullptr, devs, ids, 4, &lane) == DM_ERR_INVALID);
        uint64_t xn = 9;
        double xs = -1, xm = -1;
        int xg = -1;
        EXPECT(dm_set_timing(c, 1) == DM_OK);
        check_buffer(c, (3u << 20) + 5, 4096, 6);
        EXPECT(dm_exchange_timing(c, &xn, &xs, &xm, &xg) == DM_OK && xn == 0 && xs == 0 && xg == 0);
        EXPECT(dm_set_timing(c, 0) == DM_OK);
    }

    // chunk list with empty chunks, and batches
    std::vector<std::vector<uint8_t>> ch;
    for (int i = 0; i < 37; i++) ch.push_back(bytes((i * 977) % 5000, 100 + i));
    std::vector<const void*> ptrs;
    std::vector<uint64_t> lens;
    for (auto& v : ch) {
        ptrs.push_back(v.data());
        lens.push_back(v.size());
    }
    uint8_t rw[32], rg[32];
    std::vector<uint8_t> lw(32 * ch.size()), lg(32 * ch.size());
    EXPECT(or_root_chunks(ptrs.data(), lens.data(), ch.size(), lw.data(), rw, 1) == 0);
    EXPECT(dm_root_chunks(c, ptrs.data(), lens.data(), ch.size(), lg.data(), rg) == DM_OK);
    EXPECT(std::memcmp(rw, rg, 32) == 0 && lw == lg);
    for (auto& l : lens) l = l ? l : 1;
    std::vector<std::vector<uint8_t>> objs;
    for (size_t i = 0; i < ch.size(); i++) objs.push_back(bytes(lens[i] * 13, 500 + i));
    std::vector<const void*> op;
    std::vector<uint64_t> ol;
    for (auto& v : objs) {
        op.push_back(v.data());
        ol.push_back(v.size());
    }
    std::vector<uint8_t> roots(32 * objs.size());
    EXPECT(dm_root_batch(c, op.data(), ol.data(), objs.size(), 4096, roots.data()) == DM_OK);
    for (size_t i = 0; i < objs.size(); i++) {
        uint8_t r[32];
        or_root_buffer(objs[i].data(), ol[i], 4096, nullptr, r, 1);
        EXPECT(std::memcmp(r, roots.data() + 32 * i, 32) == 0);
    }

    // Reed-Solomon 4 + 8: host encode / reconstruct / verify / split, device encode, vs the oracle
    {
        dm_rs* rs = nullptr;
        EXPECT(dm_rs_create(c, 9, 2, &rs) == DM_ERR_INVALID && rs == nullptr);
        EXPECT(dm_rs_create(c, 4, 8, &rs) == DM_OK && rs != nullptr);
        uint8_t mat[12 * 4];
        EXPECT(dm_rs_matrix(rs, mat) == DM_OK && mat[0] == 1 && mat[5] == 1 && mat[16] == 0x1b);
        for (uint64_t shard : {1ull, 17ull, 4096ull, 100003ull}) {
            std::vector<std::vector<uint8_t>> sh(12);
            for (int j = 0; j < 4; j++) sh[j] = bytes(shard, 7000 + j + shard);
            for (int i = 4; i < 12; i++) sh[i].assign(shard, 0);
            std::vector<std::vector<uint8_t>> want(8, std::vector<uint8_t>(shard));
            const uint8_t* dp[4];
            uint8_t* wp[8];
            void* pp[8];
            for (int j = 0; j < 4; j++) dp[j] = sh[j].data();
            for (int i = 0; i < 8; i++) {
                wp[i] = want[i].data();
                pp[i] = sh[4 + i].data();
            }
            EXPECT(or_rs_encode(4, 8, dp, wp, shard, 1) == 0);
            EXPECT(dm_rs_encode(rs, reinterpret_cast<const void* const*>(dp), pp, shard) == DM_OK);
            for (int i = 0; i < 8; i++) EXPECT(sh[4 + i] == want[i]);
            std::vector<void*> all(12);
            for (int i = 0; i < 12; i++) all[i] = sh[i].data();
            int ok = 0;
            EXPECT(dm_rs_verify(rs, all.data(), shard, &ok) == DM_OK && ok == 1);
            auto keep = sh;
            uint8_t present[12];
            for (int i = 0; i < 12; i++) present[i] = (i % 3 == 1) || i == 11;   // 1,4,7,10,11
            for (int i = 0; i < 12; i++)
                if (!present[i]) std::fill(sh[i].begin(), sh[i].end(), 0xEE);
            EXPECT(dm_rs_reconstruct(rs, all.data(), present, shard) == DM_OK);
            EXPECT(sh == keep);
            uint8_t few[12] = {1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
            EXPECT(dm_rs_reconstruct(rs, all.data(), few, shard) == DM_ERR_INVALID);
        }
        // Split + Encode of one odd-sized segment
        auto seg = bytes(1001, 99);
        std::vector<uint8_t> out(12 * 251);
        uint64_t per = 0;
        EXPECT(dm_rs_encode_buffer(rs, seg.data(), seg.size(), out.data(), &per) == DM_OK && per == 251);
        EXPECT(std::memcmp(out.data(), seg.data(), seg.size()) == 0 && out[1001] == 0 && out[1003] == 0);
        EXPECT(dm_rs_encode_buffer(rs, seg.data(), 0, out.data(), &per) == DM_ERR_EMPTY);
        // device-resident batch: 3 segments of 4 x 4096 bytes
        const uint64_t shard = 4096, nseg = 3;
        auto data = bytes(nseg * 4 * shard, 4242);
        void *dd = nullptr, *dpar = nullptr;
        EXPECT(hipMalloc(&dd, data.size()) == hipSuccess && hipMalloc(&dpar, nseg * 8 * shard) == hipSuccess);
        EXPECT(hipMemcpy(dd, data.data(), data.size(), hipMemcpyHostToDevice) == hipSuccess);
        EXPECT(dm_rs_encode_device_async(rs, dd, 4 * shard, dpar, 8 * shard, shard, nseg, nullptr) == DM_OK);
        EXPECT(dm_rs_encode_device_async(rs, (uint8_t*)dd + 1, 4 * shard, dpar, 8 * shard, shard, nseg, nullptr) ==
               DM_ERR_INVALID);
        EXPECT(hipDeviceSynchronize() == hipSuccess);
        std::vector<uint8_t> par(nseg * 8 * shard);
        EXPECT(hipMemcpy(par.data(), dpar, par.size(), hipMemcpyDeviceToHost) == hipSuccess);
        for (uint64_t s2 = 0; s2 < nseg; s2++) {
            const uint8_t* dp[4];
            std::vector<std::vector<uint8_t>> want(8, std::vector<uint8_t>(shard));
            uint8_t* wp[8];
            for (int j = 0; j < 4; j++) dp[j] = data.data() + s2 * 4 * shard + j * shard;
            for (int i = 0; i < 8; i++) wp[i] = want[i].data();
            EXPECT(or_rs_encode(4, 8, dp, wp, shard, 1) == 0);
            for (int i = 0; i < 8; i++)
                EXPECT(std::memcmp(par.data() + s2 * 8 * shard + i * shard, want[i].data(), shard) == 0);
        }
        // device reconstruct of segment 0 with fragments 0, 2 and 9 lost
        void* dev_sh[12];
        std::vector<void*> fr(12);
        void* dall = nullptr;
        EXPECT(hipMalloc(&dall, 12 * shard) == hipSuccess);
        EXPECT(hipMemcpy(dall, data.data(), 4 * shard, hipMemcpyHostToDevice) == hipSuccess);
        EXPECT(hipMemcpy((uint8_t*)dall + 4 * shard, par.data(), 8 * shard, hipMemcpyHostToDevice) == hipSuccess);
        EXPECT(hipMemset(dall, 0, shard) == hipSuccess);
        for (int i = 0; i < 12; i++) dev_sh[i] = (uint8_t*)dall + i * shard;
        uint8_t pres[12] = {0, 1, 0, 1, 1, 1, 1, 1, 1, 0, 1, 1};
        EXPECT(dm_rs_reconstruct_device_async(rs, dev_sh, pres, shard, nullptr) == DM_OK);
        EXPECT(hipDeviceSynchronize() == hipSuccess);
        std::vector<uint8_t> back(12 * shard);
        EXPECT(hipMemcpy(back.data(), dall, back.size(), hipMemcpyDeviceToHost) == hipSuccess);
        EXPECT(std::memcmp(back.data(), data.data(), 4 * shard) == 0);
        EXPECT(std::memcmp(back.data() + 4 * shard, par.data(), 8 * shard) == 0);
        (void)hipFree(dall);
        (void)hipFree(dd);
        (void)hipFree(dpar);
        dm_rs_destroy(rs);
    }

    // FullProcessing: host and device forms vs the oracle (small segments, 4 + 8)
    {
        dm_rs* rs = nullptr;
        EXPECT(dm_rs_create(c, 4, 8, &rs) == DM_OK);
        const uint64_t seg = 4096, frag = seg / 4;
        for (uint64_t len : {1ull, 4096ull, 4097ull, 50000ull}) {
            const uint64_t nseg = (len + seg - 1) / seg;
            auto obj = bytes(len, 31337 + len);
            std::vector<uint8_t> ws(32 * nseg), wf(32 * nseg * 12), wfr(nseg * 12 * frag), gs(ws.size()),
                gf(wf.size()), gfr(wfr.size());
            uint8_t wfid[32], gfid[32];
            EXPECT(or_full_processing(obj.data(), len, seg, 4, 8, ws.data(), wf.data(), wfid, wfr.data(), 1) ==
                   (int64_t)nseg);
            EXPECT(dm_process_buffer(rs, obj.data(), len, seg, gfr.data(), gs.data(), gf.data(), gfid) == DM_OK);
            EXPECT(ws == gs && wf == gf && wfr == gfr && std::memcmp(wfid, gfid, 32) == 0);
            // device form, stale bytes in the padding
            void *dobj = nullptr, *dpar = nullptr, *dh = nullptr;
            EXPECT(hipMalloc(&dobj, nseg * seg) == hipSuccess && hipMalloc(&dpar, nseg * 8 * frag) == hipSuccess &&
                   hipMalloc(&dh, 32 * nseg * 13 + 32) == hipSuccess);
            EXPECT(hipMemset(dobj, 0x5a, nseg * seg) == hipSuccess);
            EXPECT(hipMemcpy(dobj, obj.data(), len, hipMemcpyHostToDevice) == hipSuccess);
            uint8_t* h = static_cast<uint8_t*>(dh);
            EXPECT(dm_process_device_async(rs, dobj, len, seg, dpar, h, h + 32 * nseg, h + 32 * nseg * 13, nullptr) ==
                   DM_OK);
            EXPECT(hipDeviceSynchronize() == hipSuccess);
            std::vector<uint8_t> back(32 * nseg * 13 + 32);
            EXPECT(hipMemcpy(back.data(), dh, back.size(), hipMemcpyDeviceToHost) == hipSuccess);
            EXPECT(std::memcmp(back.data(), ws.data(), ws.size()) == 0);
            EXPECT(std::memcmp(back.data() + ws.size(), wf.data(), wf.size()) == 0);
            EXPECT(std::memcmp(back.data() + 32 * nseg * 13, wfid, 32) == 0);
            (void)hipFree(dobj);
            (void)hipFree(dpar);
            (void)hipFree(dh);
            // file form (dm_full_processing): digests, fid and every fragment / segment file;
            // small slots and windows (test hooks) so slot reuse and the multi-window fid run too
            const std::string src = tmpdir + "/fp_obj_" + std::to_string(len);
            const std::string out = tmpdir + "/fp_out_" + std::to_string(len);
            std::ofstream(src, std::ios::binary).write(reinterpret_cast<const char*>(obj.data()), (std::streamsize)len);
            for (int hooks = 0; hooks < 2; hooks++) {
                if (hooks) {
                    setenv("DEOSS_FP_SLOT_BYTES", "8192", 1);
                    setenv("DEOSS_FP_WINDOW_BYTES", "8192", 1);
                }
                std::vector<uint8_t> fs_(ws.size()), ff(wf.size());
                uint8_t ffid[32];
                uint64_t ns = 0;
                EXPECT(dm_full_processing(rs, src.c_str(), out.c_str(), seg, DM_FP_SEGMENT_FILES, fs_.data(), ff.data(),
                                          nseg, &ns, ffid) == DM_OK);
                EXPECT(ns == nseg && fs_ == ws && ff == wf && std::memcmp(ffid, wfid, 32) == 0);
                static const char* hx = "0123456789abcdef";
                for (uint64_t t = 0; t < nseg * 12; t++) {
                    std::string name;
                    for (int i = 0; i < 32; i++) {
                        name += hx[wf[32 * t + i] >> 4];
                        name += hx[wf[32 * t + i] & 15];
                    }
                    std::ifstream in(out + "/" + name, std::ios::binary);
                    std::vector<uint8_t> got((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
                    EXPECT(got.size() == frag && std::memcmp(got.data(), wfr.data() + t * frag, frag) == 0);
                }
                unsetenv("DEOSS_FP_SLOT_BYTES");
                unsetenv("DEOSS_FP_WINDOW_BYTES");
            }
            // streamed form (dm_pstream): random pieces, small slots and batches, then an aborted one
            for (int hooks = 0; hooks < 2; hooks++) {
                if (hooks) {
                    setenv("DEOSS_FP_SLOT_BYTES", "8192", 1);
                    setenv("DEOSS_PS_BATCH_CHUNKS", "2", 1);
                }
                dm_pstream* ps = nullptr;
                EXPECT(dm_pstream_open(rs, seg, (out + "_ps").c_str(), DM_FP_SEGMENT_FILES, &ps) == DM_OK);
                std::mt19937_64 rng(len * 7 + hooks);
                for (uint64_t pos = 0; pos < len;) {
                    const uint64_t m = std::min<uint64_t>(len - pos, 1 + rng() % 7000);
                    EXPECT(dm_pstream_write(ps, obj.data() + pos, m) == DM_OK);
                    pos += m;
                }
                std::vector<uint8_t> ps_s(ws.size()), ps_f(wf.size());
                uint8_t pfid[32];
                uint64_t pn = 0;
                EXPECT(dm_pstream_close(ps, ps_s.data(), ps_f.data(), nseg, &pn, pfid) == DM_OK);
                EXPECT(pn == nseg && ps_s == ws && ps_f == wf && std::memcmp(pfid, wfid, 32) == 0);
                EXPECT(dm_pstream_open(rs, seg, (out + "_ab").c_str(), 0, &ps) == DM_OK);
                EXPECT(dm_pstream_write(ps, obj.data(), len) == DM_OK);
                dm_pstream_abort(ps);
                unsetenv("DEOSS_FP_SLOT_BYTES");
                unsetenv("DEOSS_PS_BATCH_CHUNKS");
            }
            uint64_t ns = 0;
            EXPECT(dm_full_processing(rs, src.c_str(), out.c_str(), seg, 0, gs.data(), gf.data(), nseg - 1, &ns, gfid) ==
                       DM_ERR_INVALID && ns == nseg);   // digest arrays one segment short
            EXPECT(dm_full_processing(rs, (tmpdir + "/fp_missing").c_str(), out.c_str(), seg, 0, nullptr, nullptr, 0,
                                      nullptr, gfid) == DM_ERR_IO);
            EXPECT(std::string(dm_last_error(c)) == "open " + tmpdir + "/fp_missing: no such file or directory");
            std::remove(src.c_str());
        }
        uint8_t fid[32];
        EXPECT(dm_process_buffer(rs, nullptr, 0, seg, nullptr, nullptr, nullptr, fid) == DM_ERR_EMPTY);
        EXPECT(dm_process_buffer(rs, fid, 1, 100, nullptr, nullptr, nullptr, fid) == DM_ERR_INVALID);
        dm_rs_destroy(rs);
    }

    // batched FullProcessing and the coalescing executor (12 threads x 3 blocking requests)
    {
        dm_rs* rs = nullptr;
        EXPECT(dm_rs_create(c, 4, 8, &rs) == DM_OK);
        const uint64_t seg = 4096, frag = 1024;
        std::vector<std::vector<uint8_t>> objs;
        for (int i = 0; i < 9; i++) objs.push_back(bytes(1 + (uint64_t)i * 3001, 8800 + i));
        std::vector<const void*> op;
        std::vector<uint64_t> ol;
        std::vector<std::vector<uint8_t>> gs(9), gf(9);
        std::vector<uint8_t*> sp(9), fp(9);
        for (int i = 0; i < 9; i++) {
            op.push_back(objs[i].data());
            ol.push_back(objs[i].size());
            const uint64_t ns = (ol[i] + seg - 1) / seg;
            gs[i].resize(32 * ns);
            gf[i].resize(32 * ns * 12);
            sp[i] = gs[i].data();
            fp[i] = gf[i].data();
        }
        std::vector<uint8_t> fids(32 * 9);
        EXPECT(dm_process_batch(rs, op.data(), ol.data(), 9, seg, nullptr, sp.data(), fp.data(), fids.data()) == DM_OK);
        for (int i = 0; i < 9; i++) {
            const uint64_t ns = (ol[i] + seg - 1) / seg;
            std::vector<uint8_t> ws(32 * ns), wf(32 * ns * 12);
            uint8_t wfid[32];
            or_full_processing(op[i], ol[i], seg, 4, 8, ws.data(), wf.data(), wfid, nullptr, 1);
            EXPECT(ws == gs[i] && wf == gf[i] && std::memcmp(wfid, fids.data() + 32 * i, 32) == 0);
        }
        dm_rs_destroy(rs);

        dm_batcher* bp = nullptr;
        const int dev0[2] = {0, 0};   // the same GPU twice: slots of two "devices"
        EXPECT(dm_batcher_create(dev0, 2, DM_BATCH_PROCESS, seg, 4, 8, 1, 0, 0, 100, &bp) == DM_OK);
        dm_batcher* br = nullptr;
        EXPECT(dm_batcher_create(nullptr, 0, DM_BATCH_ROOT, 4096, 0, 0, 3, 64, 0, 0, &br) == DM_OK);
        std::vector<std::thread> ts;
        std::atomic<int> bad{0};
        for (int t = 0; t < 12; t++)
            ts.emplace_back([&, t] {
                for (int r = 0; r < 3; r++) {
                    auto o = bytes(1 + (uint64_t)(t * 7 + r) * 1777, 9900 + t * 3 + r);
                    uint8_t fid[32], wfid[32], root[32], wroot[32];
                    const uint64_t ns = (o.size() + seg - 1) / seg;
                    std::vector<uint8_t> fr(ns * 12 * frag), wfr(ns * 12 * frag), ws(32 * ns), wf(32 * ns * 12);
                    if (dm_batcher_process(bp, o.data(), o.size(), fr.data(), nullptr, nullptr, fid) != DM_OK) bad++;
                    or_full_processing(o.data(), o.size(), seg, 4, 8, ws.data(), wf.data(), wfid, wfr.data(), 1);
                    if (std::memcmp(fid, wfid, 32) != 0 || fr != wfr) bad++;
                    std::vector<uint8_t> lv(32 * ((o.size() + 4095) / 4096)), wl(lv.size());
                    if (dm_batcher_root(br, o.data(), o.size(), lv.data(), root) != DM_OK) bad++;
                    or_root_buffer(o.data(), o.size(), 4096, wl.data(), wroot, 1);
                    if (std::memcmp(root, wroot, 32) != 0 || lv != wl) bad++;
                }
            });
        for (auto& x : ts) x.join();
        EXPECT(bad.load() == 0);
        uint64_t nreq = 0, nb = 0, mx = 0;
        EXPECT(dm_batcher_stats(bp, &nreq, &nb, &mx) == DM_OK && nreq == 36 && nb >= 1 && nb <= 36);
        uint8_t tmp[32];
        EXPECT(dm_batcher_process(bp, nullptr, 0, nullptr, nullptr, nullptr, tmp) == DM_ERR_EMPTY);
        EXPECT(std::string(dm_batcher_last_error()) == "Empty data");
        EXPECT(dm_batcher_root(bp, tmp, 1, nullptr, tmp) == DM_ERR_INVALID);   // wrong mode
        dm_batcher_destroy(bp);
        dm_batcher_destroy(br);
    }

    // Merkle proofs: levels, paths, verification (host forms)
    {
        const uint64_t n = 1000;
        std::vector<std::vector<uint8_t>> ct;
        std::vector<uint8_t> lv(32 * n);
        for (uint64_t i = 0; i < n; i++) {
            ct.push_back(bytes(i % 300, 77 + i % 500));   // repeated contents
            or_sha256(ct.back().data(), ct.back().size(), lv.data() + 32 * i);
        }
        EXPECT(dm_tree_node_count(n) == 500 + 250 + 125 + 63 + 32 + 16 + 8 + 4 + 2 + 1);
        EXPECT(dm_tree_depth(n) == 10 && dm_tree_depth(1) == 1 && dm_tree_depth(2) == 1 && dm_tree_depth(3) == 2);
        std::vector<uint8_t> nodes(32 * dm_tree_node_count(n));
        EXPECT(dm_tree_levels(c, lv.data(), n, nodes.data()) == DM_OK);
        uint8_t want_root[32];
        or_reduce(lv.data(), n, -1, want_root);
        EXPECT(std::memcmp(nodes.data() + nodes.size() - 32, want_root, 32) == 0);
        std::vector<uint64_t> idx(n);
        for (uint64_t i = 0; i < n; i++) idx[i] = i;
        const uint32_t D = dm_tree_depth(n);
        std::vector<uint8_t> paths(32 * D * n), bits(D * n), ok(n);
        EXPECT(dm_merkle_paths(c, lv.data(), n, idx.data(), n, paths.data(), bits.data()) == DM_OK);
        std::vector<const void*> cp(n);
        std::vector<uint64_t> cl(n);
        for (uint64_t i = 0; i < n; i++) {
            cp[i] = ct[i].data();
            cl[i] = ct[i].size();
        }
        EXPECT(dm_verify_paths(c, cp.data(), cl.data(), n, paths.data(), bits.data(), D, want_root, 0, ok.data()) ==
               DM_OK);
        uint64_t good = 0;
        for (auto v : ok) good += v;
        EXPECT(good == n);
        paths[32 * D * 17 + 5] ^= 1;
        EXPECT(dm_verify_paths(c, cp.data(), cl.data(), n, paths.data(), bits.data(), D, want_root, 0, ok.data()) ==
               DM_OK);
        EXPECT(ok[17] == 0 && ok[16] == 1 && ok[18] == 1);
        EXPECT(dm_tree_levels(c, lv.data(), 0, nodes.data()) == DM_ERR_EMPTY);
        EXPECT(dm_verify_paths(c, cp.data(), cl.data(), n, paths.data(), bits.data(), D, want_root, 16, ok.data()) ==
               DM_ERR_INVALID);
    }

    // dm_last_error: the calling thread's last failure, never another thread's, never stale
    {
        EXPECT(dm_root_buffer(c, nullptr, 0, 64, nullptr, root) == DM_ERR_EMPTY);
        std::thread other([c] {
            uint8_t r[32];
            const char* gone[] = {"/nonexistent/other/thread"};
            EXPECT(dm_new_hash_tree(c, gone, 1, nullptr, r) == DM_ERR_IO);
            EXPECT(std::string(dm_last_error(c)).find("/nonexistent/other/thread") != std::string::npos);
        });
        other.join();
        EXPECT(std::string(dm_last_error(c)) == "Empty data");
        EXPECT(dm_root_buffer(c, root, 1, 0, nullptr, root) == DM_ERR_INVALID);
        EXPECT(std::string(dm_last_error(c)) == "invalid argument");
    }

    // NewHashTree from files: Go's error order and text, packed and striped layouts
    {
        const std::string d = tmpdir;
        const std::vector<std::vector<uint8_t>> two = {bytes(10, 1), bytes(20, 2)};
        auto paths = write_files(d, two, "err");
        std::string miss = d + "/missing_file_x";
        const char* order[] = {paths[0].c_str(), d.c_str(), miss.c_str(), paths[1].c_str()};
        EXPECT(dm_new_hash_tree(c, order, 4, nullptr, root) == DM_ERR_IO);   // the directory comes first
        EXPECT(std::string(dm_last_error(c)) == "read " + d + ": is a directory");
        const char* order2[] = {paths[0].c_str(), miss.c_str(), d.c_str()};
        EXPECT(dm_new_hash_tree(c, order2, 3, nullptr, root) == DM_ERR_IO);
        EXPECT(std::string(dm_last_error(c)) == "open " + miss + ": no such file or directory");
        for (auto& p : paths) std::remove(p.c_str());
        std::vector<std::vector<uint8_t>> small;
        for (int i = 0; i < 300; i++) small.push_back(bytes((uint64_t)(i * 7919) % 70000, 4000 + i));   // incl. 0 B
        check_files(c, d, small, "small");
        std::vector<std::vector<uint8_t>> segs;   // 12 near-equal 24 MiB files: 288 MiB, striped
        for (int i = 0; i < 12; i++) segs.push_back(bytes((24u << 20) - (i == 11 ? 12345 : 0), 6000 + i));
        check_files(c, d, segs, "seg");
        segs.resize(5);                          // 5 x 24 MiB: 120 MiB, packed through the pinned ring
        check_files(c, d, segs, "seg5_");
    }

    // ndev > 1 semantics on this box's one GPU (DEOSS_FORCE_SHARDED): block partition, RCCL
    // all-gather, leaf_out at odd and even n, an async call of the same context queued first
    {
        setenv("DEOSS_FORCE_SHARDED", "1", 1);
        dm_ctx* cs = nullptr;
        EXPECT(dm_create(&cs, nullptr, 0) == DM_OK);
        unsetenv("DEOSS_FORCE_SHARDED");
        if (cs) {
            for (auto [len, chunk] : {std::pair<uint64_t, uint64_t>{1000ull * 4096, 4096},       // n = 1000 (even)
                                      {1001ull * 4096 - 7, 4096},                                 // n = 1001 (odd)
                                      {(300ull << 20) + 5, 32ull << 20},                          // 10 striped leaves
                                      {3 * 64, 64}}) {
                auto b = bytes(len, len + 3);
                const uint64_t n = (len + chunk - 1) / chunk;
                // async root of another object on the null stream, enqueued before the sharded call
                auto other = bytes(5u << 20, 77);
                void* dev = nullptr;
                void* droot = nullptr;
                EXPECT(hipMalloc(&dev, other.size() + 64) == hipSuccess && hipMalloc(&droot, 32) == hipSuccess);
                EXPECT(hipMemcpy(dev, other.data(), other.size(), hipMemcpyHostToDevice) == hipSuccess);
                EXPECT(dm_root_device_async(cs, dev, other.size(), 1 << 16, droot, nullptr, nullptr) == DM_OK);
                std::vector<uint8_t> lw(32 * n), lg(32 * n);
                uint8_t rw[32], rg[32], ro[32], rd[32];
                EXPECT(or_root_buffer(b.data(), len, chunk, lw.data(), rw, 4) == 0);
                EXPECT(dm_root_buffer(cs, b.data(), len, chunk, lg.data(), rg) == DM_OK);
                EXPECT(std::memcmp(rw, rg, 32) == 0 && lw == lg);
                EXPECT(hipDeviceSynchronize() == hipSuccess);
                EXPECT(hipMemcpy(rd, droot, 32, hipMemcpyDeviceToHost) == hipSuccess);
                EXPECT(or_root_buffer(other.data(), other.size(), 1 << 16, nullptr, ro, 2) == 0);
                EXPECT(std::memcmp(ro, rd, 32) == 0);
                (void)hipFree(dev);
                (void)hipFree(droot);
            }
            std::vector<std::vector<uint8_t>> files;
            for (int i = 0; i < 37; i++) files.push_back(bytes(1000 + (uint64_t)i * 333, 7000 + i));
            check_files(cs, tmpdir, files, "shard");
            dm_destroy(cs);
        }
    }

    // the Go Stream call sequence: random pieces, an aborted body, concurrent uploads
    go_stream_sequence(c, (9u << 20) + 123, 1u << 20, 11, false);
    go_stream_sequence(c, (40u << 20) + 5, 32u << 20, 12, false);
    go_stream_sequence(c, 10u << 20, 1u << 16, 13, true);
    {
        std::vector<std::thread> ups;
        for (int t = 0; t < 6; t++)
            ups.emplace_back([c, t] { go_stream_sequence(c, 3000000 + 4097 * t, 65536, 50 + t, t == 3); });
        for (auto& x : ups) x.join();
    }

    // round 3: four context devices on this one GPU (DEOSS_VIRTUAL_DEVICES): per-device locks,
    // least-busy routing, pooled stream kits and the reaper under 8 threads mixing host buffers,
    // streams (some aborted) and batches, then sharded calls over the four devices (forced)
    {
        setenv("DEOSS_VIRTUAL_DEVICES", "4", 1);
        dm_ctx* cv = nullptr;
        EXPECT(dm_create(&cv, nullptr, 0) == DM_OK);
        setenv("DEOSS_FORCE_SHARDED", "1", 1);
        dm_ctx* cvs = nullptr;
        EXPECT(dm_create(&cvs, nullptr, 0) == DM_OK);
        unsetenv("DEOSS_FORCE_SHARDED");
        unsetenv("DEOSS_VIRTUAL_DEVICES");
        if (cv && cvs) {
            EXPECT(dm_device_count(cv) == 4);
            std::vector<std::thread> vt;
            for (int t = 0; t < 8; t++) vt.emplace_back([cv, t] { mixed_calls(cv, t); });
            for (auto& x : vt) x.join();
            for (auto [len, chunk] : {std::pair<uint64_t, uint64_t>{777ull * 4096 + 5, 4096}, {(100ull << 20) + 3, 8ull << 20}}) {
                auto b = bytes(len, len + 5);
                const uint64_t n = (len + chunk - 1) / chunk;
                std::vector<uint8_t> lw(32 * n), lg(32 * n);
                uint8_t rw[32], rg[32];
                EXPECT(or_root_buffer(b.data(), len, chunk, lw.data(), rw, 4) == 0);
                EXPECT(dm_root_buffer(cvs, b.data(), len, chunk, lg.data(), rg) == DM_OK);
                EXPECT(std::memcmp(rw, rg, 32) == 0 && lw == lg);
            }
        }
        dm_destroy(cv);
        dm_destroy(cvs);
    }

    // call lanes (dm_create_lanes): four lanes of this GPU, each with its own streams, scratch and
    // lock, under the same 8-thread mix; bad lane counts are rejected
    {
        dm_ctx* cl = nullptr;
        EXPECT(dm_create_lanes(&cl, nullptr, 0, 0) == DM_ERR_INVALID && cl == nullptr);
        EXPECT(dm_create_lanes(&cl, nullptr, 0, 9) == DM_ERR_INVALID && cl == nullptr);
        EXPECT(dm_create_lanes(&cl, nullptr, 0, 4) == DM_OK);
        if (cl) {
            EXPECT(dm_device_count(cl) == 1 && dm_lane_count(cl) == 4);
            std::vector<std::thread> lt;
            for (int t = 0; t < 8; t++) lt.emplace_back([cl, t] { mixed_calls(cl, t); });
            for (auto& x : lt) x.join();
        }
        dm_destroy(cl);
    }

    // concurrent callers on one context
    std::vector<std::thread> th;
    for (int t = 0; t < 4; t++) th.emplace_back([c, t] { check_buffer(c, 200000 + 1111 * t, 4096, 900 + t); });
    for (auto& x : th) x.join();

    dm_destroy(c);
    const int status = fails ? 1 : 0;
    if (fails) std::fprintf(stderr, "%d failures\n", fails.load());
    else std::printf("PASS\n");
    std::fflush(stdout);
    // ASan leg (run_host_tests.sh): every context is destroyed by now.  Exit without the runtime's
    // exit-time teardown: under ASan, device chunks freed during the run wait in ASan's quarantine,
    // and one recycled after the HSA runtime has unloaded trips ASan's own device-allocator CHECK
    // (sanitizer_allocator_device.h, "dev_runtime_unloaded_"), inside HSA's teardown, not ours.
    if (std::getenv("DEOSS_TEST_QUICK_EXIT")) std::_Exit(status);
    return status;
}
