// files_capi.inl -- dm_new_hash_tree: NewHashTree(chunkPath) (common/hashtree/types.go:19-39) from
// files, streamed: file bytes go from the page cache straight into pinned staging (parallel pread),
// H2D copies overlap the reads and the leaf kernel, and no whole-object copy is ever held in host
// memory (the reference reads every file whole with io.ReadAll and copies it again into a string,
// types.go:29,34).  Included by merkle_capi.hip (shares its helpers).
//
// Two layouts, chosen per device share of the files:
//  - packed: files laid out back to back in HBM (256-B aligned starts); the image is filled through
//    a ring of two pinned slots, one H2D per slot, then one table-mode leaf launch over all files.
//    Used when hashing is fast next to reading (many or small files: the wide kernel).
//  - striped: few long, near-equal files (DeOSS's 32 MiB segment files).  Every file advances W
//    bytes per step (W x nfiles <= 256 MiB): the reads of step j+1 overlap the H2D and the
//    resumable leaf launch of step j, so every leaf chain is in flight from the first stripe and the
//    call ends one stripe after the last read instead of one leaf-chain after it.
#include <fcntl.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

// Go's error text for an errno: strerror with a lower-case first letter ("no such file or directory").
std::string go_errno(int e) {
    std::string m = std::strerror(e);
    if (!m.empty()) m[0] = (char)std::tolower((unsigned char)m[0]);
    return m;
}

struct FileSet {
    std::vector<std::string> path;
    std::vector<uint64_t> size;
    std::vector<int> fd;                       // -1: closed, reopened by the reader
    std::vector<std::vector<uint8_t>> mem;     // non-regular files (pipes, devices): read whole at open
    ~FileSet() {
        for (int f : fd)
            if (f >= 0) ::close(f);
    }
};

// types.go:24-33: files are opened and read in order and the first failure is returned, with Go's
// messages: "open <path>: <errno text>", "read <path>: is a directory".
int open_files(dm_ctx* c, const char* const* paths, uint64_t n, FileSet& fs) {
    // Keep every file open when the descriptor limit allows (Go raises the soft limit to the hard
    // one at start-up; Python keeps 1,024): striped reads touch every file once per step, and
    // reopening 4,096 files per step would cost more than reading them.
    struct rlimit rl {};
    const uint64_t limit = getrlimit(RLIMIT_NOFILE, &rl) == 0 ? (uint64_t)rl.rlim_cur : 1024;
    const bool keep_open = n + 256 <= limit;
    fs.path.resize(n);
    fs.size.assign(n, 0);
    fs.fd.assign(n, -1);
    fs.mem.resize(n);
    for (uint64_t i = 0; i < n; i++) {
        if (!paths[i]) return fail(c, DM_ERR_INVALID, "path %llu is NULL", (unsigned long long)i);
        fs.path[i] = paths[i];
        const int fd = ::open(paths[i], O_RDONLY | O_CLOEXEC);
        if (fd < 0) return fail(c, DM_ERR_IO, "open %s: %s", paths[i], go_errno(errno).c_str());
        struct stat st {};
        if (::fstat(fd, &st) != 0) {
            const int e = errno;
            ::close(fd);
            return fail(c, DM_ERR_IO, "read %s: %s", paths[i], go_errno(e).c_str());
        }
        if (S_ISDIR(st.st_mode)) {
            ::close(fd);
            return fail(c, DM_ERR_IO, "read %s: is a directory", paths[i]);
        }
        if (!S_ISREG(st.st_mode)) {   // io.ReadAll semantics for streams: read to EOF now
            uint8_t tmp[1 << 16];
            for (;;) {
                const ssize_t r = ::read(fd, tmp, sizeof tmp);
                if (r == 0) break;
                if (r < 0) {
                    if (errno == EINTR) continue;
                    const int e = errno;
                    ::close(fd);
                    return fail(c, DM_ERR_IO, "read %s: %s", paths[i], go_errno(e).c_str());
                }
                fs.mem[i].insert(fs.mem[i].end(), tmp, tmp + r);
            }
            ::close(fd);
            fs.size[i] = fs.mem[i].size();
            continue;
        }
        fs.size[i] = (uint64_t)st.st_size;
        if (keep_open) fs.fd[i] = fd;
        else ::close(fd);
    }
    return DM_OK;
}

// One piece of one file: bytes [off, off + len) of file `file` into dst.
struct FilePart {
    uint64_t file, off, len;
    uint8_t* dst;
};

// Read one part (pread loop; a file shorter than its fstat size is an error: it changed under us).
bool read_part(const FileSet& fs, const FilePart& p, std::string* err) {
    if (!fs.mem[p.file].empty() || fs.size[p.file] == 0) {
        if (p.len) std::memcpy(p.dst, fs.mem[p.file].data() + p.off, p.len);
        return true;
    }
    int fd = fs.fd[p.file];
    const bool own = fd < 0;
    if (own && (fd = ::open(fs.path[p.file].c_str(), O_RDONLY | O_CLOEXEC)) < 0) {
        *err = "open " + fs.path[p.file] + ": " + go_errno(errno);
        return false;
    }
    uint64_t done = 0;
    bool ok = true;
    while (done < p.len) {
        const ssize_t r = ::pread(fd, p.dst + done, p.len - done, (off_t)(p.off + done));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
            *err = "read " + fs.path[p.file] + ": " + (r < 0 ? go_errno(errno) : std::string("unexpected EOF"));
            ok = false;
            break;
        }
        done += (uint64_t)r;
    }
    if (own) ::close(fd);
    return ok;
}

constexpr int kReaders = 4;   // pread threads per device (page-cache copies run ~5-10 GB/s each)

// Read every part, up to `readers` threads; on failure the lowest failing file wins (Go's order).
int read_parts(dm_ctx* c, const FileSet& fs, const std::vector<FilePart>& parts, int readers = kReaders) {
    if (parts.empty()) return DM_OK;
    uint64_t bytes = 0;
    for (const auto& p : parts) bytes += p.len;
    const int R = (int)std::min<uint64_t>((uint64_t)readers,
                                          std::max<uint64_t>(1, std::min<uint64_t>(parts.size(), bytes >> 22)));
    std::vector<uint64_t> bad(R, ~0ull);
    std::vector<std::string> msg(R);
    auto run = [&](int t) {
        for (size_t i = t; i < parts.size(); i += R) {
            if (parts[i].file >= bad[t]) continue;
            std::string e;
            if (!read_part(fs, parts[i], &e)) {
                bad[t] = parts[i].file;
                msg[t] = e;
            }
        }
    };
    if (R == 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 1; t < R; t++) th.emplace_back(run, t);
        run(0);
        for (auto& x : th) x.join();
    }
    int w = -1;
    for (int t = 0; t < R; t++)
        if (bad[t] != ~0ull && (w < 0 || bad[t] < bad[w])) w = t;
    return w < 0 ? DM_OK : fail(c, DM_ERR_IO, "%s", msg[w].c_str());
}

// Leaf digests of files [l0, l1) into d.leaves (stream-ordered on d.stream).
int files_leaves(dm_ctx* c, Dev& d, const FileSet& fs, uint64_t l0, uint64_t l1) {
    const uint64_t n = l1 - l0;
    uint64_t total = 0, maxlen = 0;
    for (uint64_t i = l0; i < l1; i++) {
        total += fs.size[i];
        maxlen = std::max(maxlen, fs.size[i]);
    }
    HIP_TRY(d.leaves.ensure(n * 32));
    const int kind = pick_leaf_kernel(c, d, n);
    const bool striped = kind != DM_LEAF_WIDE && total > kStripeBudget && n * maxlen <= 2 * total;
    hipStream_t s = d.stream;
    dm::LeafArgs la{};
    la.nleaves = n;
    la.digests = d.leaves.u8();
    la.byte_end = ~0ull;
    if (!striped) {
        // packed image, filled slot by slot: slot k holds image bytes [k*kStageBytes, (k+1)*kStageBytes)
        std::vector<uint64_t> off(n), addr(n), lens(n);
        uint64_t img = 0;
        for (uint64_t i = 0; i < n; i++) {
            off[i] = img;
            lens[i] = fs.size[l0 + i];
            img = round_up(img + lens[i], kAlign);
        }
        HIP_TRY(d.data.ensure(std::max<uint64_t>(img, kAlign)));
        for (uint64_t i = 0; i < n; i++) addr[i] = reinterpret_cast<uint64_t>(d.data.u8() + off[i]);
        HIP_TRY(d.stage[0].ensure(kStageBytes));
        HIP_TRY(d.stage[1].ensure(kStageBytes));
        bool busy[2] = {false, false};
        uint64_t f = 0;   // first file that may overlap the current slot
        for (uint64_t a = 0, slot = 0; a < img; a += kStageBytes, slot ^= 1) {
            const uint64_t b = std::min(img, a + kStageBytes);
            if (busy[slot]) HIP_TRY(hipEventSynchronize(d.ev_copy[slot]));
            std::vector<FilePart> parts;
            while (f < n && off[f] + lens[f] <= a) f++;
            for (uint64_t i = f; i < n && off[i] < b; i++) {
                const uint64_t s0 = std::max(a, off[i]), s1 = std::min(b, off[i] + lens[i]);
                if (s1 > s0) parts.push_back({l0 + i, s0 - off[i], s1 - s0, d.stage[slot].u8() + (s0 - a)});
            }
            RC_TRY(read_parts(c, fs, parts));
            HIP_TRY(hipMemcpyAsync(d.data.u8() + a, d.stage[slot].p, b - a, hipMemcpyHostToDevice, d.copy));
            HIP_TRY(hipEventRecord(d.ev_copy[slot], d.copy));
            busy[slot] = true;
        }
        HIP_TRY(hipEventRecord(d.ev_step[0], d.copy));
        HIP_TRY(hipStreamWaitEvent(s, d.ev_step[0], 0));
        RC_TRY(tables_begin(c, d, n * 16 + 1024));
        RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), n * 8));
        RC_TRY(upload(c, d, s, d.tab_len, lens.data(), n * 8));
        la.addrs = static_cast<const uint64_t*>(d.tab_addr.p);
        la.lens = static_cast<const uint64_t*>(d.tab_len.p);
        return launch_leaves(c, d, s, la, true, true, kind);
    }
    // striped: file i's bytes [j*W, (j+1)*W) arrive in step j.  Copy mode: row i of the HBM image
    // has pitch P.  Zero-copy mode (auto, latency regime: zero_copy_regime): K1Q reads each stripe
    // straight out of the pinned staging slot it was pread into, no H2D copy and no HBM image
    // (profiles/r02/LOGS.md (r02v_*.log)); a slot is refilled once the launch that read it has finished.
    const uint64_t W = std::max<uint64_t>(64, (kStripeBudget / n) / 64 * 64);
    std::vector<uint64_t> so, sw;   // ramped stripes (stripe_schedule)
    stripe_schedule(W, maxlen, so, sw);
    const uint64_t nsteps = so.size(), P = so.back() + sw.back();
    const bool zc = zero_copy_regime(c, d, n);
    HIP_TRY(d.nodes_b.ensure(n * 32));   // chaining state between stripes (8 words per leaf)
    HIP_TRY(d.stage[0].ensure(n * W));
    HIP_TRY(d.stage[1].ensure(n * W));
    std::vector<uint64_t> addr(zc ? 2 * n : nsteps * n), lens(n);
    for (uint64_t i = 0; i < n; i++) lens[i] = fs.size[l0 + i];
    if (zc) {   // staging slot k: row i (W bytes) holds leaf i's current stripe
        for (int k = 0; k < 2; k++) {
            void* dp = nullptr;
            HIP_TRY(hipHostGetDevicePointer(&dp, d.stage[k].p, 0));
            for (uint64_t i = 0; i < n; i++) addr[k * n + i] = reinterpret_cast<uint64_t>(dp) + i * W;
        }
    } else {    // HBM image, row pitch P; the kernel expects each leaf's pointer at its stripe's offset
        HIP_TRY(d.data.ensure(n * P));
        for (uint64_t jj = 0; jj < nsteps; jj++)
            for (uint64_t i = 0; i < n; i++) addr[jj * n + i] = reinterpret_cast<uint64_t>(d.data.u8() + i * P + so[jj]);
    }
    RC_TRY(tables_begin(c, d, (addr.size() + n) * 8 + 1024));
    RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), addr.size() * 8));
    RC_TRY(upload(c, d, s, d.tab_len, lens.data(), n * 8));
    bool busy[2] = {false, false};
    la.lens = static_cast<const uint64_t*>(d.tab_len.p);
    la.state = static_cast<uint32_t*>(d.nodes_b.p);
    for (uint64_t jj = 0, slot = 0; jj < nsteps; jj++, slot ^= 1) {
        hipEvent_t slot_free = zc ? d.ev_step[slot] : d.ev_copy[slot];
        if (busy[slot]) HIP_TRY(hipEventSynchronize(slot_free));
        uint8_t* st = d.stage[slot].u8();
        std::vector<FilePart> parts;
        for (uint64_t i = 0; i < n; i++)
            if (lens[i] > so[jj]) parts.push_back({l0 + i, so[jj], std::min(sw[jj], lens[i] - so[jj]), st + i * W});
        RC_TRY(read_parts(c, fs, parts));
        if (!zc) {
            HIP_TRY(hipMemcpy2DAsync(d.data.u8() + so[jj], P, st, W, sw[jj], n, hipMemcpyHostToDevice, d.copy));
            HIP_TRY(hipEventRecord(d.ev_copy[slot], d.copy));
            HIP_TRY(hipStreamWaitEvent(s, d.ev_copy[slot], 0));
        }
        la.addrs = static_cast<const uint64_t*>(d.tab_addr.p) + (zc ? slot : jj) * n;
        la.byte_off = so[jj];
        la.byte_end = so[jj] + sw[jj];
        RC_TRY(launch_leaves(c, d, s, la, true, true, zc ? DM_LEAF_QUAD : kind));
        if (zc) HIP_TRY(hipEventRecord(d.ev_step[slot], s));
        busy[slot] = true;
    }
    return DM_OK;
}

}  // namespace

extern "C" {

int dm_new_hash_tree(dm_ctx* ctx, const char* const* paths, uint64_t n, uint8_t* leaf_out, uint8_t root[32]) {
    if (!ctx || !root || (n && !paths)) return bad_arg();
    DeviceRestore dr;
    dm_ctx* c = ctx;
    if (n == 0) return fail(c, DM_ERR_EMPTY, "Empty data");   // types.go:20-22
    FileSet fs;
    RC_TRY(open_files(c, paths, n, fs));
    uint64_t bytes = 0, maxlen = 0;
    for (uint64_t i = 0; i < n; i++) {
        bytes += fs.size[i];
        maxlen = std::max(maxlen, fs.size[i]);
    }
    // 256 x 32 MiB segment files: one device (every chain resident; sharding only occupies more
    // GPUs), so concurrent calls land on different devices
    const int G = route_call(c, n, bytes, maxlen, DM_SRC_FILES);
    if (sharded(c, G, n)) {
        RangeLock lk(c, G);
        auto produce = [&](dm_ctx* cc, Dev& d, uint64_t l0, uint64_t l1) -> int {
            return files_leaves(cc, d, fs, l0, l1);
        };
        return multi_root(c, G, n, produce, leaf_out, root);
    }
    const int g = pick_device(c);
    CallLock lk(c, g, kReserved);
    Dev& d = c->devs[g];
    RC_TRY(begin_call(c, d, d.stream));
    RC_TRY(files_leaves(c, d, fs, 0, n));
    return reduce_leaves_to_host(c, d, n, leaf_out, root);
}

}  // extern "C"
