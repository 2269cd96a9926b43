// fullproc_capi.inl -- dm_full_processing: cess-go-sdk process.FullProcessing(file, "", savedir)
// (go.mod:8; called at node/objectHandler.go:168, node/fileHandler.go:771,
// node/filesHandler.go:201, node/resumeHandler.go:326, node/tracker.go:767-769) from the file path,
// in one call.  Part of merkle_capi.hip (after files_capi.inl, rs_capi.inl, process_capi.inl).
//
// Per window of segments (up to kFpWindowBytes of file; one window up to 32 GiB):
//   A. the file is pread into pinned slots (whole segments per slot, parallel readers) and each
//      slot is copied to HBM -- nothing else, so the leaf chains can start as soon as the reads
//      allow (the last segment's zero padding is filled in the slot);
//   B. one RS launch and one leaf launch over the window's segments and fragments
//      (process_segments, the same GPU pass as dm_process_buffer);
//   C. while the leaf kernel's serial chains run (~0.5 s for 32 MiB segments), the data fragments
//      and segment files -- plain file bytes -- are copied from the file by background writers
//      (copy_file_range, page cache to page cache), and the parity fragments come back through
//      the slots and are written to temporary files;
//   D. the digests come back and every temporary file is renamed to savedir/<hex SHA-256>.
// The fid is the hashtree root over all segment digests.  The Go shim's window path (read a
// window, one batched GPU call, then write its fragments) leaves the GPU idle during the writes
// and the writes idle during the hashing; here they overlap.

namespace {

constexpr uint64_t kFpSlotBytes = 64ull << 20;         // pinned slot (whole segments / parity sets)
constexpr int kFpSlots = 4;                             // = dm_rs::fp_slot
constexpr int kFpWritersPerSlot = 4;                    // background write jobs per parity slot
constexpr size_t kFpDataWriters = 8;                    // jobs copying data fragments / segments from the file
constexpr int kFpReaders = 8;                           // pread threads per slot (phase A gates the leaf pass)

struct FdGuard {
    int fd = -1;
    ~FdGuard() {
        if (fd >= 0) ::close(fd);
    }
};
constexpr uint64_t kFpWindowBytes = 32ull << 30;        // file bytes per GPU pass (+ 2x parity in HBM)
constexpr uint64_t kFpStripeMinSegs = 4;                // windows of at least this many segments read in stripes

std::atomic<uint64_t> g_fp_seq{0};

// DEOSS_FP_TRACE=1: phase times of each dm_full_processing window on stderr (diagnostics)
struct FpTrace {
    bool on = std::getenv("DEOSS_FP_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void mark(const char* what) const {
        if (on)
            std::fprintf(stderr, "[fp] %-28s %8.1f ms\n", what,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

uint64_t env_bytes(const char* name, uint64_t dflt) {
    const char* v = std::getenv(name);
    const unsigned long long x = v ? std::strtoull(v, nullptr, 10) : 0;
    return x ? (uint64_t)x : dflt;
}

std::string hex32(const uint8_t* d) {
    static const char* x = "0123456789abcdef";
    std::string s(64, '0');
    for (int i = 0; i < 32; i++) {
        s[2 * i] = x[d[i] >> 4];
        s[2 * i + 1] = x[d[i] & 15];
    }
    return s;
}

// os.WriteFile(path, data, os.ModePerm), as the Go shim writes fragments; "" on success.
std::string write_whole(const std::string& path, const uint8_t* p, uint64_t len) {
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0777);
    if (fd < 0) return "open " + path + ": " + go_errno(errno);
    uint64_t done = 0;
    while (done < len) {
        const ssize_t w = ::write(fd, p + done, len - done);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) {
            const int e = w < 0 ? errno : EIO;
            ::close(fd);
            return "write " + path + ": " + go_errno(e);
        }
        done += (uint64_t)w;
    }
    if (::close(fd) != 0) return "close " + path + ": " + go_errno(errno);
    return "";
}

// os.MkdirAll(dir, 0755)
std::string mkdir_all(const std::string& dir) {
    for (size_t i = 1; i <= dir.size(); i++) {
        if (i < dir.size() && dir[i] != '/') continue;
        const std::string p = dir.substr(0, i);
        struct stat st {};
        if (::stat(p.c_str(), &st) == 0) {
            if (!S_ISDIR(st.st_mode)) return "mkdir " + p + ": not a directory";
            continue;
        }
        if (::mkdir(p.c_str(), 0755) != 0 && errno != EEXIST) return "mkdir " + p + ": " + go_errno(errno);
    }
    return "";
}

struct FpFile {          // one file to write: its bytes (memory, or a range of an open file) and temporary name
    const uint8_t* src;
    uint64_t len;
    std::string tmp;
    int in_fd = -1;         // >= 0: the bytes are [in_off, in_off + len) of this file (copied in the kernel)
    uint64_t in_off = 0;
};

// A file range into a new file: copy_file_range (page cache to page cache in the kernel, no user
// copy), or pread / write through a bounce buffer where the kernel cannot.
std::string copy_whole(const std::string& path, int in_fd, uint64_t off, uint64_t len) {
    const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0777);
    if (fd < 0) return "open " + path + ": " + go_errno(errno);
    uint64_t done = 0;
    bool kernel = true;
    std::vector<uint8_t> bounce;
    while (done < len) {
        if (kernel) {
            loff_t io = (loff_t)(off + done);
            const ssize_t w = ::copy_file_range(in_fd, &io, fd, nullptr, len - done, 0);
            if (w > 0) {
                done += (uint64_t)w;
                continue;
            }
            if (w < 0 && errno == EINTR) continue;
            if (w < 0 && errno != EXDEV && errno != ENOSYS && errno != EINVAL && errno != EOPNOTSUPP) {
                const int e = errno;
                ::close(fd);
                return "write " + path + ": " + go_errno(e);
            }
            kernel = false;   // 0 (short source) or unsupported: finish through user space
            bounce.resize(8ull << 20);
        }
        const uint64_t n = std::min<uint64_t>(bounce.size(), len - done);
        const ssize_t r = ::pread(in_fd, bounce.data(), n, (off_t)(off + done));
        if (r <= 0) {
            ::close(fd);
            return "read: " + (r < 0 ? go_errno(errno) : std::string("unexpected EOF"));
        }
        for (ssize_t put = 0; put < r;) {
            const ssize_t w = ::write(fd, bounce.data() + put, (size_t)(r - put));
            if (w < 0 && errno == EINTR) continue;
            if (w <= 0) {
                const int e = w < 0 ? errno : EIO;
                ::close(fd);
                return "write " + path + ": " + go_errno(e);
            }
            put += w;
        }
        done += (uint64_t)r;
    }
    if (::close(fd) != 0) return "close " + path + ": " + go_errno(errno);
    return "";
}

// Background writes out of one pinned slot; wait() joins them before the slot is refilled.
struct SlotWrites {
    std::vector<std::future<std::string>> jobs;
    void start(std::vector<FpFile> files, size_t jobs_max = kFpWritersPerSlot) {
        const size_t J = std::min<size_t>(jobs_max, files.size());
        for (size_t j = 0; j < J; j++) {
            std::vector<FpFile> mine;
            for (size_t i = j; i < files.size(); i += J) mine.push_back(files[i]);
            jobs.push_back(std::async(std::launch::async, [mine]() {
                for (const auto& f : mine) {
                    std::string e = f.in_fd >= 0 ? copy_whole(f.tmp, f.in_fd, f.in_off, f.len)
                                                 : write_whole(f.tmp, f.src, f.len);
                    if (!e.empty()) return e;
                }
                return std::string();
            }));
        }
    }
    std::string wait() {   // first error, once every job has finished
        std::string err;
        for (auto& j : jobs) {
            std::string e = j.get();
            if (err.empty()) err = e;
        }
        jobs.clear();
        return err;
    }
    ~SlotWrites() { (void)wait(); }
};

constexpr uint64_t kFpKeepBytes = 4ull << 30;   // window scratch kept between dm_full_processing calls

struct FpEvents {
    hipEvent_t slot[kFpSlots] = {}, rs = nullptr, copied = nullptr;
    ~FpEvents() {
        for (hipEvent_t e : slot)
            if (e) (void)hipEventDestroy(e);
        if (rs) (void)hipEventDestroy(rs);
        if (copied) (void)hipEventDestroy(copied);
    }
};

// Striped pass over one window of ns segments (file bytes [fbeg, fend)): for every stripe [o, o + w)
// of the segment (stripe_schedule, split at fragment boundaries) the window's ns pieces are pread
// into one pinned slot, copied to HBM with one 2D copy (segment pitch), and two resumable leaf
// launches absorb them: the ns segment chains (kit->comp[0]) and the ns chains of the data fragment
// the stripe lies in (kit->comp[1]).  After the last stripe: RS over the window and one leaf launch
// over the parity fragments (on s), then the fid over the segment digests.  d.leaves: segment t at
// t, data fragment (t, q) at ns * (1 + q) + t, parity fragment (t, i) at ns * (1 + k) + t * m + i.
template <class TakeSlot>
int fp_striped_pass(dm_rs* r, Dev& d, hipStream_t s, StreamKit* kit, const FileSet& fs, uint64_t fbeg, uint64_t fend,
                    uint64_t ns, uint64_t seg, uint64_t slot_cap, int readers, TakeSlot& take_slot,
                    bool (&busy)[kFpSlots], FpEvents& ev, uint8_t* parity, uint8_t* dfid, FpTrace& tr) {
    dm_ctx* c = r->c;
    const int k = r->k, m = r->m;
    const uint64_t frag = seg / (uint64_t)k;
    const uint64_t W = std::max<uint64_t>(64, (slot_cap / ns) / 64 * 64);   // slot row pitch
    std::vector<uint64_t> so0, sw0, so, sw;
    stripe_schedule(W, seg, so0, sw0);
    for (size_t j = 0; j < so0.size(); j++)   // no stripe crosses a fragment boundary
        for (uint64_t o = so0[j], e = std::min(seg, so0[j] + sw0[j]); o < e;) {
            const uint64_t b = std::min(e, (o / frag + 1) * frag);
            so.push_back(o);
            sw.push_back(b - o);
            o = b;
        }
    const uint64_t nsteps = so.size();
    uint32_t* seg_state = reinterpret_cast<uint32_t*>(dfid + 256);
    uint32_t* frag_state = seg_state + 8 * ns;
    // tables: row j = the ns segment pointers at stripe j's offset; lens = ns segments, ns fragments;
    // the parity launch: ns x m fragment pointers and lengths
    std::vector<uint64_t> addr(nsteps * ns), lens(2 * ns, seg), paddr(ns * m), plen(ns * m, frag);
    for (uint64_t t = 0; t < ns; t++) lens[ns + t] = frag;
    for (uint64_t j = 0; j < nsteps; j++)
        for (uint64_t t = 0; t < ns; t++) addr[j * ns + t] = reinterpret_cast<uint64_t>(d.data.u8() + t * seg + so[j]);
    for (uint64_t i = 0; i < ns * m; i++) paddr[i] = reinterpret_cast<uint64_t>(parity + i * frag);
    RC_TRY(tables_begin(c, d, (addr.size() + lens.size() + 2 * ns * m) * 8 + 4096));
    HIP_TRY(d.leaves.ensure(32 * ns * (1 + (uint64_t)(k + m))));
    RC_TRY(upload(c, d, s, d.tab_addr, addr.data(), addr.size() * 8));
    RC_TRY(upload(c, d, s, d.tab_len, lens.data(), lens.size() * 8));
    RC_TRY(upload(c, d, s, d.tab_first, paddr.data(), paddr.size() * 8));
    RC_TRY(upload(c, d, s, d.tab_ids, plen.data(), plen.size() * 8));
    HIP_TRY(hipEventRecord(ev.copied, s));   // the tables are on the device before any launch
    for (hipStream_t x : {kit->comp[0], kit->comp[1]}) HIP_TRY(hipStreamWaitEvent(x, ev.copied, 0));
    const int kind = pick_leaf_kernel(c, d, ns);
    for (uint64_t j = 0; j < nsteps; j++) {
        const uint64_t o = so[j], w = sw[j], q = o / frag;
        int sl;
        RC_TRY(take_slot(&sl));
        uint8_t* buf = rs_ln(r, d).fp_slot[sl].u8();
        std::vector<FilePart> parts;
        for (uint64_t t = 0; t < ns; t++) {
            const uint64_t a = fbeg + t * seg + o;
            const uint64_t have = a < fend ? std::min(w, fend - a) : 0;
            if (have) parts.push_back({0, a, have, buf + t * W});
            if (have < w) std::memset(buf + t * W + have, 0, w - have);   // the last segment's zero padding
        }
        RC_TRY(read_parts(c, fs, parts, readers));
        HIP_TRY(hipMemcpy2DAsync(d.data.u8() + o, seg, buf, W, w, ns, hipMemcpyHostToDevice, d.copy));
        HIP_TRY(hipEventRecord(ev.slot[sl], d.copy));
        busy[sl] = true;
        dm::LeafArgs la{};
        la.addrs = static_cast<const uint64_t*>(d.tab_addr.p) + j * ns;
        la.nleaves = ns;
        la.byte_off = o;
        la.byte_end = o + w;
        la.state = seg_state;
        la.lens = static_cast<const uint64_t*>(d.tab_len.p);
        la.digests = d.leaves.u8();
        HIP_TRY(hipStreamWaitEvent(kit->comp[0], ev.slot[sl], 0));
        RC_TRY(launch_leaves(c, d, kit->comp[0], la, true, true, kind));
        la.byte_off = o - q * frag;
        la.byte_end = la.byte_off + w;
        la.state = frag_state;   // re-initialised where each fragment starts (byte_off 0)
        la.lens = static_cast<const uint64_t*>(d.tab_len.p) + ns;
        la.digests = d.leaves.u8() + 32 * ns * (1 + q);
        HIP_TRY(hipStreamWaitEvent(kit->comp[1], ev.slot[sl], 0));
        RC_TRY(launch_leaves(c, d, kit->comp[1], la, true, true, kind));
    }
    tr.mark("A': stripes read, launched");
    // RS after the last copy, then the parity fragments' chains (8 MiB: shorter than the segments')
    HIP_TRY(hipEventRecord(ev.copied, d.copy));
    HIP_TRY(hipStreamWaitEvent(s, ev.copied, 0));
    dm::RsArgs a{};
    for (int j = 0; j < k; j++) a.in[j] = d.data.u8() + (uint64_t)j * frag;
    for (int i = 0; i < m; i++) a.out[i] = parity + (uint64_t)i * frag;
    a.in_seg_stride = seg;
    a.out_seg_stride = (uint64_t)m * frag;
    a.units_per_seg = frag / 16;
    a.nseg = ns;
    a.table = static_cast<const uint2*>(r->enc_tab.p);
    a.nout = (uint32_t)m;
    launch_rs(d, s, k, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev.rs, s));
    dm::LeafArgs pa{};
    pa.addrs = static_cast<const uint64_t*>(d.tab_first.p);
    pa.lens = static_cast<const uint64_t*>(d.tab_ids.p);
    pa.nleaves = ns * m;
    pa.byte_end = ~0ull;
    pa.digests = d.leaves.u8() + 32 * ns * (1 + (uint64_t)k);
    RC_TRY(launch_leaves(c, d, s, pa, true, true, pick_leaf_kernel(c, d, ns * m)));
    // the fid once the segment chains are done
    HIP_TRY(hipEventRecord(kit->ev[0], kit->comp[0]));
    HIP_TRY(hipEventRecord(kit->ev[1], kit->comp[1]));
    HIP_TRY(hipStreamWaitEvent(s, kit->ev[0], 0));
    HIP_TRY(hipStreamWaitEvent(s, kit->ev[1], 0));
    RC_TRY(finish(c, d, s, d.leaves.u8(), ns, true, dfid));
    return DM_OK;
}

// Everything but the renames; `pend` collects (temporary name, digest slot) of every file written.
int full_processing_windows(dm_rs* r, Dev& d, const FileSet& fs, const std::string& dir, uint64_t seg, int flags,
                            std::vector<uint8_t>& segd, std::vector<uint8_t>& fragd,
                            std::vector<std::pair<std::string, uint64_t>>& pend, uint8_t fid[32]) {
    dm_ctx* c = r->c;
    const int g = (int)(&d - c->devs.data());   // the call's lane
    RsLane& L = rs_ln(r, d);
    hipStream_t s = d.stream;
    const int k = r->k, m = r->m, total = k + m;
    const uint64_t frag = seg / (uint64_t)k, pbytes = (uint64_t)m * frag;   // parity bytes per segment
    const uint64_t size = fs.size[0], nseg = ceil_div(size, seg);
    // test hooks (env, read per call): smaller slots / windows exercise slot reuse and multi-window fids
    const uint64_t slot_bytes = env_bytes("DEOSS_FP_SLOT_BYTES", kFpSlotBytes);
    const uint64_t window_bytes = env_bytes("DEOSS_FP_WINDOW_BYTES", kFpWindowBytes);
    const uint64_t spd = std::max<uint64_t>(1, slot_bytes / seg);            // segments per data slot
    const uint64_t spp = std::max<uint64_t>(1, slot_bytes / pbytes);         // segments per parity slot
    const uint64_t slot_cap = std::max(spd * seg, spp * pbytes);
    const uint64_t win = std::max<uint64_t>(spd, window_bytes / seg / spd * spd);   // segments per window
    const int readers = (int)std::min<uint64_t>(64, env_bytes("DEOSS_FP_READERS", kFpReaders));
    RC_TRY(begin_call(c, d, s));
    for (auto& b : L.fp_slot) HIP_TRY(b.ensure(slot_cap));
    FpEvents ev;
    for (auto& e : ev.slot) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ev.rs, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ev.copied, hipEventDisableTiming));
    const std::string base = dir + "/.dm-fp-" + std::to_string((long long)::getpid()) + "-" +
                             std::to_string((unsigned long long)g_fp_seq++) + "-";
    // where data files are copied from: the open file (kernel copies) or, for a pipe, its bytes
    const uint8_t* mem = fs.mem[0].empty() ? nullptr : fs.mem[0].data();
    int in_fd = fs.fd[0];
    FdGuard own_fd;
    if (!mem && in_fd < 0) {
        in_fd = own_fd.fd = ::open(fs.path[0].c_str(), O_RDONLY | O_CLOEXEC);
        if (in_fd < 0) return fail(c, DM_ERR_IO, "open %s: %s", fs.path[0].c_str(), go_errno(errno).c_str());
    }
    std::vector<uint8_t> tail;      // the zero-padded last segment (its data files are written from here)
    uint64_t tail_seg = ~0ull;
    SlotWrites wd;                  // data-fragment / segment-file writers (declared after their sources)
    SlotWrites wr[kFpSlots];
    bool busy[kFpSlots] = {false, false, false, false};
    uint64_t next = 0;   // slot round robin across both phases and windows
    auto take_slot = [&](int* out) -> int {
        const int sl = (int)(next++ % kFpSlots);
        if (busy[sl]) {
            HIP_TRY(hipEventSynchronize(ev.slot[sl]));
            const std::string e = wr[sl].wait();
            if (!e.empty()) return fail(c, DM_ERR_IO, "%s", e.c_str());
            busy[sl] = false;
        }
        *out = sl;
        return DM_OK;
    };
    // The window's data fragments and segment files -- plain file bytes -- are copied from the
    // file itself by background jobs (copy_file_range: page cache to page cache); the zero-padded
    // last segment's from `tail`.
    auto start_data_files = [&](uint64_t w0, uint64_t ns) {
        std::vector<FpFile> files;
        for (uint64_t gs = w0; gs < w0 + ns; gs++) {
            const bool padded = gs == tail_seg;
            auto add = [&](uint64_t off_in_seg, uint64_t len, const std::string& tmp) {
                if (padded) files.push_back({tail.data() + off_in_seg, len, tmp});
                else if (mem) files.push_back({mem + gs * seg + off_in_seg, len, tmp});
                else files.push_back({nullptr, len, tmp, in_fd, gs * seg + off_in_seg});
            };
            for (int j = 0; j < k; j++) {
                const uint64_t id = gs * (uint64_t)total + (uint64_t)j;
                add((uint64_t)j * frag, frag, base + "f" + std::to_string(id));
                pend.emplace_back(files.back().tmp, 32 * id);
            }
            if (flags & DM_FP_SEGMENT_FILES) {
                add(0, seg, base + "s" + std::to_string(gs));
                pend.emplace_back(files.back().tmp, ~(32 * gs));   // ~: a segment digest
            }
        }
        wd.start(std::move(files), (size_t)env_bytes("DEOSS_FP_DATA_WRITERS", kFpDataWriters));
    };
    const bool one_window = nseg <= win;
    const char* stripes_env = std::getenv("DEOSS_FP_STRIPES");
    const bool stripes_off = stripes_env != nullptr && stripes_env[0] == '0';
    // two extra compute streams for the striped pass (segment and data-fragment chains side by side)
    StreamKit* kit = nullptr;
    RC_TRY(kit_acquire(c, g, &kit));
    struct KitBack {
        dm_ctx* c;
        int g;
        StreamKit* k;
        ~KitBack() {
            for (hipStream_t x : {k->comp[0], k->comp[1]}) (void)hipStreamSynchronize(x);
            kit_release(c, g, k);
        }
    } kit_back{c, g, kit};
    FpTrace tr;
    for (uint64_t w0 = 0; w0 < nseg; w0 += win) {
        const uint64_t ns = std::min(win, nseg - w0);
        const uint64_t fbeg = w0 * seg, fend = std::min(size, (w0 + ns) * seg);
        // striped (round 3): the window is read in stripes [o, o + w) of EVERY segment, so the segment
        // and data-fragment chains start with the first stripe instead of after the whole window
        // (the reads of an 8 GiB file took 236 ms before any chain started); needs whole 64-B blocks
        // per fragment.  DEOSS_FP_STRIPES=0 keeps the read-then-launch order (A/B).
        const bool striped = ns >= kFpStripeMinSegs && frag % 64 == 0 && !stripes_off;
        HIP_TRY(d.data.ensure(ns * seg + kAlign));
        HIP_TRY(L.work.ensure(ns * pbytes + 256 + 2 * ns * 32));
        uint8_t* parity = L.work.u8();
        uint8_t* dfid = parity + ns * pbytes;
        if (!striped) {
            // A: file -> slots -> HBM, nothing else, so the leaf chains start as early as the reads allow
            for (uint64_t t0 = 0; t0 < ns; t0 += spd) {
                const uint64_t nt = std::min(spd, ns - t0), len = nt * seg, a = fbeg + t0 * seg;
                int sl;
                RC_TRY(take_slot(&sl));
                uint8_t* buf = L.fp_slot[sl].u8();
                const uint64_t have = a < fend ? std::min(len, fend - a) : 0;
                std::vector<FilePart> parts;
                for (uint64_t q = 0; q < have; q += 8ull << 20)
                    parts.push_back({0, a + q, std::min<uint64_t>(8ull << 20, have - q), buf + q});
                RC_TRY(read_parts(c, fs, parts, readers));
                if (have < len) std::memset(buf + have, 0, len - have);
                HIP_TRY(hipMemcpyAsync(d.data.u8() + t0 * seg, buf, len, hipMemcpyHostToDevice, d.copy));
                HIP_TRY(hipEventRecord(ev.slot[sl], d.copy));
                busy[sl] = true;
                if (t0 + nt == ns && have < len) {   // the file's last, zero-padded segment: keep a copy
                    tail.assign(buf + (nt - 1) * seg, buf + nt * seg);
                    tail_seg = w0 + t0 + nt - 1;
                }
            }
            tr.mark("A: reads + H2D enqueued");
            // B: RS + one leaf launch over segments and fragments, after the last H2D
            HIP_TRY(hipEventRecord(ev.copied, d.copy));
            HIP_TRY(hipStreamWaitEvent(s, ev.copied, 0));
            RC_TRY(process_segments(r, d, s, d.data.u8(), seg, parity, {0, ns}, dfid, ev.rs));
        } else {
            if (fend - fbeg < ns * seg) {   // the file's last, zero-padded segment, for its data files
                tail.assign(seg, 0);
                const uint64_t a = fbeg + (ns - 1) * seg;
                RC_TRY(read_parts(c, fs, {{0, a, fend - a, tail.data()}}, readers));
                tail_seg = w0 + ns - 1;
            }
            // the data files need only the file: their copies run from the start, beside the reads
            start_data_files(w0, ns);
            RC_TRY(fp_striped_pass(r, d, s, kit, fs, fbeg, fend, ns, seg, slot_cap, readers, take_slot, busy, ev,
                                   parity, dfid, tr));
        }
        // C: while the leaf chains run, the parity comes back through the slots and is written as
        // each set lands (the data fragments and segment files are already being copied)
        if (!striped) start_data_files(w0, ns);
        HIP_TRY(hipStreamWaitEvent(d.copy, ev.rs, 0));
        tr.mark("B: launched, data copies started");
        for (uint64_t t0 = 0; t0 < ns; t0 += spp) {
            const uint64_t nt = std::min(spp, ns - t0);
            int sl;
            RC_TRY(take_slot(&sl));
            uint8_t* buf = L.fp_slot[sl].u8();
            HIP_TRY(hipMemcpyAsync(buf, parity + t0 * pbytes, nt * pbytes, hipMemcpyDeviceToHost, d.copy));
            HIP_TRY(hipEventRecord(ev.slot[sl], d.copy));
            HIP_TRY(hipEventSynchronize(ev.slot[sl]));
            std::vector<FpFile> files;
            for (uint64_t u = 0; u < nt; u++) {
                const uint64_t gs = w0 + t0 + u;
                for (int i = 0; i < m; i++) {
                    const uint64_t id = gs * (uint64_t)total + (uint64_t)(k + i);
                    files.push_back({buf + u * pbytes + (uint64_t)i * frag, frag, base + "f" + std::to_string(id)});
                    pend.emplace_back(files.back().tmp, 32 * id);
                }
            }
            wr[sl].start(std::move(files));
            busy[sl] = true;
        }
        tr.mark("C: parity back, writes queued");
        // D: digests.  One pass: d.leaves holds segment t at t, fragment (t, j) at ns + t * total + j.
        // Striped: segment t at t, data fragment (t, q) at ns * (1 + q) + t, parity fragment (t, i)
        // at ns * (1 + k) + t * m + i (interleaved here)
        std::vector<uint8_t> lv;
        if (striped) {
            lv.resize(32 * ns * (1 + (uint64_t)total));
            HIP_TRY(hipMemcpyAsync(lv.data(), d.leaves.p, lv.size(), hipMemcpyDeviceToHost, s));
        } else {
            HIP_TRY(hipMemcpyAsync(segd.data() + 32 * w0, d.leaves.p, 32 * ns, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(fragd.data() + 32 * w0 * total, d.leaves.u8() + 32 * ns, 32 * ns * total,
                                   hipMemcpyDeviceToHost, s));
        }
        if (one_window) HIP_TRY(hipMemcpyAsync(fid, dfid, 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (striped) {
            std::memcpy(segd.data() + 32 * w0, lv.data(), 32 * ns);
            for (uint64_t t = 0; t < ns; t++)
                for (int j = 0; j < total; j++) {
                    const uint64_t from = j < k ? ns * (1 + (uint64_t)j) + t : ns * (1 + (uint64_t)k) + t * m + (j - k);
                    std::memcpy(fragd.data() + 32 * ((w0 + t) * total + j), lv.data() + 32 * from, 32);
                }
        }
        HIP_TRY(hipStreamSynchronize(d.copy));   // this window's slots are in host memory: HBM reusable
        tr.mark("D: leaf pass done");
        const std::string e = wd.wait();
        tr.mark("data files written");   // the window's data files, before the next window reuses `tail`
        if (!e.empty()) return fail(c, DM_ERR_IO, "%s", e.c_str());
    }
    for (int sl = 0; sl < kFpSlots; sl++) {
        const std::string e = wr[sl].wait();
        if (!e.empty()) return fail(c, DM_ERR_IO, "%s", e.c_str());
    }
    tr.mark("parity files written");
    if (!one_window) {   // several windows: the fid is the tree over every segment digest
        HIP_TRY(d.leaves.ensure(32 * nseg));
        HIP_TRY(hipMemcpyAsync(d.leaves.p, segd.data(), 32 * nseg, hipMemcpyHostToDevice, s));
        RC_TRY(finish(c, d, s, d.leaves.u8(), nseg, true, d.root.u8()));
        HIP_TRY(hipMemcpyAsync(fid, d.root.p, 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return DM_OK;
}

}  // namespace

extern "C" {

int dm_full_processing(dm_rs* r, const char* path, const char* savedir, uint64_t segment, int flags,
                       uint8_t* seg_hashes, uint8_t* frag_hashes, uint64_t cap, uint64_t* nseg_out, uint8_t fid[32]) {
    if (!r || !path || !savedir || !fid) return bad_arg();
    dm_ctx* c = r->c;
    const int g = rs_lane(c);
    CallLock lk(c, g, kReserved);
    if (nseg_out) *nseg_out = 0;
    FileSet fs;
    RC_TRY(open_files(c, &path, 1, fs));   // "open <path>: ..." first, as os.Open would fail
    const uint64_t size = fs.size[0];
    if (size == 0) return fail(c, DM_ERR_EMPTY, "Empty data");
    RC_TRY(process_check(r, size, segment));
    const uint64_t nseg = ceil_div(size, segment);
    if (nseg_out) *nseg_out = nseg;
    if ((seg_hashes || frag_hashes) && cap < nseg)
        return fail(c, DM_ERR_INVALID, "dm_full_processing: %llu segments, digest arrays hold %llu",
                    (unsigned long long)nseg, (unsigned long long)cap);
    std::string dir = savedir;
    while (dir.size() > 1 && dir.back() == '/') dir.pop_back();
    const std::string me = mkdir_all(dir);
    if (!me.empty()) return fail(c, DM_ERR_IO, "%s", me.c_str());
    const int total = r->k + r->m;
    std::vector<uint8_t> segd(32 * nseg), fragd(32 * nseg * total);
    std::vector<std::pair<std::string, uint64_t>> pend;
    Dev& d = c->devs[g];
    int rc = full_processing_windows(r, d, fs, dir, segment, flags, segd, fragd, pend, fid);
    {
        if (rc != DM_OK) {   // a failed call may leave copies queued: none may land in a slot the next call fills
            (void)hipStreamSynchronize(d.copy);
            (void)hipStreamSynchronize(d.stream);
        }
        // the window buffers grow with the file (up to 32 GiB of segments + 64 GiB of parity): give
        // back what a large call took beyond kFpKeepBytes, so it does not stay resident beside
        // other work on this GPU; the call has synchronised its streams already
        if (d.data.cap > kFpKeepBytes) c->reaper.put(d.id, d.data);
        if (rs_ln(r, d).work.cap > kFpKeepBytes) c->reaper.put(d.id, rs_ln(r, d).work);
    }
    for (size_t i = 0; rc == DM_OK && i < pend.size(); i++) {
        const uint64_t at = pend[i].second;
        const uint8_t* dig = (at >> 63) ? segd.data() + ~at : fragd.data() + at;
        const std::string to = dir + "/" + hex32(dig);
        if (::rename(pend[i].first.c_str(), to.c_str()) != 0)
            rc = fail(c, DM_ERR_IO, "rename %s %s: %s", pend[i].first.c_str(), to.c_str(), go_errno(errno).c_str());
        else
            pend[i].first.clear();
    }
    if (rc != DM_OK) {   // no temporary survives a failed call
        for (const auto& p : pend)
            if (!p.first.empty()) ::unlink(p.first.c_str());
        return rc;
    }
    if (seg_hashes) std::memcpy(seg_hashes, segd.data(), segd.size());
    if (frag_hashes) std::memcpy(frag_hashes, fragd.data(), fragd.size());
    return DM_OK;
}

}  // extern "C"
