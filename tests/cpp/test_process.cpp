// C++ mirror of the Go process shim (include/deoss_process.hpp) on the GPU: FullProcessing over a
// file and the streaming Writer, both against the CPU oracle's restatement of the SDK composition
// (oracle/process_oracle.c, linked in only as the checker).  Prints "PASS" and exits 0 on success.
#include <cstdio>
#include <cctype>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "deoss_process.hpp"

extern "C" {
void or_fill_splitmix(void* dst, uint64_t off, uint64_t nbytes, uint64_t seed);
int64_t or_full_processing(const void* buf, uint64_t len, uint64_t segment, int data, int parity,
                           uint8_t* seg_hashes, uint8_t* frag_hashes, uint8_t fid[32], uint8_t* frags, int nthreads);
}

static int fails = 0;
#define EXPECT(c)                                                                     \
    do {                                                                              \
        if (!(c)) {                                                                   \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);         \
            fails++;                                                                  \
        }                                                                             \
    } while (0)

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const uint64_t len = 3 * process::SegmentSize + 777;
    std::vector<uint8_t> obj(len + 8);
    or_fill_splitmix(obj.data(), 0, (len + 7) / 8 * 8, 0xDE0552500);
    obj.resize(len);
    const uint64_t nseg = 4;
    std::vector<uint8_t> ws(32 * nseg), wf(32 * nseg * 12);
    uint8_t wfid[32];
    EXPECT(or_full_processing(obj.data(), len, process::SegmentSize, 4, 8, ws.data(), wf.data(), wfid, nullptr, 8) ==
           (int64_t)nseg);
    const std::string want_fid = process::hex32(wfid);
    const std::string file = dir + "/upload.bin";
    std::ofstream(file, std::ios::binary).write(reinterpret_cast<const char*>(obj.data()), (std::streamsize)len);

    // FullProcessing(file, "", savedir)
    auto [info, fid, err] = process::FullProcessing(file, "", dir + "/cache");
    EXPECT(!err && fid == want_fid && info.size() == nseg);
    for (uint64_t s = 0; s < info.size(); s++) {
        EXPECT(info[s].SegmentHash == dir + "/cache/" + process::hex32(ws.data() + 32 * s));
        EXPECT(info[s].FragmentHash.size() == 12);
        for (int j = 0; j < 12 && j < (int)info[s].FragmentHash.size(); j++)
            EXPECT(info[s].FragmentHash[j] == dir + "/cache/" + process::hex32(wf.data() + 32 * (s * 12 + j)));
    }
    {   // data fragment 1 of segment 0 holds file bytes [8 MiB, 16 MiB)
        std::ifstream in(info.empty() ? std::string() : info[0].FragmentHash[1], std::ios::binary);
        std::vector<uint8_t> got((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        const uint64_t frag = process::SegmentSize / 4;
        EXPECT(got.size() == frag && std::memcmp(got.data(), obj.data() + frag, frag) == 0);
    }

    // FindFragment (the download handler's one fragment): the same bytes FullProcessing wrote, by name
    for (auto [s, j] : {std::pair<uint64_t, int>{0, 1}, {nseg - 1, 11}}) {
        const std::string name = process::hex32(wf.data() + 32 * (s * 12 + j));
        auto [bytes, ferr] = process::FindFragment(file, name);
        std::ifstream in(dir + "/cache/" + name, std::ios::binary);
        std::vector<uint8_t> disk((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
        EXPECT(!ferr && !bytes.empty() && bytes == disk);
    }
    {
        auto [none, nerr] = process::FindFragment(file, std::string(64, 'a'));
        EXPECT(!nerr && none.empty());
        auto [bad, berr] = process::FindFragment(file, "xyz");   // names no fragment: not found, no error
        EXPECT(!berr && bad.empty());
        const std::string upper = [&] {
            std::string u = process::hex32(wf.data() + 32);
            for (char& ch : u) ch = (char)std::toupper((unsigned char)ch);
            return u;
        }();
        auto [up, uerr] = process::FindFragment(file, upper);     // the lower-case name exists; this spelling does not
        EXPECT(!uerr && up.empty());
    }

    // Writer: io.MultiWriter(f, w) in the handler; pieces of 1 B .. 5 MiB
    auto [w, werr] = process::Writer::New(dir + "/cache_stream");
    EXPECT(!werr && w);
    if (w) {
        uint64_t pos = 0, step = 1;
        while (pos < len) {
            const uint64_t n = std::min<uint64_t>(len - pos, step);
            EXPECT(!w->Write(obj.data() + pos, n));
            pos += n;
            step = step * 7 % (5u << 20) + 1;
        }
        auto [sinfo, sfid, serr] = w->Close();
        EXPECT(!serr && sfid == want_fid && sinfo.size() == nseg);
    }

    // errors keep the Go shape
    EXPECT(std::get<2>(process::FullProcessing(file, "key", dir + "/cache")).has_value());
    auto missing = std::get<2>(process::FullProcessing(dir + "/nope", "", dir + "/cache"));
    EXPECT(missing && missing->message == "open " + dir + "/nope: no such file or directory");
    std::ofstream(dir + "/empty.bin").close();
    auto empty = std::get<2>(process::FullProcessing(dir + "/empty.bin", "", dir + "/cache"));
    EXPECT(empty && empty->message == "Empty data");
    auto [w2, e2] = process::Writer::New(dir + "/cache_empty");
    if (w2) {
        auto r2 = w2->Close();
        EXPECT(std::get<2>(r2) && std::get<2>(r2)->message == "Empty data");
    }
    if (fails) {
        std::printf("FAILED %d\n", fails);
        return 1;
    }
    std::printf("PASS\n");
    return 0;
}
