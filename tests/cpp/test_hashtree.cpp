// C++ mirror of the reference test common/hashtree/hashtree_test.go:20-82, through the C++ host
// API (include/deoss_hashtree.hpp) and the GPU library.  Prints "PASS" and exits 0 on success.
// Expected digests are computed independently with the CPU oracle's SHA-256 (linked in only as
// the checker, never by the product library).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "deoss_hashtree.hpp"

extern "C" void or_sha256(const void* data, uint64_t len, uint8_t out[32]);

static int fails = 0;
#define EXPECT(c)                                                   \
    do {                                                            \
        if (!(c)) {                                                 \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                \
        }                                                           \
    } while (0)

static hashtree::Digest sha(const std::string& s) {
    hashtree::Digest d;
    or_sha256(s.data(), s.size(), d.data());
    return d;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    const char* contents[] = {"content_one", "content_two", "content_three", "content_four"};
    std::vector<std::string> chunks;
    std::vector<hashtree::Digest> hashes;
    for (const char* c : contents) {
        std::string p = dir + "/" + c;
        FILE* f = std::fopen(p.c_str(), "wb");
        std::fwrite(c, 1, std::strlen(c), f);
        std::fclose(f);
        chunks.push_back(p);
        hashes.push_back(sha(c));
    }
    auto cat = [](const hashtree::Digest& a, const hashtree::Digest& b) {
        return std::string(reinterpret_cast<const char*>(a.data()), 32) + std::string(reinterpret_cast<const char*>(b.data()), 32);
    };
    hashtree::Digest five = sha(cat(hashes[0], hashes[1])), six = sha(cat(hashes[2], hashes[3]));
    hashtree::Digest root = sha(cat(five, six));

    auto [mtree, err] = hashtree::NewHashTree(chunks);
    EXPECT(!err.has_value());
    EXPECT(mtree && mtree->Leafs.size() == 4);
    for (int i = 0; i < 4 && mtree; i++) EXPECT(mtree->Leafs[i].Hash == hashes[i]);
    EXPECT(mtree && mtree->MerkleRoot() == root);

    auto [t0, e0] = hashtree::NewHashTree({});
    EXPECT(!t0 && e0 && e0->message == "Empty data");
    auto [t1, e1] = hashtree::NewHashTree({dir + "/does_not_exist"});
    EXPECT(!t1 && e1 && e1->message.find("no such file or directory") != std::string::npos);

    // odd leaf count: Leafs gets the duplicated last leaf
    std::vector<std::string> three(chunks.begin(), chunks.begin() + 3);
    auto [t3, e3] = hashtree::NewHashTree(three);
    EXPECT(!e3 && t3 && t3->Leafs.size() == 4 && t3->Leafs[3].dup && t3->Leafs[3].Hash == hashes[2]);
    hashtree::Digest h01 = sha(cat(hashes[0], hashes[1])), h22 = sha(cat(hashes[2], hashes[2]));
    EXPECT(t3 && t3->MerkleRoot() == sha(cat(h01, h22)));

    // buffer entry point
    std::string obj = "content_onecontent_two";
    auto [tb, eb] = hashtree::NewHashTreeFromBuffer(obj.data(), obj.size(), 11);
    EXPECT(!eb && tb && tb->MerkleRoot() == sha(cat(hashes[0], hashes[1])));

    auto [tz, ez] = hashtree::NewHashTreeFromBuffer(obj.data(), obj.size(), 0);
    EXPECT(!tz && ez && ez->code == DM_ERR_INVALID);

    // Stream: the Go NewStream call sequence (pieces of any size, Close, Abort, empty body)
    std::string body;
    for (int i = 0; i < 300000; i++) body.push_back((char)(i * 131 + (i >> 9)));
    auto [whole, ew] = hashtree::NewHashTreeFromBuffer(body.data(), body.size(), 4096);
    EXPECT(!ew && whole);
    auto [st, es] = hashtree::Stream::New(4096);
    EXPECT(!es && st);
    for (size_t pos = 0, step = 1; st && pos < body.size(); step = step * 7 % 100003 + 1) {
        const size_t m = std::min(step, body.size() - pos);
        EXPECT(!st->Write(body.data() + pos, m));
        pos += m;
    }
    if (st) {
        auto [ts, ec] = st->Close();
        EXPECT(!ec && ts && whole && ts->MerkleRoot() == whole->MerkleRoot() && ts->Leafs.size() == whole->Leafs.size());
        auto [tc2, ec2] = st->Close();
        EXPECT(!tc2 && ec2);
    }
    auto [se, ese] = hashtree::Stream::New(64);
    if (se) {
        auto [te, ee] = se->Close();
        EXPECT(!te && ee && ee->message == "Empty data");
    }
    auto [sa, esa] = hashtree::Stream::New(64);
    if (sa) {
        EXPECT(!sa->Write(body.data(), 1000));
        sa->Abort();
    }
    auto [sb, esb] = hashtree::Stream::New(100);
    EXPECT(!sb && esb && esb->code == DM_ERR_INVALID);

    // concurrent callers (the batcher path) get the trees a single call gives
    {
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        for (int g = 0; g < 16; g++)
            th.emplace_back([&, g] {
                std::string b(3 * 4096 + 17 * g + 5, '\0');
                for (size_t i = 0; i < b.size(); i++) b[i] = (char)(i * 13 + g);
                auto [t, e] = hashtree::NewHashTreeFromBuffer(b.data(), b.size(), 4096);
                if (e || !t) {
                    bad++;
                    return;
                }
                std::vector<hashtree::Digest> level;
                for (size_t o = 0; o < b.size(); o += 4096) level.push_back(sha(b.substr(o, 4096)));
                for (size_t i = 0; i < level.size(); i++)
                    if (t->Leafs[i].Hash != level[i]) bad++;
                do {   // merkletree v0.2.0: pair (i, i+1), the odd last node with itself
                    std::vector<hashtree::Digest> up;
                    for (size_t i = 0; i < level.size(); i += 2)
                        up.push_back(sha(cat(level[i], level[std::min(i + 1, level.size() - 1)])));
                    level = up;
                } while (level.size() > 1);
                if (t->MerkleRoot() != level[0]) bad++;
            });
        for (auto& x : th) x.join();
        EXPECT(bad == 0);
    }

    // PinnedBuffer: the same body hashed in place from page-locked memory (zero-copy path)
    auto [pb, epb] = hashtree::PinnedBuffer::New(body.size());
    EXPECT(!epb && pb);
    if (pb) {
        std::memcpy(pb->data(), body.data(), body.size());
        auto [tp, etp] = hashtree::NewHashTreeFromBuffer(pb->data(), pb->size(), 4096);
        EXPECT(!etp && tp && whole && tp->MerkleRoot() == whole->MerkleRoot());
    }
    auto [p0, ep0] = hashtree::PinnedBuffer::New(0);
    EXPECT(!p0 && ep0 && ep0->code == DM_ERR_INVALID);

    if (fails) return 1;
    std::printf("PASS\n");
    return 0;
}
