/*
 * merkle_oracle.c -- CPU restatement of DeOSS common/hashtree (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity oracle and the CPU baseline ("port") for the MI355X Merkle path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / the baseline being timed.  The product (deoss_amd/libdeoss_merkle.so)
 * never links or calls it.
 *
 * What it restates (reference paths relative to /root/reference):
 *   - common/hashtree/hashtree.go:23-30  HashTreeContent.CalculateHash = SHA-256(chunk bytes),
 *                                        no prefix, big-endian digest (Go crypto/sha256, FIPS 180-4).
 *   - common/hashtree/types.go:19-39     NewHashTree: one leaf per chunk, empty list -> "Empty data".
 *   - github.com/cbergoon/merkletree v0.2.0 (go.mod:10, not vendored; restated from its published
 *     source): buildWithContent duplicates the last leaf when the leaf count is odd, then
 *     buildIntermediate hashes pairs (i, i+1), or (i, i) for a trailing odd node, SHA-256(left||right),
 *     one level per call, returning when a level has exactly 2 nodes.  Equivalent rule used here:
 *        L = leaves; do { L = [H(L[2j] || L[min(2j+1,|L|-1)])] } while (|L| > 1)   (>= 1 level)
 *
 * Pinning: the only reference known-answer test is common/hashtree/hashtree_test.go:20-82
 * (4 leaves "content_one".."content_four"); tests/test_oracle.py checks this file against it,
 * against NIST FIPS 180-4 SHA-256 vectors, and against Python hashlib restatement fixtures.
 *
 * Two SHA-256 back ends: portable scalar C, and x86 SHA-NI (the instructions Go 1.22's
 * crypto/sha256 uses on amd64 when the CPU has them), selected at run time.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t IV256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                  0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

/* ---- portable scalar compression (FIPS 180-4 section 6.2.2) ---- */
static void compress_scalar(uint32_t st[8], const uint8_t *p, size_t nblocks) {
    while (nblocks--) {
        uint32_t w[64];
        for (int t = 0; t < 16; t++)
            w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) |
                   ((uint32_t)p[4 * t + 2] << 8) | (uint32_t)p[4 * t + 3];
        for (int t = 16; t < 64; t++) {
            uint32_t s0 = ROR(w[t - 15], 7) ^ ROR(w[t - 15], 18) ^ (w[t - 15] >> 3);
            uint32_t s1 = ROR(w[t - 2], 17) ^ ROR(w[t - 2], 19) ^ (w[t - 2] >> 10);
            w[t] = w[t - 16] + s0 + w[t - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
        for (int t = 0; t < 64; t++) {
            uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
            uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
        p += 64;
    }
}

#if defined(__x86_64__)
/* ---- x86 SHA-NI compression (Intel SHA extensions) ---- */
__attribute__((target("sha,sse4.1")))
static void compress_shani(uint32_t st[8], const uint8_t *p, size_t nblocks) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_loadu_si128((const __m128i *)&st[0]);   /* a b c d */
    __m128i s1 = _mm_loadu_si128((const __m128i *)&st[4]);    /* e f g h */
    tmp = _mm_shuffle_epi32(tmp, 0xB1);                       /* c d a b -> CDAB */
    s1 = _mm_shuffle_epi32(s1, 0x1B);                         /* h g f e -> EFGH */
    __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);                 /* ABEF */
    s1 = _mm_blend_epi16(s1, tmp, 0xF0);                      /* CDGH */
    while (nblocks--) {
        __m128i abef = s0, cdgh = s1, msg, m0, m1, m2, m3;
        m0 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 0)), MASK);
        m1 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16)), MASK);
        m2 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 32)), MASK);
        m3 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 48)), MASK);
#define RND4(mi, k)                                                            \
    msg = _mm_add_epi32(mi, _mm_loadu_si128((const __m128i *)&K256[k]));     \
    s1 = _mm_sha256rnds2_epu32(s1, s0, msg);                                 \
    s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(msg, 0x0E));
#define SCHED(ma, mb, mc, md)                                                  \
    ma = _mm_sha256msg1_epu32(ma, mb);                                        \
    ma = _mm_add_epi32(ma, _mm_alignr_epi8(md, mc, 4));                       \
    ma = _mm_sha256msg2_epu32(ma, md);
        RND4(m0, 0); RND4(m1, 4); RND4(m2, 8); RND4(m3, 12);
        for (int k = 16; k < 64; k += 16) {
            SCHED(m0, m1, m2, m3); RND4(m0, k);
            SCHED(m1, m2, m3, m0); RND4(m1, k + 4);
            SCHED(m2, m3, m0, m1); RND4(m2, k + 8);
            SCHED(m3, m0, m1, m2); RND4(m3, k + 12);
        }
#undef RND4
#undef SCHED
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
        p += 64;
    }
    tmp = _mm_shuffle_epi32(s0, 0x1B);                        /* FEBA */
    s1 = _mm_shuffle_epi32(s1, 0xB1);                         /* DCHG */
    s0 = _mm_blend_epi16(tmp, s1, 0xF0);                      /* DCBA */
    s1 = _mm_alignr_epi8(s1, tmp, 8);                         /* HGFE */
    _mm_storeu_si128((__m128i *)&st[0], s0);
    _mm_storeu_si128((__m128i *)&st[4], s1);
}

static int cpu_has_shani(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    return (b >> 29) & 1;
}
#endif

/* backend: 0 = auto, 1 = scalar, 2 = sha-ni */
static int g_backend = 0;

int or_set_backend(int b) { g_backend = b; return 0; }

int or_backend(void) {
#if defined(__x86_64__)
    if (g_backend == 1) return 1;
    if (cpu_has_shani()) return 2;
#endif
    return 1;
}

static void compress(uint32_t st[8], const uint8_t *p, size_t nblocks) {
#if defined(__x86_64__)
    if (or_backend() == 2) { compress_shani(st, p, nblocks); return; }
#endif
    compress_scalar(st, p, nblocks);
}

/* SHA-256 of len bytes (FIPS 180-4 padding: 0x80, zeros, 64-bit big-endian bit length). */
void or_sha256(const void *data, uint64_t len, uint8_t out[32]) {
    const uint8_t *p = (const uint8_t *)data;
    uint32_t st[8];
    memcpy(st, IV256, sizeof st);
    uint64_t full = len / 64;
    compress(st, p, full);
    uint8_t tail[128];
    uint64_t r = len - full * 64;
    memset(tail, 0, sizeof tail);
    if (r) memcpy(tail, p + full * 64, r);
    tail[r] = 0x80;
    uint64_t tb = (r + 9 <= 64) ? 64 : 128;
    uint64_t bits = len * 8;
    for (int i = 0; i < 8; i++) tail[tb - 1 - i] = (uint8_t)(bits >> (8 * i));
    compress(st, tail, tb / 64);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24); out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8); out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* One tree level, merkletree v0.2.0 buildIntermediate: out[j] = H(in[2j] || in[min(2j+1,n-1)]). */
static uint64_t level_up(const uint8_t *in, uint64_t n, uint8_t *out) {
    uint64_t m = (n + 1) / 2;
    for (uint64_t j = 0; j < m; j++) {
        uint8_t buf[64];
        uint64_t r = (2 * j + 1 < n) ? 2 * j + 1 : n - 1;
        memcpy(buf, in + 64 * j, 32);
        memcpy(buf + 32, in + 32 * r, 32);
        or_sha256(buf, 64, out + 32 * j);
    }
    return m;
}

/* Reduce n digests for exactly `levels` levels (levels = -1: until one node, >= 1 level).
 * Result nodes are written to `out` (capacity n*32); returns the node count. */
uint64_t or_reduce(const uint8_t *digests, uint64_t n, int levels, uint8_t *out) {
    if (n == 0) return 0;
    uint8_t *a = (uint8_t *)malloc(32 * n), *b = (uint8_t *)malloc(32 * ((n + 1) / 2 + 1));
    memcpy(a, digests, 32 * n);
    uint64_t cur = n;
    int done = 0;
    for (;;) {
        if (levels >= 0 && done >= levels) break;
        if (levels < 0 && done >= 1 && cur == 1) break;
        uint64_t m = level_up(a, cur, b);
        uint8_t *t = a; a = b; b = t;
        /* a must have room for the next level's input; b capacity (n+1)/2+1 suffices after the swap. */
        cur = m; done++;
    }
    memcpy(out, a, 32 * cur);
    free(a); free(b);
    return cur;
}

/* ---- leaf hashing, serial ("faithful") or threaded ---- */
typedef struct {
    const void *const *ptrs; const uint64_t *lens; uint8_t *leaf;
    uint64_t begin, end;
} leaf_job;

static void *leaf_worker(void *arg) {
    leaf_job *j = (leaf_job *)arg;
    for (uint64_t i = j->begin; i < j->end; i++) or_sha256(j->ptrs[i], j->lens[i], j->leaf + 32 * i);
    return NULL;
}

static void hash_leaves(const void *const *ptrs, const uint64_t *lens, uint64_t n, uint8_t *leaf, int nthreads) {
    if (nthreads <= 1 || n < 2) {
        for (uint64_t i = 0; i < n; i++) or_sha256(ptrs[i], lens[i], leaf + 32 * i);
        return;
    }
    if ((uint64_t)nthreads > n) nthreads = (int)n;
    pthread_t th[256];
    leaf_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    /* interleaved-by-bytes balance is unnecessary: leaves are near-uniform in size */
    for (int t = 0; t < nthreads; t++) {
        jobs[t].ptrs = ptrs; jobs[t].lens = lens; jobs[t].leaf = leaf;
        jobs[t].begin = n * t / nthreads; jobs[t].end = n * (t + 1) / nthreads;
        pthread_create(&th[t], NULL, leaf_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* NewHashTree over an explicit chunk list (types.go:19-39 with the file reads replaced by
 * in-memory chunks).  Returns -1 for an empty list ("Empty data"), else 0. */
int or_root_chunks(const void *const *ptrs, const uint64_t *lens, uint64_t n,
                   uint8_t *leaf_out, uint8_t root[32], int nthreads) {
    if (n == 0) return -1;
    uint8_t *leaf = leaf_out ? leaf_out : (uint8_t *)malloc(32 * n);
    hash_leaves(ptrs, lens, n, leaf, nthreads);
    uint8_t *tmp = (uint8_t *)malloc(32 * n);
    or_reduce(leaf, n, -1, tmp);
    memcpy(root, tmp, 32);
    free(tmp);
    if (!leaf_out) free(leaf);
    return 0;
}

/* Object buffer split into fixed-size chunks (the last one short). */
int or_root_buffer(const void *buf, uint64_t len, uint64_t chunk, uint8_t *leaf_out,
                   uint8_t root[32], int nthreads) {
    if (chunk == 0) return -2;
    uint64_t n = len ? (len + chunk - 1) / chunk : 0;
    if (n == 0) return -1;
    const void **ptrs = (const void **)malloc(sizeof(void *) * n);
    uint64_t *lens = (uint64_t *)malloc(sizeof(uint64_t) * n);
    for (uint64_t i = 0; i < n; i++) {
        ptrs[i] = (const uint8_t *)buf + i * chunk;
        lens[i] = (i + 1 < n) ? chunk : len - i * chunk;
    }
    int rc = or_root_chunks(ptrs, lens, n, leaf_out, root, nthreads);
    free(ptrs); free(lens);
    return rc;
}

/* ---- synthetic object bytes: word[i] = splitmix64(seed ^ i), little-endian ----
 * Same function as the device generator (deoss_amd/csrc/merkle_kernels.hip). Fills bytes
 * [off, off+nbytes) of the object stream; off and nbytes multiples of 8. */
static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

void or_fill_splitmix(void *dst, uint64_t off, uint64_t nbytes, uint64_t seed) {
    uint64_t *w = (uint64_t *)dst;
    uint64_t i0 = off / 8, nw = nbytes / 8;
    for (uint64_t i = 0; i < nw; i++) w[i] = splitmix64(seed ^ (i0 + i));
}

/* ---- root of a synthetic object that never exists in memory as a whole ----
 * The object is bytes [base, base + len) of the splitmix64 stream `seed` (base and len multiples
 * of 8; base 0 but for one GPU's share of a larger object, or_root_synthetic_at), split into
 * `chunk`-byte leaves (chunk a multiple of 64).  Each thread takes whole leaves (atomic counter),
 * regenerates a leaf's bytes 1 MiB at a time into its own buffer and feeds them to the compression
 * function, so a 1 TiB object (BASELINE configs[3]) is checked with nthreads x 1 MiB of memory. */
typedef struct {
    uint64_t base, len, chunk, seed, n;
    uint64_t next;           /* next leaf to take (atomic) */
    uint8_t *leaf;
} synth_job;

static void synth_leaf(const synth_job *j, uint64_t i, uint8_t *buf, uint64_t bufsz) {
    const uint64_t b0 = i * j->chunk;
    const uint64_t l = (i + 1 < j->n) ? j->chunk : j->len - b0;
    uint32_t st[8];
    memcpy(st, IV256, sizeof st);
    uint64_t done = 0;
    while (done + 64 <= l) {   /* whole blocks, bufsz (a multiple of 64) at a time */
        uint64_t take = l - done < bufsz ? (l - done) / 64 * 64 : bufsz;
        or_fill_splitmix(buf, j->base + b0 + done, take, j->seed);
        compress(st, buf, take / 64);
        done += take;
    }
    uint8_t tail[128];
    const uint64_t r = l - done;   /* < 64, a multiple of 8 */
    memset(tail, 0, sizeof tail);
    if (r) or_fill_splitmix(tail, j->base + b0 + done, r, j->seed);
    tail[r] = 0x80;
    const uint64_t tb = (r + 9 <= 64) ? 64 : 128, bits = l * 8;
    for (int k = 0; k < 8; k++) tail[tb - 1 - k] = (uint8_t)(bits >> (8 * k));
    compress(st, tail, tb / 64);
    uint8_t *out = j->leaf + 32 * i;
    for (int k = 0; k < 8; k++) {
        out[4 * k] = (uint8_t)(st[k] >> 24); out[4 * k + 1] = (uint8_t)(st[k] >> 16);
        out[4 * k + 2] = (uint8_t)(st[k] >> 8); out[4 * k + 3] = (uint8_t)st[k];
    }
}

static void *synth_worker(void *arg) {
    synth_job *j = (synth_job *)arg;
    const uint64_t bufsz = 1u << 20;
    uint8_t *buf = (uint8_t *)malloc(bufsz);
    for (;;) {
        uint64_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        synth_leaf(j, i, buf, bufsz);
    }
    free(buf);
    return NULL;
}

/* Root of the tree over bytes [base, base + len) of the stream: one GPU's share of a larger object
 * (configs[3]: 4,096 leaves at base = rank x 128 GiB), whose subtree root the device computes.
 * Returns -1 for len 0, -2 for a bad chunk/len/base, else 0; leaf_out (nullable) gets n x 32 bytes. */
int or_root_synthetic_at(uint64_t base, uint64_t len, uint64_t chunk, uint64_t seed, uint8_t *leaf_out,
                         uint8_t root[32], int nthreads) {
    if (len == 0) return -1;
    if (chunk == 0 || chunk % 64 || len % 8 || base % 8) return -2;
    synth_job j = {base, len, chunk, seed, (len + chunk - 1) / chunk, 0, NULL};
    j.leaf = leaf_out ? leaf_out : (uint8_t *)malloc(32 * j.n);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((uint64_t)nthreads > j.n) nthreads = (int)j.n;
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, synth_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    uint8_t *tmp = (uint8_t *)malloc(32 * j.n);
    or_reduce(j.leaf, j.n, -1, tmp);
    memcpy(root, tmp, 32);
    free(tmp);
    if (!leaf_out) free(j.leaf);
    return 0;
}

/* Returns -1 for len 0, -2 for a bad chunk/len, else 0; leaf_out (nullable) gets n x 32 bytes. */
int or_root_synthetic(uint64_t len, uint64_t chunk, uint64_t seed, uint8_t *leaf_out, uint8_t root[32],
                      int nthreads) {
    return or_root_synthetic_at(0, len, chunk, seed, leaf_out, root, nthreads);
}
