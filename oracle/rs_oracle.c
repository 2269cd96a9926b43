/*
 * rs_oracle.c -- CPU restatement of the Reed-Solomon fragment coding DeOSS's upload path uses
 * (TEST INFRASTRUCTURE ONLY: the checker for deoss_amd's dm_rs_* kernels and the CPU baseline
 * bench.py times; the product library never links or calls it).
 *
 * Reference: DeOSS calls the cess-go-sdk (go.mod:8), which erasure-codes every 32 MiB segment into
 * chain.DataShards = 4 data + chain.ParShards = 8 parity fragments (constants used at
 * node/tracker.go:250,369 and node/fileHandler.go:250) with github.com/klauspost/reedsolomon
 * v1.12.4 (go.mod:65).  Neither module is vendored under /root/reference, so this file restates
 * klauspost/reedsolomon's published algorithm for New(dataShards, parityShards) with default
 * options:
 *   - GF(2^8) with generating polynomial 29 (x^8 + x^4 + x^3 + x^2 + 1, 0x11d), generator 2
 *     (galois.go: logTable / expTable, galMultiply, galExp);
 *   - buildMatrix (reedsolomon.go): vm = vandermonde(total, data) with vm[r][c] = galExp(r, c),
 *     encoding matrix = vm * inverse(top data x data square of vm) -> systematic, top = identity;
 *   - Encode: parity[i] = sum_j M[data+i][j] * data[j] (bytewise GF multiply-add);
 *   - Reconstruct: take the first `data` present shards in index order, invert their rows of M,
 *     rebuild missing data shards from that inverse, then missing parity shards from the data;
 *   - Split: perShard = ceil(len / data), zero padding of the last shard.
 * Parity is UNPINNED against klauspost itself (no fixtures in the reference; the module is
 * absent): tests/test_rs.py checks this file against an independent Python restatement and
 * against the algebraic properties (systematic top, any `data` of the shards reconstruct all).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

static uint8_t gf_exp[510], gf_log[256];
static uint8_t gf_mul_tab[256][256];
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_init(void) {
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        gf_exp[i] = (uint8_t)x;
        gf_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x100 | 29;   /* reduce by x^8 + 29 */
    }
    for (int i = 255; i < 510; i++) gf_exp[i] = gf_exp[i - 255];
    gf_log[0] = 0;
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            gf_mul_tab[a][b] = (a == 0 || b == 0) ? 0 : gf_exp[gf_log[a] + gf_log[b]];
}

static uint8_t gf_mul(uint8_t a, uint8_t b) { return gf_mul_tab[a][b]; }

/* galExp(a, n): a^n in GF(2^8); galExp(a, 0) = 1, galExp(0, n>0) = 0. */
static uint8_t gf_pow(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return gf_exp[(gf_log[a] * n) % 255];
}

/* Gauss-Jordan inverse of the k x k matrix m (row-major) into inv; 0 on success, -1 singular. */
static int gf_invert(const uint8_t *m, int k, uint8_t *inv) {
    uint8_t w[16][32];
    if (k > 16) return -1;
    for (int r = 0; r < k; r++) {
        for (int c = 0; c < k; c++) {
            w[r][c] = m[r * k + c];
            w[r][k + c] = (uint8_t)(r == c);
        }
    }
    for (int c = 0; c < k; c++) {
        int p = c;
        while (p < k && w[p][c] == 0) p++;
        if (p == k) return -1;
        if (p != c) {
            uint8_t t[32];
            memcpy(t, w[p], sizeof t);
            memcpy(w[p], w[c], sizeof t);
            memcpy(w[c], t, sizeof t);
        }
        const uint8_t s = gf_exp[255 - gf_log[w[c][c]]];   /* 1 / pivot */
        for (int j = 0; j < 2 * k; j++) w[c][j] = gf_mul(w[c][j], s);
        for (int r = 0; r < k; r++) {
            if (r == c || w[r][c] == 0) continue;
            const uint8_t f = w[r][c];
            for (int j = 0; j < 2 * k; j++) w[r][j] ^= gf_mul(f, w[c][j]);
        }
    }
    for (int r = 0; r < k; r++) memcpy(inv + r * k, &w[r][k], (size_t)k);
    return 0;
}

int or_rs_gf_mul(int a, int b) {
    pthread_once(&gf_once, gf_init);
    return gf_mul((uint8_t)a, (uint8_t)b);
}

/* Encoding matrix (total x data, row-major) of New(data, parity): buildMatrix restated. */
int or_rs_matrix(int data, int total, uint8_t *out) {
    pthread_once(&gf_once, gf_init);
    if (data < 1 || data > 16 || total <= data || total > 256) return -1;
    uint8_t top[256], inv[256];
    for (int r = 0; r < data; r++)
        for (int c = 0; c < data; c++) top[r * data + c] = gf_pow((uint8_t)r, c);
    if (gf_invert(top, data, inv) != 0) return -1;
    for (int r = 0; r < total; r++) {
        for (int c = 0; c < data; c++) {
            uint8_t acc = 0;
            for (int t = 0; t < data; t++) acc ^= gf_mul(gf_pow((uint8_t)r, t), inv[t * data + c]);
            out[r * data + c] = acc;
        }
    }
    return 0;
}

/* out[i] = sum_j rows[i][j] * in[j] over bytes [lo, hi). */
static void code_range(const uint8_t *rows, int nin, int nout, const uint8_t *const *in, uint8_t *const *out,
                       size_t lo, size_t hi) {
    for (int i = 0; i < nout; i++) {
        uint8_t *o = out[i];
        memset(o + lo, 0, hi - lo);
        for (int j = 0; j < nin; j++) {
            const uint8_t *tab = gf_mul_tab[rows[i * nin + j]];
            const uint8_t *p = in[j];
            for (size_t x = lo; x < hi; x++) o[x] ^= tab[p[x]];
        }
    }
}

typedef struct {
    const uint8_t *rows;
    int nin, nout;
    const uint8_t *const *in;
    uint8_t *const *out;
    size_t lo, hi;
} code_job;

static void *code_thread(void *arg) {
    code_job *j = (code_job *)arg;
    code_range(j->rows, j->nin, j->nout, j->in, j->out, j->lo, j->hi);
    return NULL;
}

static void code_shards(const uint8_t *rows, int nin, int nout, const uint8_t *const *in, uint8_t *const *out,
                        size_t n, int nthreads) {
    if (nthreads <= 1 || n < 65536) {
        code_range(rows, nin, nout, in, out, 0, n);
        return;
    }
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    code_job jobs[256];
    const size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = per * (size_t)t, hi = lo + per;
        if (lo >= n) break;
        if (hi > n) hi = n;
        jobs[t] = (code_job){rows, nin, nout, in, out, lo, hi};
        if (pthread_create(&th[t], NULL, code_thread, &jobs[t]) != 0) {
            code_range(rows, nin, nout, in, out, lo, hi);
            continue;
        }
        started = t + 1;
    }
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
}

/* Encode: parity[i] (i < parity) from data[j] (j < data), shard bytes each. */
int or_rs_encode(int data, int parity, const uint8_t *const *dshards, uint8_t *const *pshards, size_t shard,
                 int nthreads) {
    uint8_t m[256 * 16];
    if (or_rs_matrix(data, data + parity, m) != 0) return -1;
    code_shards(m + data * data, data, parity, dshards, pshards, shard, nthreads);
    return 0;
}

/* Reconstruct every shard whose present[i] == 0 (all data + parity shards, in place). */
int or_rs_reconstruct(int data, int parity, uint8_t *const *shards, const uint8_t *present, size_t shard,
                      int nthreads) {
    const int total = data + parity;
    uint8_t m[256 * 16], sub[256], inv[256];
    if (or_rs_matrix(data, total, m) != 0) return -1;
    int valid[16], nv = 0;
    for (int r = 0; r < total && nv < data; r++)
        if (present[r]) valid[nv++] = r;
    if (nv < data) return -2;   /* too few shards */
    for (int r = 0; r < data; r++) memcpy(sub + r * data, m + valid[r] * data, (size_t)data);
    if (gf_invert(sub, data, inv) != 0) return -1;
    const uint8_t *in[16];
    for (int r = 0; r < data; r++) in[r] = shards[valid[r]];
    uint8_t rows[256 * 16];
    uint8_t *out[256];
    int nout = 0;
    for (int i = 0; i < data; i++) {
        if (present[i]) continue;
        memcpy(rows + nout * data, inv + i * data, (size_t)data);
        out[nout++] = shards[i];
    }
    if (nout) code_shards(rows, data, nout, in, out, shard, nthreads);
    nout = 0;
    for (int i = data; i < total; i++) {
        if (present[i]) continue;
        memcpy(rows + nout * data, m + i * data, (size_t)data);
        out[nout++] = shards[i];
    }
    if (nout) code_shards(rows, data, nout, (const uint8_t *const *)shards, out, shard, nthreads);
    return 0;
}
