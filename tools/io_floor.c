// io_floor.c -- the host file-I/O floor of FullProcessing(file, "", savedir): read <file> with R
// threads (pread, 16 MiB parts) and write the same number and sizes of output files the call
// writes (<nfrag> files of <frag> bytes + <nseg> files of <seg> bytes, from a buffer of the file's
// first bytes) with W threads into <dir>.  No hashing, no coding, no GPU: the bound that
// dm_full_processing's overlapped pipeline is measured against (bench.py --workload fullprocessing).
// usage: io_floor <file> <dir> <frag> <nfrag> <seg> <nseg> <R> <W>   -> prints seconds
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

static const char *g_file, *g_dir;
static uint64_t g_size, g_frag, g_nfrag, g_seg, g_nseg;
static int g_R, g_W;
static uint8_t *g_src;   // first max(frag, seg) bytes of the file (write source)

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *reader(void *arg) {
    const int id = (int)(intptr_t)arg;
    const uint64_t part = 16ull << 20;
    uint8_t *buf = malloc(part);
    const int fd = open(g_file, O_RDONLY);
    for (uint64_t off = (uint64_t)id * part; off < g_size; off += (uint64_t)g_R * part) {
        const uint64_t n = g_size - off < part ? g_size - off : part;
        if (pread(fd, buf, n, (off_t)off) != (ssize_t)n) { perror("pread"); exit(1); }
    }
    close(fd);
    free(buf);
    return NULL;
}

static void *writer(void *arg) {
    const int id = (int)(intptr_t)arg;
    char path[4096];
    for (uint64_t i = (uint64_t)id; i < g_nfrag + g_nseg; i += (uint64_t)g_W) {
        const uint64_t len = i < g_nfrag ? g_frag : g_seg;
        snprintf(path, sizeof path, "%s/io%llu", g_dir, (unsigned long long)i);
        const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) { perror("open"); exit(1); }
        for (uint64_t d = 0; d < len;) {
            const ssize_t w = write(fd, g_src + d, len - d);
            if (w <= 0) { perror("write"); exit(1); }
            d += (uint64_t)w;
        }
        close(fd);
    }
    return NULL;
}

int main(int argc, char **argv) {
    if (argc != 9) {
        fprintf(stderr, "usage: io_floor <file> <dir> <frag> <nfrag> <seg> <nseg> <R> <W>\n");
        return 2;
    }
    g_file = argv[1];
    g_dir = argv[2];
    g_frag = strtoull(argv[3], 0, 10);
    g_nfrag = strtoull(argv[4], 0, 10);
    g_seg = strtoull(argv[5], 0, 10);
    g_nseg = strtoull(argv[6], 0, 10);
    g_R = atoi(argv[7]);
    g_W = atoi(argv[8]);
    struct stat st;
    if (stat(g_file, &st) != 0) { perror("stat"); return 1; }
    g_size = (uint64_t)st.st_size;
    const uint64_t srcn = g_frag > g_seg ? g_frag : g_seg;
    g_src = malloc(srcn);
    memset(g_src, 0x5a, srcn);
    pthread_t th[256];
    const double t0 = now();
    for (int i = 0; i < g_R; i++) pthread_create(&th[i], NULL, reader, (void *)(intptr_t)i);
    for (int i = 0; i < g_W; i++) pthread_create(&th[g_R + i], NULL, writer, (void *)(intptr_t)i);
    for (int i = 0; i < g_R + g_W; i++) pthread_join(th[i], NULL);
    printf("%.6f\n", now() - t0);
    free(g_src);
    return 0;
}
