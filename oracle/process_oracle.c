/*
 * process_oracle.c -- CPU restatement of cess-go-sdk process.FullProcessing with cipher "" (TEST
 * INFRASTRUCTURE ONLY: the checker for deoss_amd's dm_process_* pipeline and the CPU baseline
 * bench.py times for it; the product library never links or calls it).
 *
 * Reference: every DeOSS upload and the fragment download path compute the file id ("fid") and
 * the fragment names with process.FullProcessing(file, cipher, savedir) from cess-go-sdk
 * (go.mod:8, v0.7.1-0.20250210085828-e5828b43cd15; not vendored under /root/reference).  Call
 * sites: node/fileHandler.go:771, node/objectHandler.go:168, node/filesHandler.go:201,
 * node/resumeHandler.go:326, node/tracker.go:767-769, node/fileHandler.go:964,997 (the last two
 * with cipher "").  Restated composition (the SDK's published source, not checkable offline):
 *   1. cut the file into chain.SegmentSize (32 MiB) segments, the last one zero-padded
 *      (node/fileHandler.go:862-872 sizes storage by whole segments the same way);
 *   2. each segment is coded with klauspost/reedsolomon New(chain.DataShards = 4,
 *      chain.ParShards = 8) Split + Encode into 12 fragments of chain.FragmentSize = 8 MiB
 *      (node/tracker.go:250 checks FragmentSize * 12 = "96M"); rs_oracle.c restates the coder;
 *   3. every segment and fragment is named by the hex SHA-256 of its bytes: SegmentDataInfo
 *      .SegmentHash / .FragmentHash hold savedir/<hex> paths (node/fileHandler.go:967-969
 *      matches filepath.Base(FragmentHash[j]) against the requested fragment hash);
 *   4. fid = hex(MerkleRoot()) of common/hashtree.NewHashTree(segment paths) (types.go:19-39),
 *      i.e. the merkle_oracle.c tree over the segment digests.
 * Parity of the composition is UNPINNED (no SDK source or fixture in the container); its parts
 * are pinned: SHA-256 (NIST), the hashtree root (hashtree_test.go:20-82), the RS coder
 * (klauspost TestOneEncode).  The cipher branch (AES before coding) is not restated.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>

void or_sha256(const void *data, uint64_t len, uint8_t out[32]);
uint64_t or_reduce(const uint8_t *digests, uint64_t n, int levels, uint8_t *out);
int or_rs_encode(int data, int parity, const uint8_t *const *dshards, uint8_t *const *pshards, size_t shard,
                 int nthreads);

/* FullProcessing over an in-memory object of len bytes.  segment % data == 0.
 * seg_hashes: nseg x 32; frag_hashes: nseg x (data + parity) x 32 (data fragments first);
 * frags (nullable): nseg x (data + parity) x (segment / data) bytes, segment-major.
 * Returns nseg (> 0), -1 for an empty object, -2 for bad arguments. */
int64_t or_full_processing(const void *buf, uint64_t len, uint64_t segment, int data, int parity,
                           uint8_t *seg_hashes, uint8_t *frag_hashes, uint8_t fid[32], uint8_t *frags,
                           int nthreads) {
    if (len == 0) return -1;
    if (segment == 0 || data < 1 || parity < 1 || data > 16 || parity > 16 || segment % (uint64_t)data) return -2;
    const uint64_t nseg = (len + segment - 1) / segment, frag = segment / (uint64_t)data;
    const int total = data + parity;
    uint8_t *seg = (uint8_t *)malloc(segment);
    uint8_t *par = (uint8_t *)malloc(frag * (uint64_t)parity);
    if (!seg || !par) { free(seg); free(par); return -2; }
    for (uint64_t s = 0; s < nseg; s++) {
        const uint64_t off = s * segment, have = len - off < segment ? len - off : segment;
        memcpy(seg, (const uint8_t *)buf + off, have);               /* step 1: cut + zero pad */
        memset(seg + have, 0, segment - have);
        or_sha256(seg, segment, seg_hashes + 32 * s);                /* segment name / leaf */
        const uint8_t *din[16];
        uint8_t *pout[16];
        for (int j = 0; j < data; j++) din[j] = seg + (uint64_t)j * frag;   /* Split: in order */
        for (int i = 0; i < parity; i++) pout[i] = par + (uint64_t)i * frag;
        or_rs_encode(data, parity, din, pout, frag, nthreads);              /* step 2 */
        for (int j = 0; j < total; j++) {                                   /* step 3 */
            const uint8_t *f = j < data ? din[j] : pout[j - data];
            or_sha256(f, frag, frag_hashes + 32 * ((uint64_t)s * total + j));
            if (frags) memcpy(frags + ((uint64_t)s * total + j) * frag, f, frag);
        }
    }
    uint8_t *tmp = (uint8_t *)malloc(32 * nseg);                            /* step 4 */
    or_reduce(seg_hashes, nseg, -1, tmp);
    memcpy(fid, tmp, 32);
    free(tmp); free(seg); free(par);
    return (int64_t)nseg;
}
