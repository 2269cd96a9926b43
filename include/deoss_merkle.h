/*
 * deoss_merkle.h -- C ABI of the MI355X-native Merkle content-hashing path.
 *
 * Drop-in boundary for DeOSS common/hashtree (reference repo paths):
 *   func NewHashTree(chunkPath []string) (*merkletree.MerkleTree, error)   common/hashtree/types.go:19
 *   func (t HashTreeContent) CalculateHash() ([]byte, error)              common/hashtree/hashtree.go:23
 * The Go side binds these symbols through a cgo shim; the root and leaf digests
 * returned here are bit-identical to merkletree v0.2.0's MerkleRoot() / Leafs[i].Hash.
 *
 * Conventions
 *  - Return codes: DM_OK (0) or a negative DM_ERR_*; dm_strerror() gives the message
 *    ("Empty data" for DM_ERR_EMPTY, matching common/hashtree/types.go:21), dm_last_error()
 *    the detailed message of the CALLING THREAD's last failing dm_* call (thread-local: no other
 *    thread's failure can change or free it; every error return sets it, so it is never stale).
 *    Go: hold runtime.LockOSThread across the failing call and the dm_last_error read.
 *  - Digests are the canonical 32-byte big-endian SHA-256 output.  Leaf digests are written
 *    n x 32 bytes in chunk order (leaf_out may be NULL).  merkletree's duplicated last leaf
 *    for odd n is NOT written (it equals leaf n-1).
 *  - Ownership: the caller owns every buffer; nothing is retained after return.
 *  - Threading: every call holds ONE call lane of its context (a per-lane lock; each GPU has
 *    DEOSS_LANES lanes, see dm_create) for its duration; calls on different lanes run in parallel,
 *    calls beyond a GPU's lanes queue.  Host-memory calls (dm_root_buffer / _chunks / _batch,
 *    dm_new_hash_tree, streams) go to the least-loaded GPU and its least-loaded lane, or are sharded
 *    over several GPUs when dm_plan_route says that finishes sooner (never while other calls are
 *    in flight); device-memory calls run on a lane of the GPU that holds their memory; an rs
 *    (dm_rs_*, FullProcessing) lives on its context's first GPU and runs on its lanes.
 *  - Every call leaves the calling thread's current HIP device as it found it (the library
 *    switches to its context's devices inside the call and switches back).
 *  - `stream` arguments are hipStream_t values passed as void*, used verbatim (NULL is HIP's
 *    null stream, e.g. torch's default stream).  *_async calls only enqueue work on that
 *    stream; device inputs must be ready in stream order and outputs are valid once the
 *    stream has reached that point.  Synchronous calls use the context's own streams.
 *    Cost of NULL: the null (legacy default) stream orders with every blocking stream of its GPU,
 *    and each lane's compute stream is one (dm_create), so an *_async call on NULL starts only
 *    after the chains other lanes have queued on that GPU (up to ~0.5 s at 32 MiB chunks), and
 *    their later work waits for it.  Pass a stream created with hipStreamNonBlocking (torch's
 *    side streams are) to run beside them.  The library itself never uses the null stream.
 *  - Tree rule (merkletree v0.2.0, restated in DESIGN.md): level out[j] = SHA256(in[2j] ||
 *    in[min(2j+1, n-1)]), repeated until one node remains, at least one level (n = 1 gives
 *    SHA256(leaf || leaf)).
 */
#ifndef DEOSS_MERKLE_H
#define DEOSS_MERKLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dm_ctx dm_ctx;

enum {
    DM_OK = 0,
    DM_ERR_EMPTY = -1,   /* no chunks: "Empty data" (common/hashtree/types.go:20-22) */
    DM_ERR_INVALID = -2, /* bad argument (NULL pointer, zero chunk size, bad device id, ...) */
    DM_ERR_HIP = -3,     /* HIP runtime error */
    DM_ERR_RCCL = -4,    /* RCCL error */
    DM_ERR_NOMEM = -5,   /* device or pinned-host allocation failed */
    DM_ERR_IO = -6,      /* file open/read failed (dm_new_hash_tree; types.go:25-32) */
    DM_ERR_NODEV = -7    /* no usable GPU */
};

/* Context over one or more GPUs of this process.  devs == NULL/ndev <= 0: device 0 only.
 * With ndev > 1, each host-memory call runs whole on the least-loaded device, unless dm_plan_route
 * shards it: a single object is then split by aligned chunk ranges across devices [0, G') and the
 * per-device subtree roots are gathered with RCCL ("C1"); a batch is split by
 * objects with no exchange.
 * Every GPU carries DEOSS_LANES call lanes (at most 8; unset: 1 to 4, as many as keep at most half
 * of the first GPU's free HBM in idle lane buffers of <= 16 GiB each AND, with every other live
 * context's lanes on that GPU (dm_keep_claimed), at most half of its HBM: 4 for the first two
 * default contexts on an MI355X, 1 after that), each with its own streams,
 * scratch and lock, so that many calls run on one GPU at once and concurrent callers (one gin
 * goroutine per upload) are not serialised behind each other's leaf chains.  A
 * lane's compute stream owns a hardware queue (created with a full CU mask); like every HIP stream
 * made without hipStreamNonBlocking it orders with the legacy null stream, so a caller's stream-0
 * work and a lane's work wait for each other (the library itself never uses stream 0). */
int dm_create(dm_ctx **out, const int *devs, int ndev);
/* dm_create with an explicit lane count per GPU (1..8). */
int dm_create_lanes(dm_ctx **out, const int *devs, int ndev, int lanes);
void dm_destroy(dm_ctx *ctx);
const char *dm_strerror(int rc);
const char *dm_last_error(dm_ctx *ctx);   /* ctx is ignored (kept for ABI compatibility) */
int dm_device_count(dm_ctx *ctx);         /* GPUs of the context */
int dm_lane_count(dm_ctx *ctx);           /* call lanes per GPU */
/* GPUs visible to this process (HIP device count; 0 without a usable GPU).  Lets a binding
 * default to every GPU of the node: dm_create(ctx, {0 .. dm_gpu_count()-1}, n). */
int dm_gpu_count(void);
/* Idle object-buffer bytes the live contexts of this process may keep on HIP device `hip_device`
 * (sum over their lanes on it of the per-lane keep limit): the budget dm_create sizes its default
 * lane count against.  0 on success. */
int dm_keep_claimed(int hip_device, uint64_t *bytes);
/* 1 when the context can shard one object over its GPUs (more than one GPU and its RCCL
 * communicators up), else 0.  A multi-GPU dm_create whose ncclCommInitAll fails still succeeds:
 * the context then runs every call whole on one GPU (batches still split by objects, which needs
 * no exchange), says so once on stderr, and answers 0 here. */
int dm_can_shard(dm_ctx *ctx);

/* Page-locked host memory, visible to every GPU, for callers that want the zero-copy host paths.
 * dm_root_buffer / dm_root_chunks / dm_root_batch hash an object held in such memory in place: K1Q
 * reads it over PCIe, with no H2D copy and no HBM copy, whenever the leaf count is in the latency
 * regime.  A Go upload handler, for example, reads the request body into it
 * (go/hashtree/pinned_hip.go).  Free with dm_host_free.  Any hipHostMalloc / hipHostRegister /
 * torch pin_memory buffer works the same way. */
int dm_host_alloc(uint64_t bytes, void **out);
void dm_host_free(void *p);

/* ---- host-memory entry points (synchronous) ---------------------------------------------- */

/* NewHashTree(chunkPath) (types.go:19-39): each file is one leaf, read whole, in order, with Go's
 * errors ("open <p>: no such file or directory", "read <p>: is a directory").  Streamed: files are
 * pread straight into pinned staging by a few threads, H2D copies overlap the reads, and few long
 * near-equal files (segment files) are hashed in stripes so every leaf chain runs while the rest
 * is read.  With ndev > 1 the file list shards across the devices like dm_root_buffer. */
int dm_new_hash_tree(dm_ctx *ctx, const char *const *paths, uint64_t n, uint8_t *leaf_out,
                     uint8_t root[32]);

/* Same tree over in-memory chunks (one leaf per chunk, arbitrary lengths, 0 allowed). */
int dm_root_chunks(dm_ctx *ctx, const void *const *ptrs, const uint64_t *lens, uint64_t n,
                   uint8_t *leaf_out, uint8_t root[32]);

/* One object buffer split into fixed-size chunks (the last one short): the upload-handler
 * path (host buffer -> pinned staging -> H2D overlapped with leaf hashing -> root). */
int dm_root_buffer(dm_ctx *ctx, const void *host, uint64_t len, uint64_t chunk,
                   uint8_t *leaf_out, uint8_t root[32]);

/* Many independent objects, one root each (roots: nobj x 32 bytes). */
int dm_root_batch(dm_ctx *ctx, const void *const *objs, const uint64_t *lens, uint64_t nobj,
                  uint64_t chunk, uint8_t *roots);

/* ---- streaming: hash while the bytes arrive ------------------------------------------------
 * One object whose bytes are handed over in pieces of any size (e.g. the HTTP upload body as it
 * is received), split into `chunk`-byte leaves (chunk a multiple of 16).  Whole leaves are hashed
 * on the GPU while later pieces are still arriving; close pads the last leaf, builds the tree and
 * frees the stream.  A stream is used by one thread at a time; many streams may share a ctx. */
typedef struct dm_stream dm_stream;
int dm_stream_open(dm_ctx *ctx, uint64_t chunk, dm_stream **out);
int dm_stream_write(dm_stream *st, const void *data, uint64_t len);
/* Root of everything written; leaf_out (nullable) receives min(n, leaf_cap) x 32 bytes of leaf
 * digests, *nleaves (nullable) the leaf count n.  No bytes written -> DM_ERR_EMPTY. */
int dm_stream_close(dm_stream *st, uint8_t *leaf_out, uint64_t leaf_cap, uint64_t *nleaves,
                    uint8_t root[32]);
void dm_stream_abort(dm_stream *st);
const char *dm_stream_error(dm_stream *st);

/* ---- device-resident entry points ------------------------------------------------------- */

/* Root of an object already in HBM on the context's first device (synchronous). */
int dm_root_device(dm_ctx *ctx, const void *dev, uint64_t len, uint64_t chunk, uint8_t root[32]);

/* Stream-ordered form: writes the 32-byte root to device memory dev_root.  leaf_out_dev
 * (nullable) receives n x 32 bytes of leaf digests. */
int dm_root_device_async(dm_ctx *ctx, const void *dev, uint64_t len, uint64_t chunk,
                         void *dev_root, void *leaf_out_dev, void *stream);

/* Shard step (multi-GPU, one process per GPU): hash the leaves of a local chunk range and reduce
 * exactly `levels` levels.  The range must start at a global leaf index that is a multiple of
 * 2^levels; only the globally last range may end in a short chunk or a partial block.
 * Writes ceil(nleaves / 2^levels) nodes (32 B each) to dev_nodes and their count to *n_out. */
int dm_subtree_device_async(dm_ctx *ctx, const void *dev, uint64_t len, uint64_t chunk,
                            uint32_t levels, void *dev_nodes, uint64_t *n_out, void *stream);

/* Final levels: reduce n nodes (32 B each, device memory) to the root with the tree rule.
 * min_one_level != 0 forces at least one level (use when the nodes are leaves). */
int dm_finish_device_async(dm_ctx *ctx, const void *dev_nodes, uint64_t n, int min_one_level,
                           void *dev_root, void *stream);

/* Batched objects already in HBM: dev_objs[i] (device pointers, host array) of lens[i] bytes.
 * Writes nobj x 32 bytes of roots to dev_roots. */
int dm_root_batch_device_async(dm_ctx *ctx, const void *const *dev_objs, const uint64_t *lens,
                               uint64_t nobj, uint64_t chunk, void *dev_roots, void *stream);

/* Synthetic object bytes: word[i] = splitmix64(seed ^ i) over bytes [off, off+nbytes) of the
 * object stream, written to dev (off and nbytes multiples of 8). */
int dm_fill_synthetic_async(dm_ctx *ctx, void *dev, uint64_t off, uint64_t nbytes, uint64_t seed,
                            void *stream);

/* HBM read-bandwidth probe (measurement utility, not on the reference path): XOR of every 8-byte
 * little-endian word of dev[0, nbytes) into *dev_xor8 (device memory, zeroed by the call), one
 * streaming pass.  bench.py times it to report the measured read peak beside the 8 TB/s spec
 * (SURVEY.md 8d).  dev 16-byte aligned, nbytes a multiple of 16. */
int dm_read_probe_async(dm_ctx *ctx, const void *dev, uint64_t nbytes, void *dev_xor8, void *stream);

/* ---- Reed-Solomon fragment coding ------------------------------------------
 * The stage after hashing on DeOSS's upload path: cess-go-sdk codes every 32 MiB segment into
 * chain.DataShards = 4 data + chain.ParShards = 8 parity fragments (node/tracker.go:250,369,
 * node/fileHandler.go:250) with github.com/klauspost/reedsolomon v1.12.4 (go.mod:65).  These
 * entry points replace that Encoder (default options: GF(2^8) mod 0x11d, Vandermonde-derived
 * systematic matrix).  Coding runs on the GPU (rs_code_kernel); results are byte-identical to
 * the restated algorithm (oracle/rs_oracle.c). */
typedef struct dm_rs dm_rs;
/* reedsolomon.New(data_shards, parity_shards): 1 <= data <= 8, 1 <= parity <= 8. */
int dm_rs_create(dm_ctx *ctx, int data_shards, int parity_shards, dm_rs **out);
void dm_rs_destroy(dm_rs *rs);
/* The (data + parity) x data encoding matrix, row-major (top data rows = identity). */
int dm_rs_matrix(dm_rs *rs, uint8_t *out);
/* Encoder.Encode over host shards: data[j] (j < data) -> parity[i] (i < parity), shard bytes each. */
int dm_rs_encode(dm_rs *rs, const void *const *data, void *const *parity, uint64_t shard);
/* Encoder.Split + Encode of one segment: len bytes -> (data + parity) shards of *per_shard =
 * ceil(len / data) bytes, written back to back to out (the last data shard zero-padded). */
int dm_rs_encode_buffer(dm_rs *rs, const void *host, uint64_t len, void *out, uint64_t *per_shard);
/* Encoder.Reconstruct over host shards: rebuilds every shard with present[i] == 0 in place
 * (needs >= data present; fewer -> DM_ERR_INVALID "too few shards"). */
int dm_rs_reconstruct(dm_rs *rs, void *const *shards, const uint8_t *present, uint64_t shard);
/* Encoder.Verify: *ok = 1 when the parity shards match the data shards. */
int dm_rs_verify(dm_rs *rs, const void *const *shards, uint64_t shard, int *ok);
/* Device-resident segments (the measured path): segment s has data shard j at
 * data + s*data_stride + j*shard and gets parity shard i at parity + s*parity_stride + i*shard.
 * shard, strides and pointers 16-byte aligned; runs on `stream` (NULL = null stream). */
int dm_rs_encode_device_async(dm_rs *rs, const void *data, uint64_t data_stride, void *parity,
                              uint64_t parity_stride, uint64_t shard, uint64_t nseg, void *stream);
/* Reconstruct with device shards (16-byte aligned, shard % 16 == 0), in place, on `stream`. */
int dm_rs_reconstruct_device_async(dm_rs *rs, void *const *shards, const uint8_t *present, uint64_t shard,
                                   void *stream);

/* ---- FullProcessing: segments -> fragments -> names -> fid -----------------
 * Replaces cess-go-sdk process.FullProcessing(file, cipher = "", savedir) (go.mod:8; called at
 * node/fileHandler.go:771, node/objectHandler.go:168, node/filesHandler.go:201,
 * node/resumeHandler.go:326, node/tracker.go:767-769, node/fileHandler.go:964,997).  The object is
 * cut into `segment`-byte segments (chain.SegmentSize = 32 MiB; the last one zero-padded); each
 * segment is coded by `rs` (klauspost Split + Encode: rs data shards = the segment in order, then
 * the parity shards, `segment / data` bytes each = chain.FragmentSize); every segment and fragment
 * is named by its SHA-256 (its file name in savedir is the hex digest); the fid is the
 * common/hashtree root over the segments (NewHashTree(segmentPaths), types.go:19-39).  Coding,
 * hashing and the tree all run on the GPU.  Empty object -> DM_ERR_EMPTY.  The cipher branch
 * (AES before coding) is not implemented. */

/* Device-resident form on rs's context.  dev_obj holds len bytes with room for nseg * segment
 * (nseg = ceil(len / segment)); the padding [len, nseg * segment) is zeroed in place.  segment must
 * be a multiple of 16 * data shards; dev_obj, dev_parity 16-byte aligned.  Writes
 *   dev_parity       nseg x parity x frag bytes (segment s, parity fragment i at (s*parity + i)*frag)
 *   dev_seg_hashes   nseg x 32 (nullable)
 *   dev_frag_hashes  nseg x (data + parity) x 32, data fragments first (nullable)
 *   dev_fid          32 bytes
 * in stream order on `stream`. */
int dm_process_device_async(dm_rs *rs, void *dev_obj, uint64_t len, uint64_t segment, void *dev_parity,
                            void *dev_seg_hashes, void *dev_frag_hashes, void *dev_fid, void *stream);
/* Host form (synchronous).  frags_out (nullable) receives nseg x (data + parity) x frag bytes,
 * segment-major, data fragments first (the zero-padded segment bytes).  seg_hashes nseg x 32 and
 * frag_hashes nseg x (data + parity) x 32 are nullable; fid is required. */
int dm_process_buffer(dm_rs *rs, const void *host, uint64_t len, uint64_t segment, void *frags_out,
                      uint8_t *seg_hashes, uint8_t *frag_hashes, uint8_t fid[32]);
/* Many objects in one pass (the batch upload PUT /files, node/filesHandler.go:197-288, runs
 * FullProcessing per file): every segment of every object in one RS launch and one leaf launch.
 * Per-object outputs as in dm_process_buffer (frags_out, seg_hashes, frag_hashes: arrays of nobj
 * pointers, the arrays or their entries nullable); fids: nobj x 32 bytes. */
int dm_process_batch(dm_rs *rs, const void *const *objs, const uint64_t *lens, uint64_t nobj, uint64_t segment,
                     void *const *frags_out, uint8_t *const *seg_hashes, uint8_t *const *frag_hashes, uint8_t *fids);
/* The whole of FullProcessing(file, "", savedir) in one call, from the file path (synchronous):
 * the file is pread into pinned slots and copied to HBM while its data fragments are written out;
 * one RS launch and one leaf launch per window of segments (32 GiB of file per window); the
 * parity fragments come back and are written while the leaf kernel runs; every file is written
 * under a temporary name in savedir and renamed to savedir/<hex SHA-256> once its digest exists.
 * With DM_FP_SEGMENT_FILES the zero-padded segments are written too (savedir/<hex segment digest>,
 * = its data fragments in order).  Outputs: seg_hashes nseg x 32 and frag_hashes nseg x (data +
 * parity) x 32 (data fragments first; both nullable), fid.  cap = capacity of those arrays in
 * segments; *nseg_out (nullable) = the file's segment count, also set when cap is too small
 * (DM_ERR_INVALID).  Errors keep Go's messages ("open <path>: no such file or directory"); an
 * empty file is DM_ERR_EMPTY "Empty data"; on failure no temporary file is left behind. */
#define DM_FP_SEGMENT_FILES 1
int dm_full_processing(dm_rs *rs, const char *path, const char *savedir, uint64_t segment, int flags,
                       uint8_t *seg_hashes, uint8_t *frag_hashes, uint64_t cap, uint64_t *nseg_out, uint8_t fid[32]);
/* The fragment download path (node/fileHandler.go:958-1013) runs FullProcessing(fpath, "", cacheDir)
 * over a locally held object only to serve the ONE fragment whose name (hex SHA-256) was asked for.
 * This finds it without writing anything: the file is read window by window (double-buffered with
 * the GPU), segments are RS-coded and every fragment hashed on the device (no segment hashes, no
 * fid, no files), and the scan stops at the first window holding `want`.  *found = 1 with the
 * fragment's (segment, index) (data fragments 0 .. data-1, then parity) and, when out != NULL, its
 * segment/data bytes in out (out_cap >= that); *found = 0 when no fragment has that name.  The
 * first match in (segment, index) order wins, as the handler's scan.  Errors as dm_full_processing
 * ("open <path>: ...", "Empty data"). */
int dm_fragment_lookup(dm_rs *rs, const char *path, uint64_t segment, const uint8_t want[32], void *out,
                       uint64_t out_cap, int *found, uint64_t *seg_idx, int *frag_idx);

/* FullProcessing while the upload body arrives (SURVEY.md 8f #1 + #2): the handlers write the body
 * to a file (node/objectHandler.go:248-266, node/fileHandler.go:899-937) and then run
 * FullProcessing(fpath, "", cacheDir) over it (node/objectHandler.go:168, node/fileHandler.go:771).
 * A pstream takes the body in pieces of any size beside that file write: whole segments are
 * copied to HBM, coded and their fragment files written as they arrive, segments are hashed in
 * batches on the GPU meanwhile; close pads the last segment, finishes, and returns the same
 * digests / fid / files as dm_full_processing on the same bytes (flags: DM_FP_SEGMENT_FILES).
 * Not thread-safe per stream; separate streams (on one rs) may run concurrently.  close and abort
 * free the stream; on any failure no temporary file is left in savedir. */
typedef struct dm_pstream dm_pstream;
int dm_pstream_open(dm_rs *rs, uint64_t segment, const char *savedir, int flags, dm_pstream **out);
int dm_pstream_write(dm_pstream *st, const void *data, uint64_t len);
int dm_pstream_close(dm_pstream *st, uint8_t *seg_hashes, uint8_t *frag_hashes, uint64_t cap, uint64_t *nseg_out,
                     uint8_t fid[32]);
void dm_pstream_abort(dm_pstream *st);
/* Device memory of a pstream: chunk buffers (segments + parity, 3x the body at 4 + 8) allocated now
 * (in use or kept for reuse) and the most ever allocated.  A chunk's buffer is reused once its
 * parity is written out and the leaf launch that hashed it has finished; at the cap
 * (env DEOSS_PS_DEVICE_CAP, default 16 GiB) write blocks until the oldest one is free, so a
 * stream's HBM does not grow with the body. */
int dm_pstream_stats(dm_pstream *st, uint64_t *device_bytes, uint64_t *peak_device_bytes);

/* ---- Merkle tree levels and proofs ----------------------------------------
 * cbergoon/merkletree v0.2.0 (go.mod:10) keeps every node of the tree NewHashTree returns
 * (common/hashtree/types.go:38) for GetMerklePath, VerifyContent and VerifyTree.  Here the nodes
 * live level-major: level 1 (ceil(n/2) nodes), level 2, ..., the root last, 32 bytes each
 * (dm_tree_node_count(n) nodes); the n leaf digests are level 0.  Every leaf's path has
 * dm_tree_depth(n) = max(1, ceil(log2 n)) steps.  Path bits follow GetMerklePath: 1 = the sibling
 * is the right child (taken whenever the left child's digest equals the current node's, as the
 * reference compares hashes), 0 = the sibling is the left child. */
uint64_t dm_tree_node_count(uint64_t n);
uint32_t dm_tree_depth(uint64_t n);
/* All levels over n leaf digests (device, stream-ordered / host, synchronous). */
int dm_tree_levels_device_async(dm_ctx *ctx, const void *dev_leaves, uint64_t n, void *dev_nodes, void *stream);
int dm_tree_levels(dm_ctx *ctx, const uint8_t *leaf_digests, uint64_t n, uint8_t *nodes_out);
/* GetMerklePath for q leaf indices (uint64): paths q x depth x 32 bytes, bits q x depth bytes.
 * An index >= n yields zero digests and bits 0xff.  Device form reads nodes from
 * dm_tree_levels_device_async; host form builds the levels itself. */
int dm_merkle_paths_device_async(dm_ctx *ctx, const void *dev_leaves, const void *dev_nodes, uint64_t n,
                                 const void *dev_idx, uint64_t q, void *dev_paths, void *dev_bits, void *stream);
int dm_merkle_paths(dm_ctx *ctx, const uint8_t *leaf_digests, uint64_t n, const uint64_t *idx, uint64_t q,
                    uint8_t *paths, uint8_t *bits);
/* Verify q proofs: ok[t] = 1 when SHA-256(content t) folded with path t (depth steps, bits as
 * above) equals root t.  Roots advance root_stride bytes per proof (0: one shared root; host form:
 * 0 or 32).  Contents are device pointers (host array) / host chunks. */
int dm_verify_paths_device_async(dm_ctx *ctx, const void *const *dev_contents, const uint64_t *lens, uint64_t q,
                                 const void *dev_paths, const void *dev_bits, uint32_t depth, const void *dev_roots,
                                 uint64_t root_stride, void *dev_ok, void *stream);
/* Uniform form: the ceil(len / chunk) chunks of one object in HBM (chunk i at dev_obj + i * chunk,
 * the last one short) checked against proofs t = 0 .. n-1 -- no per-content table. */
int dm_verify_object_device_async(dm_ctx *ctx, const void *dev_obj, uint64_t len, uint64_t chunk,
                                  const void *dev_paths, const void *dev_bits, uint32_t depth, const void *dev_roots,
                                  uint64_t root_stride, void *dev_ok, void *stream);
int dm_verify_paths(dm_ctx *ctx, const void *const *contents, const uint64_t *lens, uint64_t q, const uint8_t *paths,
                    const uint8_t *bits, uint32_t depth, const uint8_t *roots, uint64_t root_stride, uint8_t *ok);

/* ---- coalescing executor for concurrent callers ------------------------------------------------
 * Upload handlers run one goroutine per request, each hashing / processing its own object.  A
 * dm_batcher takes blocking calls from any number of threads and turns whatever is queued into
 * one batched GPU pass (one leaf launch over every request's leaves, one tree per request), on
 * `slots` worker contexts so one batch collects while another runs.  Results are identical to
 * the single-object calls (dm_root_buffer / dm_process_buffer). */
typedef struct dm_batcher dm_batcher;
enum { DM_BATCH_ROOT = 0, DM_BATCH_PROCESS = 1 };
/* devs / ndev: GPUs to serve from (devs NULL: every visible GPU); objects are independent, so
 * requests spread over the GPUs with no exchange.  mode ROOT: unit = chunk size (each request:
 * NewHashTreeFromBuffer); PROCESS: unit = segment size with data/parity shards (each request:
 * FullProcessing).  slots (0 = 4) worker contexts per GPU; max_leaves / max_bytes per batch
 * (0 = 4096 leaves / 16 GiB); linger_us: how long a free worker holds a burst open for more
 * requests, counted from the oldest queued request's arrival (0 = at once).  While other slots
 * are running batches the wait grows with their share (the last free slot of 4 waits 9/256 of
 * the longest queued request's chain more: 17 ms for a 32 MiB segment), so a burst that starts
 * during a running batch is not cut into one small batch per free slot; a full batch's worth of
 * leaves queued, or an oldest request that has already waited that long, launches at once. */
int dm_batcher_create(const int *devs, int ndev, int mode, uint64_t unit, int data_shards, int parity_shards,
                      int slots, uint64_t max_leaves, uint64_t max_bytes, uint32_t linger_us, dm_batcher **out);
/* Drains queued requests, then frees the workers and their contexts. */
void dm_batcher_destroy(dm_batcher *b);
/* Blocking, thread-safe.  Same outputs as dm_root_buffer (leaf_out nullable) / dm_process_buffer. */
int dm_batcher_root(dm_batcher *b, const void *host, uint64_t len, uint8_t *leaf_out, uint8_t root[32]);
int dm_batcher_process(dm_batcher *b, const void *host, uint64_t len, void *frags_out, uint8_t *seg_hashes,
                       uint8_t *frag_hashes, uint8_t fid[32]);
/* Requests served, batches launched, largest batch (requests). */
int dm_batcher_stats(dm_batcher *b, uint64_t *requests, uint64_t *batches, uint64_t *max_batch);
/* Message of the calling thread's last failing dm_batcher_* call. */
const char *dm_batcher_last_error(void);

/* ---- multi-device plan (pure host functions: no GPU, no context) ---------------------------
 * The partition and routing rules the library applies (deoss_amd/csrc/shard_plan.hpp), exported so
 * the one-process-per-GPU path (deoss_amd/sharding.py) and the tests use the same rule. */
enum { DM_SRC_DEVICE = 0, DM_SRC_HOST_PINNED = 1, DM_SRC_HOST_PAGEABLE = 2, DM_SRC_FILES = 3 };
/* Partition of nleaves leaves over ndev devices: blocks of 2^levels leaves (*levels), *nblocks
 * blocks (= the level-`levels` nodes of the global tree), device g owns leaves [leaf_lo[g],
 * leaf_hi[g]) (arrays of ndev entries, nullable). */
int dm_plan_shards(uint64_t nleaves, int ndev, uint32_t *levels, uint64_t *nblocks, uint64_t *leaf_lo,
                   uint64_t *leaf_hi);
/* Devices a call should use (1 = whole call on one device) for nleaves leaves, `bytes` in total,
 * the longest leaf leaf_max bytes, starting at `source` (DM_SRC_*), split by objects (by_objects != 0,
 * a batch) or as one tree, with ndev devices of `cus` compute units, leaf-kernel mode leaf_mode
 * (DM_LEAF_*) and `busy` calls already in flight.  est_ms (nullable, ndev entries): the cost
 * model's time for 1 .. ndev devices. */
int dm_plan_route(uint64_t nleaves, uint64_t bytes, uint64_t leaf_max, int source, int by_objects, int ndev, int cus,
                  int leaf_mode, int busy, double *est_ms);
/* The cost model's two terms that only a multi-GPU node can measure: the all-gather of the
 * 32-byte subtree roots (default 100 us) and the host memory bandwidth every device's feed shares
 * (default 500e9 B/s).  Environment variables DEOSS_ALLGATHER_US and DEOSS_HOST_BYTES_PER_S
 * (positive numbers; the N = 8 bench line prints the measured values as route_constants) replace
 * them: read once by dm_create for its context, and per call by dm_plan_route.  The values a
 * context uses (ctx NULL: what dm_plan_route would use now); either pointer nullable.  0. */
int dm_route_constants(dm_ctx *ctx, double *allgather_us, double *host_bytes_per_s);

/* ---- tuning ------------------------------------------------------------------------------ */

/* Leaf-kernel selection for uniform-chunk objects (results are identical in every mode):
 * DM_LEAF_AUTO picks by leaf count; DM_LEAF_WIDE = one lane per leaf (K1, throughput regime);
 * DM_LEAF_LATENCY = producer/consumer waves per 64 leaves (K1L, few long leaves);
 * DM_LEAF_PAIR = K1L with each leaf's rounds packed on two lanes (K1P);
 * DM_LEAF_QUAD = each leaf's rounds spread over eight lanes (K1Q, fewest leaves). */
enum { DM_LEAF_AUTO = 0, DM_LEAF_WIDE = 1, DM_LEAF_LATENCY = 2, DM_LEAF_PAIR = 3, DM_LEAF_QUAD = 4 };
int dm_set_leaf_kernel(dm_ctx *ctx, int mode);
/* The leaf kernel (DM_LEAF_WIDE / _LATENCY / _PAIR / _QUAD) a uniform-chunk object of nleaves leaves
 * runs with under the current setting. */
int dm_leaf_kernel_for(dm_ctx *ctx, uint64_t nleaves);

/* ---- measurement ------------------------------------------------------------------------- */

/* Enable (and reset) HIP-event timing: every later call that launches the leaf kernel (K1)
 * records events on its launch stream around K1 and around the whole call, with no host sync. */
int dm_set_timing(dm_ctx *ctx, int enable);
/* Waits for the recorded events and returns: number of timed calls, sum of K1 durations (ms),
 * sum of whole-call durations (ms), longest K1 duration (ms). */
int dm_timing_summary(dm_ctx *ctx, uint64_t *ncalls, double *leaf_ms_sum, double *total_ms_sum,
                      double *leaf_ms_max);
/* Subtree-root exchanges (C1) of sharded calls since dm_set_timing(ctx, 1): their number, the sum
 * and maximum of their durations in microseconds (host clock, from every device's level-k nodes
 * being ready to the gathered slots being on every device: the ncclAllGather over G GPUs; while
 * timing is on the call waits for the subtree roots before the gather) and the G of the last one. */
int dm_exchange_timing(dm_ctx *ctx, uint64_t *n, double *us_sum, double *us_max, int *last_ndev);
/* Where the calling thread's last call on ctx ran (any entry point that holds a lane): the context
 * device indices (devs: one for a whole call, 0 .. G-1 for a call sharded over G GPUs) and their
 * HIP device ids (hip_ids), at most cap entries each (both nullable), and the lane within the GPU
 * (*lane, nullable; -1 when this thread has made no call on ctx).  Returns the device count, 0 when
 * there was no call.  Lets a gateway log which GPU served an upload. */
int dm_last_call_devices(dm_ctx *ctx, int *devs, int *hip_ids, int cap, int *lane);

#ifdef __cplusplus
}
#endif
#endif /* DEOSS_MERKLE_H */
