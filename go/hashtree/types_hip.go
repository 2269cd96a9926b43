//go:build hip

// Drop-in replacement for DeOSS common/hashtree/types.go (reference lines 19-39): the same
// NewHashTree signature and errors, with leaf hashing and the root on the GPU through the
// C ABI in include/deoss_merkle.h.  One process-wide context spans every GPU chosen by Init or
// DEOSS_GPUS (default: all visible GPUs).  Each call runs whole on the least-loaded GPU, so
// concurrent handlers spread over the node (8 concurrent NewHashTree calls over 256 x 32 MiB
// segment files: one GPU each, ~0.5 s together), on one of the GPU's DEOSS_LANES call lanes
// (4 on an MI355X: four large calls share a GPU side by side); a call is sharded by aligned chunk ranges with
// one RCCL all-gather of subtree roots only when the library's cost model says it finishes sooner
// and no other call is in flight (e.g. a 1 TiB object, or 1 MiB chunks bound by one PCIe link;
// DESIGN.md §7).  Build: CGO_ENABLED=1, -tags hip, PKG_CONFIG_PATH=<checkout>/deoss_amd.
package hashtree

/*
#cgo pkg-config: deoss_merkle
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"bytes"
	"errors"
	"fmt"
	"os"
	"runtime"
	"strconv"
	"strings"
	"sync"
	"unsafe"

	"github.com/cbergoon/merkletree"
)

var (
	ctxMu  sync.Mutex
	ctx    *C.dm_ctx
	ctxErr error
	devSel []int // nil: DEOSS_GPUS, else every visible GPU
)

// Init selects the GPUs (HIP device ids) the package's context spans.  It must run before the
// first NewHashTree / NewHashTreeFromBuffer / NewStream call; later calls return an error.
// Without Init the context uses DEOSS_GPUS ("0,1,2,3" or "all"), else every visible GPU.
func Init(devs []int) error {
	ctxMu.Lock()
	defer ctxMu.Unlock()
	if ctx != nil || ctxErr != nil {
		return errors.New("hashtree: Init after first use")
	}
	if len(devs) == 0 {
		return errors.New("hashtree: Init needs at least one device")
	}
	devSel = append([]int(nil), devs...)
	return nil
}

func deviceList() ([]int, error) {
	if devSel != nil {
		return devSel, nil
	}
	spec := strings.TrimSpace(os.Getenv("DEOSS_GPUS"))
	if spec != "" && spec != "all" {
		var out []int
		for _, f := range strings.Split(spec, ",") {
			d, err := strconv.Atoi(strings.TrimSpace(f))
			if err != nil || d < 0 {
				return nil, fmt.Errorf("hashtree: bad DEOSS_GPUS entry %q", f)
			}
			out = append(out, d)
		}
		return out, nil
	}
	n := int(C.dm_gpu_count())
	if n <= 0 {
		return nil, errors.New(C.GoString(C.dm_strerror(C.DM_ERR_NODEV)))
	}
	out := make([]int, n)
	for i := range out {
		out[i] = i
	}
	return out, nil
}

func gpu() (*C.dm_ctx, error) {
	ctxMu.Lock()
	defer ctxMu.Unlock()
	if ctx != nil || ctxErr != nil {
		return ctx, ctxErr
	}
	devs, err := deviceList()
	if err != nil {
		ctxErr = err
		return nil, err
	}
	cdevs := make([]C.int, len(devs))
	for i, d := range devs {
		cdevs[i] = C.int(d)
	}
	if rc := C.dm_create(&ctx, &cdevs[0], C.int(len(cdevs))); rc != C.DM_OK {
		ctx = nil
		ctxErr = errors.New(C.GoString(C.dm_strerror(rc)))
	}
	return ctx, ctxErr
}

// Sharding reports whether the package's context can shard one object over its GPUs: more than
// one GPU and RCCL communicators up.  A node whose RCCL init failed still hashes, every call whole
// on one GPU (dm_can_shard; the library says so once on stderr).
func Sharding() (bool, error) {
	c, err := gpu()
	if err != nil {
		return false, err
	}
	return C.dm_can_shard(c) == 1, nil
}

// rcError reads the library's thread-local message of the failing call: the caller holds
// runtime.LockOSThread from the call until here.
func rcError(c *C.dm_ctx, rc C.int) error {
	if rc == C.DM_ERR_EMPTY {
		return errors.New("Empty data") // types.go:21
	}
	if msg := C.GoString(C.dm_last_error(c)); msg != "" {
		return errors.New(msg) // e.g. "open <path>: no such file or directory"
	}
	return errors.New(C.GoString(C.dm_strerror(rc)))
}

// buildTree rebuilds the *merkletree.MerkleTree (merkleRoot is unexported) over contents that
// carry the GPU leaf digests: merkletree re-hashes only the n-1 64-byte interior nodes, and the
// result must equal the GPU root.
func buildTree(leaves []byte, root []byte) (*merkletree.MerkleTree, error) {
	n := len(leaves) / 32
	list := make([]merkletree.Content, n)
	for i := 0; i < n; i++ {
		list[i] = HashTreeContent{digest: leaves[32*i : 32*i+32]}
	}
	t, err := merkletree.NewTree(list)
	if err != nil {
		return nil, err
	}
	if !bytes.Equal(t.MerkleRoot(), root) {
		return nil, fmt.Errorf("hashtree: GPU root %x != tree root %x", root, t.MerkleRoot())
	}
	return t, nil
}

// NewHashTree build file to build hash tree
func NewHashTree(chunkPath []string) (*merkletree.MerkleTree, error) {
	if len(chunkPath) == 0 {
		return nil, errors.New("Empty data")
	}
	c, err := gpu()
	if err != nil {
		return nil, err
	}
	cpaths := make([]*C.char, len(chunkPath))
	for i, p := range chunkPath {
		cpaths[i] = C.CString(p)
	}
	defer func() {
		for _, p := range cpaths {
			C.free(unsafe.Pointer(p))
		}
	}()
	leaves := make([]byte, 32*len(chunkPath))
	root := make([]byte, 32)
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	rc := C.dm_new_hash_tree(c, (**C.char)(unsafe.Pointer(&cpaths[0])), C.uint64_t(len(chunkPath)),
		(*C.uint8_t)(unsafe.Pointer(&leaves[0])), (*C.uint8_t)(unsafe.Pointer(&root[0])))
	if rc != C.DM_OK {
		return nil, rcError(c, rc)
	}
	return buildTree(leaves, root)
}

// BatchLimit: NewHashTreeFromBuffer objects up to this size go through a process-wide coalescing
// dm_batcher per chunk size, so concurrent handler goroutines share GPU passes instead of
// queueing one chain-latency pass each on the context (DESIGN.md §6.9: 131x for 256 concurrent
// 1 MiB uploads).  Larger objects take dm_root_buffer: ramped striped H2D overlapped with
// hashing, zero-copy from pinned memory, on the least-loaded GPU (or sharded, see above).
const BatchLimit = 256 << 20

// MaxBatchers bounds the batchers (each owns 4 worker contexts per GPU): the first MaxBatchers
// distinct chunk sizes get one; calls with any other chunk size take dm_root_buffer.  DeOSS uses
// one chunk size (chain.SegmentSize).
const MaxBatchers = 4

var (
	batchMu  sync.Mutex
	batchers = map[int]*C.dm_batcher{}
)

// batcherFor returns the chunk size's batcher, or nil when MaxBatchers other sizes hold one.
func batcherFor(chunk int) (*C.dm_batcher, error) {
	if _, err := gpu(); err != nil { // fixes the device list
		return nil, err
	}
	batchMu.Lock()
	defer batchMu.Unlock()
	if b, ok := batchers[chunk]; ok {
		return b, nil
	}
	if len(batchers) >= MaxBatchers {
		return nil, nil
	}
	devs, err := deviceList()
	if err != nil {
		return nil, err
	}
	cdevs := make([]C.int, len(devs))
	for i, d := range devs {
		cdevs[i] = C.int(d)
	}
	runtime.LockOSThread() // dm_batcher_last_error is thread-local
	defer runtime.UnlockOSThread()
	var b *C.dm_batcher
	// 4 worker slots per GPU (the library default), 4,096 leaves per batch, 2 ms linger
	if rc := C.dm_batcher_create(&cdevs[0], C.int(len(cdevs)), C.DM_BATCH_ROOT, C.uint64_t(chunk), 0, 0, 0, 0, 0, 2000,
		&b); rc != C.DM_OK {
		return nil, errors.New(C.GoString(C.dm_batcher_last_error()))
	}
	batchers[chunk] = b
	return b, nil
}

// NewHashTreeFromBuffer (additive): the upload body already in memory, split into chunkSize
// chunks (the last one short) -- no temp files, one H2D pass.
func NewHashTreeFromBuffer(buf []byte, chunkSize int) (*merkletree.MerkleTree, error) {
	if chunkSize <= 0 {
		return nil, fmt.Errorf("hashtree: chunk size %d must be positive", chunkSize)
	}
	if len(buf) == 0 {
		return nil, errors.New("Empty data")
	}
	n := (len(buf) + chunkSize - 1) / chunkSize
	leaves := make([]byte, 32*n)
	root := make([]byte, 32)
	var b *C.dm_batcher
	if len(buf) <= BatchLimit {
		var err error
		if b, err = batcherFor(chunkSize); err != nil {
			return nil, err
		}
	}
	if b != nil {
		runtime.LockOSThread()
		defer runtime.UnlockOSThread()
		rc := C.dm_batcher_root(b, unsafe.Pointer(&buf[0]), C.uint64_t(len(buf)),
			(*C.uint8_t)(unsafe.Pointer(&leaves[0])), (*C.uint8_t)(unsafe.Pointer(&root[0])))
		if rc != C.DM_OK {
			if rc == C.DM_ERR_EMPTY {
				return nil, errors.New("Empty data")
			}
			return nil, errors.New(C.GoString(C.dm_batcher_last_error()))
		}
		return buildTree(leaves, root)
	}
	c, err := gpu()
	if err != nil {
		return nil, err
	}
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	rc := C.dm_root_buffer(c, unsafe.Pointer(&buf[0]), C.uint64_t(len(buf)), C.uint64_t(chunkSize),
		(*C.uint8_t)(unsafe.Pointer(&leaves[0])), (*C.uint8_t)(unsafe.Pointer(&root[0])))
	if rc != C.DM_OK {
		return nil, rcError(c, rc)
	}
	return buildTree(leaves, root)
}
