//go:build hip

// Page-locked host buffers for the zero-copy host path (DESIGN.md §5).  An upload handler that
// reads the request body into a PinnedBuffer and hashes that slice with NewHashTreeFromBuffer
// has the body hashed in place: the leaf kernel reads it over PCIe, with no H2D copy and no
// HBM copy of the object.
package hashtree

/*
#include "deoss_merkle.h"
*/
import "C"

import (
	"errors"
	"runtime"
	"unsafe"

	"github.com/cbergoon/merkletree"
)

// PinnedBuffer is page-locked host memory (dm_host_alloc) that every GPU can read.  Bytes()
// aliases that C memory.  There is no finalizer: the memory lives until Free, so a Bytes() slice
// stays valid exactly as long as the caller has not called Free -- pool the *PinnedBuffer (not
// just its slice) and Free it when the pool drops it.  NewHashTreeFromPinned keeps the buffer
// reachable for the whole call.
type PinnedBuffer struct {
	p unsafe.Pointer
	n int
}

// NewPinnedBuffer allocates n bytes of page-locked host memory; release it with Free.
func NewPinnedBuffer(n int) (*PinnedBuffer, error) {
	if n <= 0 {
		return nil, errors.New("hashtree: pinned buffer size must be positive")
	}
	runtime.LockOSThread() // dm_last_error is thread-local
	defer runtime.UnlockOSThread()
	var p unsafe.Pointer
	if rc := C.dm_host_alloc(C.uint64_t(n), &p); rc != C.DM_OK {
		return nil, errors.New(C.GoString(C.dm_last_error(nil)))
	}
	return &PinnedBuffer{p: p, n: n}, nil
}

// Bytes is the whole buffer as a Go slice over the pinned memory (nil after Free).
func (b *PinnedBuffer) Bytes() []byte {
	if b.p == nil {
		return nil
	}
	return unsafe.Slice((*byte)(b.p), b.n)
}

// Free releases the memory; Bytes() slices taken earlier become invalid.  Free is idempotent.
func (b *PinnedBuffer) Free() {
	if b.p != nil {
		C.dm_host_free(b.p)
		b.p = nil
	}
}

// NewHashTreeFromPinned hashes the first n bytes of pb (the zero-copy path: the leaf kernel reads
// them in place over PCIe).  pb stays reachable until the call returns.
func NewHashTreeFromPinned(pb *PinnedBuffer, n int, chunkSize int) (*merkletree.MerkleTree, error) {
	if pb == nil || pb.p == nil {
		return nil, errors.New("hashtree: pinned buffer is nil or freed")
	}
	if n < 0 || n > pb.n {
		return nil, errors.New("hashtree: length outside the pinned buffer")
	}
	t, err := NewHashTreeFromBuffer(pb.Bytes()[:n], chunkSize)
	runtime.KeepAlive(pb)
	return t, err
}
