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
)

// PinnedBuffer is page-locked host memory (dm_host_alloc) that every GPU can read.  Bytes()
// aliases that C memory: it must not be used after Free.
type PinnedBuffer struct {
	p unsafe.Pointer
	n int
}

// NewPinnedBuffer allocates n bytes of page-locked host memory.
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
	b := &PinnedBuffer{p: p, n: n}
	runtime.SetFinalizer(b, func(x *PinnedBuffer) { x.Free() })
	return b, nil
}

// Bytes is the whole buffer as a Go slice over the pinned memory.
func (b *PinnedBuffer) Bytes() []byte {
	if b.p == nil {
		return nil
	}
	return unsafe.Slice((*byte)(b.p), b.n)
}

// Free releases the memory; Bytes() slices taken earlier become invalid.
func (b *PinnedBuffer) Free() {
	if b.p != nil {
		C.dm_host_free(b.p)
		b.p = nil
		runtime.SetFinalizer(b, nil)
	}
}
