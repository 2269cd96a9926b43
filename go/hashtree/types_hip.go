//go:build hip

// Drop-in replacement for DeOSS common/hashtree/types.go (reference lines 19-39): the same
// NewHashTree signature and errors, with leaf hashing and the root on the GPU through the
// C ABI in include/deoss_merkle.h.
package hashtree

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../deoss_amd -ldeoss_merkle -Wl,-rpath,${SRCDIR}/../../deoss_amd
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"bytes"
	"errors"
	"fmt"
	"sync"
	"unsafe"

	"github.com/cbergoon/merkletree"
)

var (
	ctxOnce sync.Once
	ctx     *C.dm_ctx
	ctxErr  error
)

func gpu() (*C.dm_ctx, error) {
	ctxOnce.Do(func() {
		if rc := C.dm_create(&ctx, nil, 0); rc != C.DM_OK {
			ctxErr = errors.New(C.GoString(C.dm_strerror(rc)))
		}
	})
	return ctx, ctxErr
}

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
	rc := C.dm_new_hash_tree(c, (**C.char)(unsafe.Pointer(&cpaths[0])), C.uint64_t(len(chunkPath)),
		(*C.uint8_t)(unsafe.Pointer(&leaves[0])), (*C.uint8_t)(unsafe.Pointer(&root[0])))
	if rc != C.DM_OK {
		return nil, rcError(c, rc)
	}
	return buildTree(leaves, root)
}

// NewHashTreeFromBuffer (additive): the upload body already in memory, split into chunkSize
// chunks (the last one short) -- no temp files, one H2D pass.
func NewHashTreeFromBuffer(buf []byte, chunkSize int) (*merkletree.MerkleTree, error) {
	if len(buf) == 0 {
		return nil, errors.New("Empty data")
	}
	c, err := gpu()
	if err != nil {
		return nil, err
	}
	n := (len(buf) + chunkSize - 1) / chunkSize
	leaves := make([]byte, 32*n)
	root := make([]byte, 32)
	rc := C.dm_root_buffer(c, unsafe.Pointer(&buf[0]), C.uint64_t(len(buf)), C.uint64_t(chunkSize),
		(*C.uint8_t)(unsafe.Pointer(&leaves[0])), (*C.uint8_t)(unsafe.Pointer(&root[0])))
	if rc != C.DM_OK {
		return nil, rcError(c, rc)
	}
	return buildTree(leaves, root)
}
