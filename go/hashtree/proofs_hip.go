//go:build hip

// Batched Merkle proofs on the GPU (SURVEY.md 8f #4).  The *merkletree.MerkleTree NewHashTree
// returns is a genuine merkletree v0.2.0 tree, so its own GetMerklePath / VerifyContent /
// VerifyTree keep working unchanged (on the CPU, as in the reference).  These additive helpers
// serve many leaves per call through include/deoss_merkle.h: GetMerklePaths gathers every
// requested path from the tree levels in HBM (dm_merkle_paths), VerifyProofs re-hashes each
// content and folds its path on the GPU (dm_verify_paths).  Paths and indices use merkletree's
// convention: index 1 = the sibling is the right child.
package hashtree

/*
#include <stdlib.h>
#include "deoss_merkle.h"
*/
import "C"

import (
	"errors"
	"runtime"
	"unsafe"

	"github.com/cbergoon/merkletree"
)

// GetMerklePaths returns GetMerklePath's (path, index) for each leaf position of t.
func GetMerklePaths(t *merkletree.MerkleTree, leaves []int) ([][][]byte, [][]int64, error) {
	c, err := gpu()
	if err != nil {
		return nil, nil, err
	}
	// All of t.Leafs, merkletree's duplicated last leaf included: the level rule over n+1 leaves
	// whose last two are equal is the same tree (same nodes, depth and paths) as over n.
	var digests []byte
	for _, l := range t.Leafs {
		digests = append(digests, l.Hash...)
	}
	n := uint64(len(digests) / 32)
	if n == 0 {
		return nil, nil, errors.New("Empty data")
	}
	if len(leaves) == 0 {
		return nil, nil, nil
	}
	depth := uint64(C.dm_tree_depth(C.uint64_t(n)))
	idx := make([]uint64, len(leaves))
	for i, l := range leaves {
		idx[i] = uint64(l)
	}
	q := uint64(len(leaves))
	paths := make([]byte, 32*depth*q)
	bits := make([]byte, depth*q)
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	rc := C.dm_merkle_paths(c, (*C.uint8_t)(unsafe.Pointer(&digests[0])), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&idx[0])), C.uint64_t(q), (*C.uint8_t)(unsafe.Pointer(&paths[0])),
		(*C.uint8_t)(unsafe.Pointer(&bits[0])))
	if rc != C.DM_OK {
		return nil, nil, rcError(c, rc)
	}
	outP := make([][][]byte, q)
	outI := make([][]int64, q)
	for i := uint64(0); i < q; i++ {
		outP[i] = make([][]byte, depth)
		outI[i] = make([]int64, depth)
		for l := uint64(0); l < depth; l++ {
			o := 32 * (i*depth + l)
			outP[i][l] = append([]byte(nil), paths[o:o+32]...)
			outI[i][l] = int64(bits[i*depth+l])
		}
	}
	return outP, outI, nil
}

// VerifyProofs reports, per proof, whether SHA-256(contents[i]) folded with paths[i] / index[i]
// equals root.
func VerifyProofs(contents [][]byte, paths [][][]byte, index [][]int64, root []byte) ([]bool, error) {
	c, err := gpu()
	if err != nil {
		return nil, err
	}
	q := len(contents)
	if q == 0 {
		return nil, nil
	}
	depth := len(paths[0])
	pb := make([]byte, 0, 32*depth*q)
	bb := make([]byte, 0, depth*q)
	for i := 0; i < q; i++ {
		if len(paths[i]) != depth || len(index[i]) != depth {
			return nil, errors.New("hashtree: every proof needs the same depth")
		}
		for l := 0; l < depth; l++ {
			pb = append(pb, paths[i][l]...)
			bb = append(bb, byte(index[i][l]))
		}
	}
	// contents are copied into C memory: the library reads them after cgo pointer checks apply
	ptrs := C.malloc(C.size_t(q) * C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(ptrs)
	lens := make([]uint64, q)
	cp := (*[1 << 30]unsafe.Pointer)(ptrs)[:q:q]
	for i, b := range contents {
		lens[i] = uint64(len(b))
		if len(b) > 0 {
			cp[i] = C.CBytes(b)
			defer C.free(cp[i])
		} else {
			cp[i] = nil
		}
	}
	ok := make([]byte, q)
	runtime.LockOSThread() // dm_last_error is thread-local: call and read on one OS thread
	defer runtime.UnlockOSThread()
	rc := C.dm_verify_paths(c, (*unsafe.Pointer)(ptrs), (*C.uint64_t)(unsafe.Pointer(&lens[0])), C.uint64_t(q),
		(*C.uint8_t)(unsafe.Pointer(&pb[0])), (*C.uint8_t)(unsafe.Pointer(&bb[0])), C.uint32_t(depth),
		(*C.uint8_t)(unsafe.Pointer(&root[0])), 0, (*C.uint8_t)(unsafe.Pointer(&ok[0])))
	if rc != C.DM_OK {
		return nil, rcError(c, rc)
	}
	res := make([]bool, q)
	for i, v := range ok {
		res[i] = v == 1
	}
	return res, nil
}
