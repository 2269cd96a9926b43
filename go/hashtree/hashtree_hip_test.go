//go:build hip

package hashtree

import (
	"crypto/sha256"
	"encoding/hex"
	"os"
	"path/filepath"
	"sync"
	"testing"

	"github.com/cbergoon/merkletree"
	"github.com/stretchr/testify/assert"
)

// Same assertions as the reference common/hashtree/hashtree_test.go:20-82, through the GPU.
func TestNewHashTreeGPU(t *testing.T) {
	contents := []string{"content_one", "content_two", "content_three", "content_four"}
	var hashes [][32]byte
	dir := t.TempDir()
	var chunks []string
	for _, c := range contents {
		hashes = append(hashes, sha256.Sum256([]byte(c)))
		p := filepath.Join(dir, c)
		assert.NoError(t, os.WriteFile(p, []byte(c), 0o644))
		chunks = append(chunks, p)
	}
	five := sha256.Sum256(append(hashes[0][:], hashes[1][:]...))
	six := sha256.Sum256(append(hashes[2][:], hashes[3][:]...))
	root := sha256.Sum256(append(five[:], six[:]...))

	mtree, err := NewHashTree(chunks)
	assert.NoError(t, err)
	assert.Equal(t, 4, len(mtree.Leafs))
	for i := range contents {
		assert.Equal(t, hex.EncodeToString(hashes[i][:]), hex.EncodeToString(mtree.Leafs[i].Hash))
	}
	assert.Equal(t, "b513419286835c1e36fa520b86cbf37650db82e73f510f0e6a699cc0505f1151", hex.EncodeToString(mtree.MerkleRoot()))
	assert.Equal(t, hex.EncodeToString(root[:]), hex.EncodeToString(mtree.MerkleRoot()))

	_, err = NewHashTree(nil)
	assert.EqualError(t, err, "Empty data")
}

// NewHashTreeFromBuffer rejects a non-positive chunk size with an error (no panic).
func TestFromBufferChunkSize(t *testing.T) {
	_, err := NewHashTreeFromBuffer([]byte("abc"), 0)
	assert.Error(t, err)
	_, err = NewHashTreeFromBuffer([]byte("abc"), -5)
	assert.Error(t, err)
}

// A Stream fed in uneven pieces builds the same tree as NewHashTreeFromBuffer over the whole body.
func TestStreamGPU(t *testing.T) {
	body := make([]byte, 9<<20+123)
	for i := range body {
		body[i] = byte(i*131 + i>>9)
	}
	want, err := NewHashTreeFromBuffer(body, 1<<20)
	assert.NoError(t, err)
	hs, err := NewStream(1 << 20)
	assert.NoError(t, err)
	for pos, step := 0, 1; pos < len(body); step = step*7%1000003 + 1 {
		n := min(step, len(body)-pos)
		w, err := hs.Write(body[pos : pos+n])
		assert.NoError(t, err)
		assert.Equal(t, n, w)
		pos += n
	}
	got, err := hs.Close()
	assert.NoError(t, err)
	assert.Equal(t, want.MerkleRoot(), got.MerkleRoot())
	assert.Equal(t, len(want.Leafs), len(got.Leafs))

	empty, err := NewStream(1 << 20)
	assert.NoError(t, err)
	_, err = empty.Close()
	assert.EqualError(t, err, "Empty data")

	aborted, err := NewStream(64)
	assert.NoError(t, err)
	_, _ = aborted.Write(body[:1000])
	aborted.Abort()
	_, err = aborted.Close()
	assert.Error(t, err)
}

// A body read into pinned memory hashes in place (zero-copy) to the same tree as a Go slice.
func TestPinnedBufferZeroCopy(t *testing.T) {
	b, err := NewPinnedBuffer(8<<20 + 77)
	assert.NoError(t, err)
	defer b.Free()
	body := b.Bytes()
	for i := range body {
		body[i] = byte(i*7 + i>>11)
	}
	goCopy := append([]byte(nil), body...)
	want, err := NewHashTreeFromBuffer(goCopy, 1<<20)
	assert.NoError(t, err)
	got, err := NewHashTreeFromBuffer(body, 1<<20)
	assert.NoError(t, err)
	assert.Equal(t, want.MerkleRoot(), got.MerkleRoot())
	part, err := NewHashTreeFromPinned(b, len(body)-77, 1<<20)
	assert.NoError(t, err)
	wantPart, err := NewHashTreeFromBuffer(goCopy[:len(body)-77], 1<<20)
	assert.NoError(t, err)
	assert.Equal(t, wantPart.MerkleRoot(), part.MerkleRoot())
	_, err = NewHashTreeFromPinned(b, len(body)+1, 1<<20)
	assert.Error(t, err)
	_, err = NewPinnedBuffer(0)
	assert.Error(t, err)
	b.Free()
	b.Free() // idempotent
	_, err = NewHashTreeFromPinned(b, 1, 1<<20)
	assert.Error(t, err)
}

// cpuTree: the merkletree over crypto/sha256 leaf digests (Go's own hashing, no GPU).
func cpuTree(t *testing.T, chunks [][]byte) *merkletree.MerkleTree {
	list := make([]merkletree.Content, len(chunks))
	for i, c := range chunks {
		d := sha256.Sum256(c)
		list[i] = HashTreeContent{digest: d[:]}
	}
	tree, err := merkletree.NewTree(list)
	assert.NoError(t, err)
	return tree
}

// More distinct chunk sizes than MaxBatchers: the extra sizes take dm_root_buffer, same trees.
func TestBatcherBound(t *testing.T) {
	body := make([]byte, 3<<20+5)
	for i := range body {
		body[i] = byte(i * 13)
	}
	for c := 1; c <= MaxBatchers+3; c++ {
		chunk := c << 16
		got, err := NewHashTreeFromBuffer(body, chunk)
		assert.NoError(t, err)
		var chunks [][]byte
		for off := 0; off < len(body); off += chunk {
			chunks = append(chunks, body[off:min(off+chunk, len(body))])
		}
		want := cpuTree(t, chunks)
		assert.Equal(t, want.MerkleRoot(), got.MerkleRoot())
	}
	batchMu.Lock()
	assert.LessOrEqual(t, len(batchers), MaxBatchers)
	batchMu.Unlock()
}

// Concurrent handler goroutines (the batcher path) get the trees a single call gives.
func TestFromBufferConcurrent(t *testing.T) {
	var wg sync.WaitGroup
	for g := 0; g < 32; g++ {
		wg.Add(1)
		go func(g int) {
			defer wg.Done()
			body := make([]byte, 3<<20+g*4099)
			for i := range body {
				body[i] = byte(i*13 + g)
			}
			got, err := NewHashTreeFromBuffer(body, 1<<20)
			assert.NoError(t, err)
			var leaves [][32]byte
			for o := 0; o < len(body); o += 1 << 20 {
				leaves = append(leaves, sha256.Sum256(body[o:min(o+1<<20, len(body))]))
			}
			assert.Equal(t, len(leaves)+len(leaves)%2, len(got.Leafs))
			for i := range leaves {
				assert.Equal(t, leaves[i][:], got.Leafs[i].Hash)
			}
		}(g)
	}
	wg.Wait()
}
