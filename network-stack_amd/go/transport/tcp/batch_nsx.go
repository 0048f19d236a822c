//go:build nsx

// Batch entry points over the MI355X library: many segments per cgo call,
// checksummed on the GPU(s). Segments are densely packed into pinned
// (DMA-registered) C memory — Go heap memory is not DMA-registered and C may
// not retain Go pointers — and handed to nsx_csum_ragged_host, which shards
// them over the node's GPUs (no collective) and pipelines H2D → kernel → D2H.
//
// Pinning memory (nsx_alloc_pinned) registers its pages with the driver, which
// costs far more than a small batch's transfer: a transport keeps one
// PinnedBatch (or Sender, build_nsx.go) per connection or receive loop and
// reuses it batch after batch — Reset, Append, Checksum / Verify — so the
// registration is paid only when a batch outgrows the block. ChecksumSegments,
// VerifyDatagrams and BuildSegments are the one-shot forms (a block per call).
package tcp

/*
#include "nsx_csum.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// pinnedArena is a grow-only block of pinned host memory reused across calls.
type pinnedArena struct {
	base unsafe.Pointer
	buf  []byte
}

// reserve makes the arena at least n bytes long, keeping its first keep bytes.
// Growing allocates a new block of at least twice the old size, copies, and
// frees the old one.
func (a *pinnedArena) reserve(n, keep uint64) error {
	if n <= uint64(len(a.buf)) {
		return nil
	}
	c := 2 * uint64(len(a.buf))
	if c < 4096 {
		c = 4096
	}
	for c < n {
		c *= 2
	}
	var p unsafe.Pointer
	if rc := C.nsx_alloc_pinned(C.size_t(c), &p); rc != C.NSX_OK {
		return fmt.Errorf("nsx_alloc_pinned: %s", C.GoString(C.nsx_strerror(rc)))
	}
	nb := unsafe.Slice((*byte)(p), c)
	copy(nb, a.buf[:keep])
	a.free()
	a.base, a.buf = p, nb
	return nil
}

func (a *pinnedArena) free() {
	if a.base != nil {
		C.nsx_free_pinned(a.base)
		a.base, a.buf = nil, nil
	}
}

// PinnedBatch is a reusable pinned staging area for segment (or received
// frame) bytes. It grows as segments are appended and keeps its block across
// Reset, so a transport calling it once per batch pins memory only while its
// batches still grow.
type PinnedBatch struct {
	arena   pinnedArena
	offsets []uint64 // n+1 offsets into the block (Go memory: read by C only during a call)
	parts   []uint32 // pseudo-header partials, reused
	mask    []uint64 // receive-pass bitmask words, reused
}

// NewPinnedBatch allocates a batch with room for capacity bytes (it grows past
// that on demand).
func NewPinnedBatch(capacity int) (*PinnedBatch, error) {
	b := &PinnedBatch{offsets: []uint64{0}}
	if err := b.arena.reserve(uint64(capacity), 0); err != nil {
		return nil, err
	}
	return b, nil
}

// Append copies one serialized segment (e.g. segment.bytes(), tcp.go:98-128)
// or one received datagram into the batch, growing it if needed.
func (b *PinnedBatch) Append(seg []byte) error {
	at := b.offsets[len(b.offsets)-1]
	end := at + uint64(len(seg))
	if err := b.arena.reserve(end+1, at); err != nil {
		return err
	}
	copy(b.arena.buf[at:], seg)
	b.offsets = append(b.offsets, end)
	return nil
}

// Len returns the number of segments in the batch.
func (b *PinnedBatch) Len() int { return len(b.offsets) - 1 }

// Reset empties the batch for reuse; its pinned block stays.
func (b *PinnedBatch) Reset() { b.offsets = b.offsets[:1] }

// Free releases the pinned memory.
func (b *PinnedBatch) Free() { b.arena.free() }

// pseudoPartial is the integer sum of a pseudo-header's big-endian 16-bit
// words (the d_prefix_partial convention of nsx_csum.h); pseudo-headers have
// even length (12 B IPv4, 40 B IPv6).
func pseudoPartial(ph []byte) uint32 {
	var s uint32
	for i := 0; i+1 < len(ph); i += 2 {
		s += uint32(ph[i])<<8 | uint32(ph[i+1])
	}
	return s
}

// Checksum returns the raw sum of every segment in the batch, each over
// pseudo[i] ‖ segment i when pseudo is non-nil (len(pseudo) == segments):
// the batch form of computeChecksum (tcp.go:72-95). numGPUs 0 = auto: one GPU
// per 64 MiB of batch, up to all visible (nsx_csum.h, host-resident batches).
func (b *PinnedBatch) Checksum(pseudo [][]byte, numGPUs int) ([]uint16, error) {
	n := b.Len()
	out := make([]uint16, n)
	if n == 0 {
		return out, nil
	}
	var partial *C.uint32_t
	if pseudo != nil {
		if len(pseudo) != n {
			return nil, errors.New("pseudo-header count != segment count")
		}
		if cap(b.parts) < n {
			b.parts = make([]uint32, n)
		}
		b.parts = b.parts[:n]
		for i, ph := range pseudo {
			if len(ph)%2 != 0 {
				return nil, errors.New("pseudo-header of odd length")
			}
			b.parts[i] = pseudoPartial(ph)
		}
		partial = (*C.uint32_t)(unsafe.Pointer(&b.parts[0]))
	}
	rc := C.nsx_csum_ragged_host((*C.uint8_t)(b.arena.base), (*C.uint64_t)(unsafe.Pointer(&b.offsets[0])),
		C.uint64_t(n), partial, (*C.uint16_t)(unsafe.Pointer(&out[0])), C.int(numGPUs))
	if rc != C.NSX_OK {
		return nil, fmt.Errorf("nsx_csum_ragged_host: %s", C.GoString(C.nsx_strerror(rc)))
	}
	return out, nil
}

// ChecksumSegments checksums segs (each already serialized) on the GPU(s): the
// one-shot form of PinnedBatch.Checksum (pins a block for this call only).
func ChecksumSegments(segs [][]byte, pseudo [][]byte, numGPUs int) ([]uint16, error) {
	total := 0
	for _, s := range segs {
		total += len(s)
	}
	b, err := NewPinnedBatch(total + 1)
	if err != nil {
		return nil, err
	}
	defer b.Free()
	for _, s := range segs {
		if err := b.Append(s); err != nil {
			return nil, err
		}
	}
	return b.Checksum(pseudo, numGPUs)
}
