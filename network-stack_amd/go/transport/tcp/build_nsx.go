//go:build nsx

// Sender-side batch build over the MI355X library (SURVEY.md §8 f1). A Go
// transport's send loop — per segment bytes() (tcp.go:98-128), the checksum
// over its ipPseudoHeader (tcp.go:72-95) stored as ^sum in bytes 16-17
// (tcp.go:110, :68-71), then Write into the pipe or socket
// (transport/pipe/pipe.go:92-124) — becomes one nsx_tcp_build_host call: the
// segments' header fields, serialised options, payloads and pseudo-header
// partials are staged in one pinned (DMA-registered) block, the GPU(s) build
// every wire image, and the images and raw sums come back into the same block,
// ready to be written. C never sees a Go pointer: everything the call reads or
// writes is in the pinned block. A send loop keeps one Sender and reuses its
// block batch after batch; BuildSegments is the one-shot form.
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

// BuiltSegments holds a batch's wire images in pinned host memory.
type BuiltSegments struct {
	own    *pinnedArena // the block, when this batch owns it (BuildSegments); nil for a Sender's batch
	out    []byte
	outOff []uint64
	wire   []int
	// Raw is the raw sum of each image taken with its checksum field zero; the
	// field holds ^Raw[i], so a receiver re-summing pseudo[i] ‖ image gets
	// 0xFFFF (tcp.go:70).
	Raw []uint16
}

// Len returns the number of segments in the batch.
func (b *BuiltSegments) Len() int { return len(b.wire) }

// Image returns segment i's wire image: a view into pinned memory, byte for
// byte what s.bytes() returns after s.checksum = ^Raw[i]. Valid until Free
// (BuildSegments) or the Sender's next Build or Close.
func (b *BuiltSegments) Image(i int) []byte {
	o := b.outOff[i]
	return b.out[o : o+uint64(b.wire[i])]
}

// Free releases the pinned memory of a batch BuildSegments made (a Sender's
// batches live in the Sender's block: Free leaves them to Sender.Close).
func (b *BuiltSegments) Free() {
	if b.own != nil {
		b.own.free()
		b.own = nil
	}
	b.out = nil
}

func alignUp(x, a uint64) uint64 { return (x + a - 1) &^ (a - 1) }

// Sender builds batches of segments on the GPU(s) through one pinned block it
// keeps across calls: a send loop calls Build once per batch and writes the
// images out before the next Build, and pins memory only while its batches
// still grow (nsx_alloc_pinned costs far more than a small batch's build).
type Sender struct {
	arena  pinnedArena
	b      BuiltSegments
	optLen []uint64
}

// NewSender returns a Sender with an empty block (the first Build sizes it).
func NewSender() *Sender { return &Sender{} }

// Close releases the Sender's pinned block (and every batch it built).
func (s *Sender) Close() { s.arena.free() }

// Build builds the wire images of segs. Each segment's header fields are used
// as they are — offset included, as bytes() expects (tcp.go:97); s.checksum is
// ignored, the sum being taken with the field zero as the sender must
// (tcp.go:68) — and its options are serialised by option.bytes()
// (tcp.go:225-231) and padded as bytes() pads them (tcp.go:118-121). pseudo[i]
// is segment i's ipPseudoHeader (even length), or pseudo is nil for none.
// numGPUs 0 = auto: one GPU per 64 MiB of images, up to all visible (nsx_csum.h,
// host-resident batches). The result is valid until the next Build or Close.
func (s *Sender) Build(segs []segment, pseudo [][]byte, numGPUs int) (*BuiltSegments, error) {
	if err := build(&s.arena, &s.b, &s.optLen, segs, pseudo, numGPUs); err != nil {
		return nil, err
	}
	return &s.b, nil
}

// BuildSegments is the one-shot form of Sender.Build: the batch owns a block
// pinned for it alone, released by Free.
func BuildSegments(segs []segment, pseudo [][]byte, numGPUs int) (*BuiltSegments, error) {
	a := &pinnedArena{}
	b := &BuiltSegments{}
	var optLen []uint64
	if err := build(a, b, &optLen, segs, pseudo, numGPUs); err != nil {
		a.free()
		return nil, err
	}
	b.own = a
	return b, nil
}

func grow[T any](v []T, n int) []T {
	if cap(v) < n {
		return make([]T, n)
	}
	return v[:n]
}

// build lays segs out in arena (grown as needed) and runs nsx_tcp_build_host.
func build(arena *pinnedArena, b *BuiltSegments, optLenBuf *[]uint64, segs []segment, pseudo [][]byte,
	numGPUs int) error {
	n := len(segs)
	if pseudo != nil && len(pseudo) != n {
		return errors.New("pseudo-header count != segment count")
	}
	b.outOff, b.wire, b.Raw = grow(b.outOff, n+1), grow(b.wire, n), grow(b.Raw, n)
	b.outOff[0] = 0
	if n == 0 {
		b.out = nil
		return nil
	}
	// sizes: serialised options, payloads, 4-aligned image slots (nsx_tcp_layout_host's rule)
	*optLenBuf = grow(*optLenBuf, n)
	optLen := *optLenBuf
	var nOpt, nData uint64
	for i, s := range segs {
		if pseudo != nil && len(pseudo[i])%2 != 0 {
			return errors.New("pseudo-header of odd length")
		}
		optLen[i] = 0
		for _, op := range s.options {
			optLen[i] += uint64(len(op.bytes()))
		}
		nOpt += optLen[i]
		nData += uint64(len(s.data))
		b.wire[i] = int(C.nsx_tcp_wire_len(C.uint64_t(optLen[i]), C.uint64_t(len(s.data))))
		b.outOff[i+1] = b.outOff[i] + alignUp(uint64(b.wire[i]), 4)
	}
	nOut := b.outOff[n]
	un := uint64(n)
	// one pinned block: the 8 header field arrays (nsx_tcp_hdr_soa order below), data/opt/out offsets,
	// partials, option bytes, payload bytes, images, raw sums
	sizes := []uint64{2 * un, 2 * un, 4 * un, 4 * un, un, un, 2 * un, 2 * un,
		8 * (un + 1), 8 * (un + 1), 8 * (un + 1), 4 * un, nOpt + 1, nData + 1, nOut, 2 * un}
	var at [17]uint64
	for k, sz := range sizes {
		at[k+1] = alignUp(at[k]+sz, 64)
	}
	if err := arena.reserve(at[len(sizes)], 0); err != nil {
		return err
	}
	region := func(k int) unsafe.Pointer { return unsafe.Pointer(&arena.buf[at[k]]) }
	srcPort := unsafe.Slice((*uint16)(region(0)), n)
	dstPort := unsafe.Slice((*uint16)(region(1)), n)
	seqNum := unsafe.Slice((*uint32)(region(2)), n)
	ackNum := unsafe.Slice((*uint32)(region(3)), n)
	offset := unsafe.Slice((*uint8)(region(4)), n)
	control := unsafe.Slice((*uint8)(region(5)), n)
	window := unsafe.Slice((*uint16)(region(6)), n)
	urgentPtr := unsafe.Slice((*uint16)(region(7)), n)
	dataOff := unsafe.Slice((*uint64)(region(8)), n+1)
	optOff := unsafe.Slice((*uint64)(region(9)), n+1)
	outOff := unsafe.Slice((*uint64)(region(10)), n+1)
	parts := unsafe.Slice((*uint32)(region(11)), n)
	opts := unsafe.Slice((*byte)(region(12)), nOpt+1)
	data := unsafe.Slice((*byte)(region(13)), nData+1)
	b.out = unsafe.Slice((*byte)(region(14)), nOut)
	raw := unsafe.Slice((*uint16)(region(15)), n)
	var d, o uint64
	for i, s := range segs {
		srcPort[i], dstPort[i], seqNum[i], ackNum[i] = s.srcPort, s.dstPort, s.seqNum, s.ackNum
		offset[i], control[i], window[i], urgentPtr[i] = s.offset, s.control.byte(), s.window, s.urgentPtr
		dataOff[i], optOff[i], outOff[i] = d, o, b.outOff[i]
		for _, op := range s.options {
			o += uint64(copy(opts[o:], op.bytes()))
		}
		d += uint64(copy(data[d:], s.data))
		if pseudo != nil {
			parts[i] = pseudoPartial(pseudo[i])
		}
	}
	dataOff[n], optOff[n], outOff[n] = d, o, nOut

	var h C.nsx_tcp_hdr_soa
	h.src_port = (*C.uint16_t)(region(0))
	h.dst_port = (*C.uint16_t)(region(1))
	h.seq_num = (*C.uint32_t)(region(2))
	h.ack_num = (*C.uint32_t)(region(3))
	h.offset = (*C.uint8_t)(region(4))
	h.control = (*C.uint8_t)(region(5))
	h.window = (*C.uint16_t)(region(6))
	h.urgent_ptr = (*C.uint16_t)(region(7))
	var partial *C.uint32_t
	if pseudo != nil {
		partial = (*C.uint32_t)(region(11))
	}
	var optOffs *C.uint64_t
	if nOpt > 0 {
		optOffs = (*C.uint64_t)(region(9))
	}
	rc := C.nsx_tcp_build_host(&h, (*C.uint8_t)(region(12)), optOffs, (*C.uint8_t)(region(13)),
		(*C.uint64_t)(region(8)), partial, C.uint64_t(n), (*C.uint8_t)(region(14)), (*C.uint64_t)(region(10)),
		(*C.uint16_t)(region(15)), C.int(numGPUs))
	if rc != C.NSX_OK {
		b.out = nil
		return fmt.Errorf("nsx_tcp_build_host: %s", C.GoString(C.nsx_strerror(rc)))
	}
	copy(b.Raw, raw)
	return nil
}
