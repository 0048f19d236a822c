//go:build nsx

// Mirrors transport/tcp/tcp_test.go:26-32 through the cgo path, plus the batch
// entry point against the single-segment one.
package tcp

import "testing"

func TestChecksum16MatchesReferenceTest(t *testing.T) {
	seg := append(make([]byte, 20), []byte("hello")...)
	raw := checksum16(nil, seg)
	if raw != 0x43D2 {
		t.Fatalf("raw = %#x, want 0x43d2", raw)
	}
	field := ^raw
	seg[16], seg[17] = byte(field>>8), byte(field)
	if got := checksum16(nil, seg); got != 0xFFFF {
		t.Fatalf("verify = %#x, want 0xffff", got)
	}
}

func TestChecksumSegmentsMatchesSingle(t *testing.T) {
	segs := [][]byte{[]byte("hello"), {}, {0xff, 0xff}, []byte("an odd-length segment")}
	pseudo := [][]byte{{10, 0, 0, 1, 10, 0, 0, 2, 0, 6, 0, 5}, {}, {0, 1}, {0, 0}}
	got, err := ChecksumSegments(segs, pseudo, 0)
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	for i := range segs {
		if want := checksum16(pseudo[i], segs[i]); got[i] != want {
			t.Fatalf("segment %d: %#x, want %#x", i, got[i], want)
		}
	}
}

// BuildSegments against the reference's own send loop: for every segment,
// s.checksum = ^s.computeChecksum(pseudo) over the field-zero image
// (tcp_test.go:28, tcp.go:68), then s.bytes() (tcp.go:98-128) — the image the
// GPU built must be those bytes and Raw the sum; the receiver's re-sum is 0xFFFF
// (tcp.go:70). Covers the reference's TestSegmentCodec segment, options with
// the reference's padding (tcp.go:118-121), empty and odd payloads.
func TestBuildSegmentsMatchesReferenceSendLoop(t *testing.T) {
	mss := option{kind: optionKindMSS, length: 4, data: []byte{0x05, 0xb4}}
	segs := []segment{
		{srcPort: 1, dstPort: 2, seqNum: 3, ackNum: 4, window: 6, checksum: 7, urgentPtr: 8, data: []byte{9}},
		{data: []byte("hello")},
		{srcPort: 443, dstPort: 51000, seqNum: 0xdeadbeef, control: ctl{ack: true, psh: true}, window: 0xffff,
			options: []option{{kind: optionKindNoOp}, {kind: optionKindNoOp}, mss}, data: make([]byte, 1460)},
		{control: ctl{syn: true}, options: []option{mss}},
		{options: []option{{kind: optionKindNoOp}}, data: []byte("odd")},
	}
	for i := range segs {
		segs[i].offset = segs[i].computeOffset()
	}
	pseudo := make([][]byte, len(segs))
	for i := range pseudo {
		pseudo[i] = []byte{10, 0, 0, 1, 10, 0, 0, byte(2 + i), 0, 6, 0, 0}
	}
	b, err := BuildSegments(segs, pseudo, 0)
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	defer b.Free()
	for i, s := range segs {
		s.checksum = 0
		raw := s.computeChecksum(pseudo[i])
		s.checksum = ^raw
		want := s.bytes()
		if b.Raw[i] != raw {
			t.Fatalf("segment %d: raw %#x, want %#x", i, b.Raw[i], raw)
		}
		if got := b.Image(i); string(got) != string(want) {
			t.Fatalf("segment %d: image %x, want %x", i, got, want)
		}
		if v := s.computeChecksum(pseudo[i]); v != 0xFFFF {
			t.Fatalf("segment %d: receiver re-sum %#x", i, v)
		}
	}
}
