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

// The reuse forms a transport keeps across batches: one Sender building batch
// after batch through its one pinned block (the results equal the one-shot
// BuildSegments'), and one PinnedBatch reset and refilled past its first
// capacity (it grows) whose checksums equal the single-segment path's.
func TestReuseFormsMatchOneShot(t *testing.T) {
	snd := NewSender()
	defer snd.Close()
	pb, err := NewPinnedBatch(16)
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	defer pb.Free()
	for round := 0; round < 4; round++ {
		segs := make([]segment, 3+round*40)
		pseudo := make([][]byte, len(segs))
		for i := range segs {
			segs[i] = segment{srcPort: uint16(i), seqNum: uint32(round<<20 | i), data: make([]byte, (i*37+round)%1500)}
			for k := range segs[i].data {
				segs[i].data[k] = byte(k*7 + i + round)
			}
			segs[i].offset = segs[i].computeOffset()
			pseudo[i] = []byte{10, 0, 0, 1, 10, 0, byte(round), byte(i), 0, 6, 0, 0}
		}
		got, err := snd.Build(segs, pseudo, 0)
		if err != nil {
			t.Skipf("no GPU: %v", err)
		}
		one, err := BuildSegments(segs, pseudo, 0)
		if err != nil {
			t.Fatal(err)
		}
		pb.Reset()
		for i := 0; i < got.Len(); i++ {
			if got.Raw[i] != one.Raw[i] || string(got.Image(i)) != string(one.Image(i)) {
				t.Fatalf("round %d segment %d: Sender.Build differs from BuildSegments", round, i)
			}
			if err := pb.Append(got.Image(i)); err != nil {
				t.Fatal(err)
			}
		}
		one.Free()
		sums, err := pb.Checksum(pseudo, 0)
		if err != nil {
			t.Fatal(err)
		}
		for i := range sums {
			if want := checksum16(pseudo[i], got.Image(i)); sums[i] != want || sums[i] != 0xFFFF {
				t.Fatalf("round %d segment %d: %#x, want %#x = 0xffff (tcp.go:70)", round, i, sums[i], want)
			}
		}
	}
}
