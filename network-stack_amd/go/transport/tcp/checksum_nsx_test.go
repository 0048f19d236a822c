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
