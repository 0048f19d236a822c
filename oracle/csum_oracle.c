/*
 * csum_oracle.c — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * CPU restatement of the reference's Internet checksum path, used solely as the
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Nothing under network-stack_amd/ links, loads or calls this file.
 *
 * Reference (oneee-playground/network-stack @ 2025-06-29, pure Go, no cgo):
 *   transport/tcp/tcp.go:72-95   func (s segment) computeChecksum(ipPseudoHeader []byte) uint16
 *   transport/tcp/tcp.go:98-128  func (s segment) bytes() []byte
 *   transport/tcp/tcp.go:59-66   func (s segment) computeOffset() uint8
 *   transport/tcp/tcp.go:188-216 ctl.byte / ctlFromByte
 *   transport/tcp/tcp.go:225-231 option.bytes
 *
 * Parity pinning: the reference is Go and no Go toolchain exists in this
 * container or on the GPU box, so the reference cannot be built or run here
 * (SURVEY.md §8c). This restatement is pinned by (1) the reference's only
 * checksum test, transport/tcp/tcp_test.go:26-32 (store ^sum over the
 * segment{data:"hello"} serialization, the re-sum must be 0xFFFF), reproduced in
 * tests/test_oracle.py, and (2) the RFC 1071 §3 numerical example plus the
 * hand-derived KATs of SURVEY.md §8c (tests/golden/kat.json).
 *
 * Two formulations that must agree bit for bit:
 *   oracle_go_checksum   — literal restatement: allocate + concatenate prefix and
 *                          segment (tcp.go:73), zero-pad an odd total (tcp.go:74-77),
 *                          16-bit big-endian words with the compare-carry end-around
 *                          add (tcp.go:79-92), return the raw sum (tcp.go:94).
 *   oracle_fold_checksum — wide form: integer sum of BE words over the virtual
 *                          concatenation into a u64, then fold to 16 bits.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_EXPORT __attribute__((visibility("default")))

/* tcp.go:72-95, statement for statement. Returns 0xFFFFFFFF on allocation
 * failure (the Go code would panic). */
ORACLE_EXPORT uint32_t oracle_go_checksum(const uint8_t* prefix, size_t prefix_len,
                                          const uint8_t* seg, size_t seg_len) {
    /* input := append(ipPseudoHeader, s.bytes()...)  (tcp.go:73) */
    size_t n = prefix_len + seg_len;
    uint8_t* input = (uint8_t*)malloc(n + 1);
    if (!input) return 0xFFFFFFFFu;
    if (prefix_len) memcpy(input, prefix, prefix_len);
    if (seg_len) memcpy(input + prefix_len, seg, seg_len);
    /* if len(input)%2 == 1 { input = append(input, byte(0)) }  (tcp.go:74-77) */
    if (n % 2 == 1) input[n++] = 0;
    /* the serial end-around-carry loop (tcp.go:79-92) */
    uint16_t sum = 0;
    for (size_t idx = 0; idx < n; idx += 2) {
        uint16_t v = (uint16_t)(((uint16_t)input[idx] << 8) + (uint16_t)input[idx + 1]);
        v = (uint16_t)(v + sum);
        if (sum > v) v++;
        sum = v;
    }
    free(input);
    return sum; /* raw sum, not complemented (tcp.go:94) */
}

static inline uint16_t fold64(uint64_t s) {
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint16_t)s;
}

/* Integer sum of the big-endian 16-bit words of bytes that begin at logical
 * position `pos` of the concatenated stream (pos parity decides pairing). */
static uint64_t be_word_sum(const uint8_t* p, size_t len, size_t pos) {
    uint64_t s = 0;
    for (size_t i = 0; i < len; i++) {
        uint64_t b = p[i];
        s += ((pos + i) & 1) ? b : (b << 8);
    }
    return s;
}

/* Wide formulation over the virtual concatenation prefix||seg (no copy). */
ORACLE_EXPORT uint32_t oracle_fold_checksum(const uint8_t* prefix, size_t prefix_len,
                                            const uint8_t* seg, size_t seg_len) {
    uint64_t s = be_word_sum(prefix, prefix_len, 0) + be_word_sum(seg, seg_len, prefix_len);
    return fold64(s);
}

/* Raw sum of one segment with a pre-summed prefix partial (the device API's
 * d_prefix_partial convention: any integer sum, folded or not, of the prefix's
 * BE words; the prefix length is even). */
static uint16_t seg_with_partial(const uint8_t* seg, size_t len, uint32_t partial) {
    return fold64((uint64_t)partial + be_word_sum(seg, len, 0));
}

/* Batch forms used as the checker of the device kernels. */
ORACLE_EXPORT void oracle_batch_fixed(const uint8_t* base, uint64_t stride, uint32_t seg_len,
                                      uint64_t n, const uint32_t* prefix_partial,
                                      uint16_t* out) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = seg_with_partial(base + i * stride, seg_len, prefix_partial ? prefix_partial[i] : 0);
}

ORACLE_EXPORT void oracle_batch_ragged(const uint8_t* base, const uint64_t* offsets, uint64_t n,
                                       const uint32_t* prefix_partial, uint16_t* out) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = seg_with_partial(base + offsets[i], (size_t)(offsets[i + 1] - offsets[i]),
                                  prefix_partial ? prefix_partial[i] : 0);
}

/* The Go-faithful form over a fixed-stride batch: one oracle_go_checksum call
 * (allocate, concatenate, pad, serial loop) per segment, exactly as a Go caller
 * looping over computeChecksum would pay it. This is bench.py's cpu_baseline leg. */
ORACLE_EXPORT void oracle_go_batch_fixed(const uint8_t* base, uint64_t stride, uint32_t seg_len,
                                         uint64_t n, const uint8_t* prefix, size_t prefix_len,
                                         uint16_t* out) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = (uint16_t)oracle_go_checksum(prefix, prefix_len, base + i * stride, seg_len);
}

/* The same with a pseudo-header of its own per segment (tcp.go:72-73: a caller
 * passes each segment's ipPseudoHeader): prefix i = pseudo[i*plen, (i+1)*plen). */
ORACLE_EXPORT void oracle_go_batch_fixed_pseudo(const uint8_t* base, uint64_t stride, uint32_t seg_len,
                                                uint64_t n, const uint8_t* pseudo, size_t plen,
                                                uint16_t* out) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = (uint16_t)oracle_go_checksum(pseudo + i * plen, plen, base + i * stride, seg_len);
}

/* The same over a ragged batch: segment i = base[offsets[i], offsets[i+1]). */
ORACLE_EXPORT void oracle_go_batch_ragged(const uint8_t* base, const uint64_t* offsets, uint64_t n,
                                          const uint8_t* prefix, size_t prefix_len, uint16_t* out) {
    for (uint64_t i = 0; i < n; i++)
        out[i] = (uint16_t)oracle_go_checksum(prefix, prefix_len, base + offsets[i],
                                              (size_t)(offsets[i + 1] - offsets[i]));
}

/* Multi-threaded variant of oracle_batch_fixed / _ragged for full-size checks
 * in the GPU tests (contiguous index shards, one pthread each). */
typedef struct {
    const uint8_t* base; uint64_t stride; uint32_t seg_len; const uint64_t* offsets;
    uint64_t lo, hi; const uint32_t* partial; uint16_t* out;
} shard_arg;

static void* shard_run(void* a_) {
    shard_arg* a = (shard_arg*)a_;
    for (uint64_t i = a->lo; i < a->hi; i++) {
        const uint8_t* p; size_t len;
        if (a->offsets) { p = a->base + a->offsets[i]; len = (size_t)(a->offsets[i + 1] - a->offsets[i]); }
        else { p = a->base + i * a->stride; len = a->seg_len; }
        a->out[i] = seg_with_partial(p, len, a->partial ? a->partial[i] : 0);
    }
    return NULL;
}

ORACLE_EXPORT void oracle_batch_mt(const uint8_t* base, uint64_t stride, uint32_t seg_len,
                                   const uint64_t* offsets, uint64_t n,
                                   const uint32_t* prefix_partial, uint16_t* out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    pthread_t th[64];
    shard_arg args[64];
    for (int t = 0; t < threads; t++) {
        args[t] = (shard_arg){base, stride, seg_len, offsets, n * t / threads, n * (t + 1) / threads,
                              prefix_partial, out};
        pthread_create(&th[t], NULL, shard_run, &args[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}

/* ---- tcp.go:98-128 segment serialization (for struct-level parity) ---- */

typedef struct {
    uint8_t kind, length;
    const uint8_t* data; size_t data_len;
} oracle_option;

typedef struct {
    uint16_t src_port, dst_port;
    uint32_t seq_num, ack_num;
    uint8_t offset, control; /* control: already-encoded ctl byte (tcp.go:197-206) */
    uint16_t window, checksum, urgent_ptr;
    const oracle_option* options; size_t n_options;
    const uint8_t* data; size_t data_len;
} oracle_segment;

/* option.bytes (tcp.go:225-231): MSS → kind,length,data...; every other kind → kind. */
static size_t option_bytes(const oracle_option* o, uint8_t* out) {
    if (o->kind == 2) {
        out[0] = o->kind; out[1] = o->length;
        if (o->data_len) memcpy(out + 2, o->data, o->data_len);
        return 2 + o->data_len;
    }
    out[0] = o->kind;
    return 1;
}

/* Returns the serialized length; writes at most `cap` bytes (call with cap=0 to
 * size). Reproduces the reference's option padding exactly: it appends
 * `remainder` zero bytes, not 4-remainder (tcp.go:118-121). */
ORACLE_EXPORT size_t oracle_segment_bytes(const oracle_segment* s, uint8_t* out, size_t cap) {
    size_t optlen = 0;
    for (size_t i = 0; i < s->n_options; i++)
        optlen += (s->options[i].kind == 2) ? 2 + s->options[i].data_len : 1;
    size_t total = 20 + optlen;
    if (s->n_options > 0) total += total % 4;
    total += s->data_len;
    if (cap < total) return total;
    uint8_t* b = out;
    b[0] = s->src_port >> 8; b[1] = s->src_port & 0xFF;
    b[2] = s->dst_port >> 8; b[3] = s->dst_port & 0xFF;
    for (int i = 0; i < 4; i++) b[4 + i] = (uint8_t)(s->seq_num >> (24 - 8 * i));
    for (int i = 0; i < 4; i++) b[8 + i] = (uint8_t)(s->ack_num >> (24 - 8 * i));
    b[12] = s->offset; b[13] = s->control;
    b[14] = s->window >> 8; b[15] = s->window & 0xFF;
    b[16] = s->checksum >> 8; b[17] = s->checksum & 0xFF;
    b[18] = s->urgent_ptr >> 8; b[19] = s->urgent_ptr & 0xFF;
    size_t at = 20;
    if (s->n_options > 0) {
        for (size_t i = 0; i < s->n_options; i++) at += option_bytes(&s->options[i], b + at);
        size_t rem = at % 4;
        memset(b + at, 0, rem);
        at += rem;
    }
    if (s->data_len) memcpy(b + at, s->data, s->data_len);
    return at + s->data_len;
}

/* computeOffset (tcp.go:59-66): ceil((20 + Σ len(option.bytes())) / 4). */
ORACLE_EXPORT uint8_t oracle_compute_offset(const oracle_segment* s) {
    size_t off = 20;
    for (size_t i = 0; i < s->n_options; i++)
        off += (s->options[i].kind == 2) ? 2 + s->options[i].data_len : 1;
    return (uint8_t)((off + 3) / 4);
}

/* Go-faithful sender loop for f1, option-less segments:
 * per segment i, build segment{fields, data} with checksum 0, s.bytes()
 * (tcp.go:98-128, a fresh allocation), sum = computeChecksum(pseudo_i)
 * (tcp.go:72-95, oracle_go_checksum: allocate + concatenate + serial loop),
 * store ^sum at bytes 16-17 (tcp.go:68,110) and copy the wire image to
 * out + out_off[i] (the transport's send buffer). pseudo: n×pseudo_len bytes or
 * NULL. raw (nullable) receives the sums. bench.py's cpu_baseline leg for
 * workload 6 and the checker for the sampled GPU output. Returns 0, or -1 if an
 * allocation failed (the Go code would panic). */
ORACLE_EXPORT int oracle_go_tcp_build_batch(const uint16_t* src_port, const uint16_t* dst_port,
                                            const uint32_t* seq_num, const uint32_t* ack_num,
                                            const uint8_t* offset, const uint8_t* control,
                                            const uint16_t* window, const uint16_t* urgent_ptr,
                                            const uint8_t* data, const uint64_t* data_off,
                                            const uint8_t* pseudo, size_t pseudo_len, uint64_t n,
                                            uint8_t* out, const uint64_t* out_off, uint16_t* raw) {
    for (uint64_t i = 0; i < n; i++) {
        oracle_segment s;
        memset(&s, 0, sizeof s);
        s.src_port = src_port[i]; s.dst_port = dst_port[i];
        s.seq_num = seq_num[i]; s.ack_num = ack_num[i];
        s.offset = offset[i]; s.control = control[i];
        s.window = window[i]; s.urgent_ptr = urgent_ptr[i];
        s.data = data + data_off[i];
        s.data_len = (size_t)(data_off[i + 1] - data_off[i]);
        const size_t len = oracle_segment_bytes(&s, NULL, 0);
        uint8_t* b = (uint8_t*)malloc(len ? len : 1);
        if (!b) return -1;
        oracle_segment_bytes(&s, b, len);
        const uint32_t sum = oracle_go_checksum(pseudo ? pseudo + i * pseudo_len : NULL, pseudo ? pseudo_len : 0, b, len);
        if (sum > 0xFFFFu) { free(b); return -1; }
        const uint16_t f = (uint16_t)~sum;
        b[16] = (uint8_t)(f >> 8);
        b[17] = (uint8_t)f;
        memcpy(out + out_off[i], b, len);
        free(b);
        if (raw) raw[i] = (uint16_t)sum;
    }
    return 0;
}

/* The same sender loop for segments with options, the options of segment i given
 * as their serialization opts[opt_off[i], opt_off[i+1]) (what a caller's
 * []option renders to, tcp.go:225-231). The span is read back into option units
 * (a byte 2 starts a kind-2 option: its next byte is the length and the rest of
 * the span its data; any other byte is a one-byte option), so the segment goes
 * through oracle_segment_bytes — tcp.go:113-123's loop and its `remainder`
 * padding — like a Go segment with that []option. Returns -1 for a span ending
 * in a lone 2 (no []option serialises to it) or a failed allocation. */
ORACLE_EXPORT int oracle_go_tcp_build_batch_opts(const uint16_t* src_port, const uint16_t* dst_port,
                                                 const uint32_t* seq_num, const uint32_t* ack_num,
                                                 const uint8_t* offset, const uint8_t* control,
                                                 const uint16_t* window, const uint16_t* urgent_ptr,
                                                 const uint8_t* opts, const uint64_t* opt_off,
                                                 const uint8_t* data, const uint64_t* data_off,
                                                 const uint8_t* pseudo, size_t pseudo_len, uint64_t n,
                                                 uint8_t* out, const uint64_t* out_off, uint16_t* raw) {
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* ob = opts + opt_off[i];
        const size_t olen = (size_t)(opt_off[i + 1] - opt_off[i]);
        oracle_option* ol = (oracle_option*)malloc((olen ? olen : 1) * sizeof(oracle_option));
        if (!ol) return -1;
        size_t no = 0;
        for (size_t p = 0; p < olen;) {
            if (ob[p] == 2) {
                if (p + 1 >= olen) { free(ol); return -1; }
                ol[no].kind = 2; ol[no].length = ob[p + 1];
                ol[no].data = ob + p + 2; ol[no].data_len = olen - p - 2;
                no++;
                break;
            }
            ol[no].kind = ob[p]; ol[no].length = 0; ol[no].data = NULL; ol[no].data_len = 0;
            no++;
            p++;
        }
        oracle_segment s;
        memset(&s, 0, sizeof s);
        s.src_port = src_port[i]; s.dst_port = dst_port[i];
        s.seq_num = seq_num[i]; s.ack_num = ack_num[i];
        s.offset = offset[i]; s.control = control[i];
        s.window = window[i]; s.urgent_ptr = urgent_ptr[i];
        s.options = ol; s.n_options = no;
        s.data = data + data_off[i];
        s.data_len = (size_t)(data_off[i + 1] - data_off[i]);
        const size_t len = oracle_segment_bytes(&s, NULL, 0);
        uint8_t* b = (uint8_t*)malloc(len ? len : 1);
        if (!b) { free(ol); return -1; }
        oracle_segment_bytes(&s, b, len);
        free(ol);
        const uint32_t sum = oracle_go_checksum(pseudo ? pseudo + i * pseudo_len : NULL, pseudo ? pseudo_len : 0, b, len);
        if (sum > 0xFFFFu) { free(b); return -1; }
        const uint16_t f = (uint16_t)~sum;
        b[16] = (uint8_t)(f >> 8);
        b[17] = (uint8_t)f;
        memcpy(out + out_off[i], b, len);
        free(b);
        if (raw) raw[i] = (uint16_t)sum;
    }
    return 0;
}

/* ---- fused receive check (SURVEY.md §8 f2 + f3), frame by frame ----
 * Frame i = base[offsets[i], offsets[i+1]): an IPv4 datagram carrying TCP. The
 * checks of nsx_rx_ipv4_tcp_verify_dev (include/nsx_csum.h), each sum through
 * oracle_go_checksum (tcp.go:72-95: allocate, concatenate, serial loop):
 *   ip_raw  = computeChecksum over the IHL*4 header bytes (RFC 791 §3.1), when
 *             the frame holds >= 20 bytes, IHL >= 5 and IHL*4 <= its length; else 0;
 *   tcp_raw = computeChecksum(pseudo) over the segment, pseudo = src(4) dst(4)
 *             0 6 len(2) from the header's own addresses (ip.Addr.Raw(),
 *             network/ip/v4/ipv4.go:15; ip.NextProtoTCP = 6, protocols.go:8),
 *             when the frame is also version 4, total length == frame length,
 *             unfragmented, protocol 6 and the segment >= 20 bytes (tcp.go:131);
 *             else 0;
 *   bit i   = both checks apply and both sums are 0xFFFF (tcp.go:70).
 * mask holds ceil(n/64) words; ip_raw / tcp_raw nullable. */
ORACLE_EXPORT void oracle_go_rx_ipv4_tcp(const uint8_t* base, const uint64_t* offsets, uint64_t n, uint64_t* mask,
                                         uint16_t* ip_raw, uint16_t* tcp_raw) {
    memset(mask, 0, (size_t)((n + 63) / 64) * 8);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* p = base + offsets[i];
        const uint64_t len = offsets[i + 1] - offsets[i];
        uint32_t ipr = 0, tcpr = 0;
        int valid = 0;
        if (len >= 20) {
            const uint32_t ihl = p[0] & 15u, hlen = ihl * 4u;
            if (ihl >= 5 && hlen <= len) {
                ipr = oracle_go_checksum(NULL, 0, p, hlen);
                const uint32_t total = ((uint32_t)p[2] << 8) | p[3];
                const uint32_t frag = (((uint32_t)p[6] << 8) | p[7]) & 0x3FFFu;
                if ((p[0] >> 4) == 4 && total == len && frag == 0 && p[9] == 6 && total - hlen >= 20) {
                    const uint32_t tlen = total - hlen;
                    uint8_t pseudo[12];
                    memcpy(pseudo, p + 12, 4);      /* src: ip.Addr.Raw() */
                    memcpy(pseudo + 4, p + 16, 4);  /* dst */
                    pseudo[8] = 0;
                    pseudo[9] = 6;                  /* ip.NextProtoTCP */
                    pseudo[10] = (uint8_t)(tlen >> 8);
                    pseudo[11] = (uint8_t)tlen;
                    tcpr = oracle_go_checksum(pseudo, 12, p + hlen, tlen);
                    valid = ipr == 0xFFFFu && tcpr == 0xFFFFu;
                }
            }
        }
        if (ip_raw) ip_raw[i] = (uint16_t)ipr;
        if (tcp_raw) tcp_raw[i] = (uint16_t)tcpr;
        if (valid) mask[i / 64] |= 1ull << (i % 64);
    }
}

/* Frame i: an IPv6 packet (RFC 8200 §3, fixed 40-byte header) carrying TCP
 * directly. The checks of nsx_rx_ipv6_tcp_verify_dev:
 *   tcp_raw = computeChecksum(pseudo) over the payload (tcp.go:72-95), pseudo =
 *             src(16) dst(16) len(4) 0 0 0 6 (RFC 8200 §8.1) from the header's own
 *             addresses (ip.Addr.Raw(), network/ip/v6/ipv6.go:16; ip.NextProtoTCP,
 *             protocols.go:8), when the frame holds >= 40 bytes, version 6,
 *             40 + payload length == frame length, Next Header 6 and a payload of
 *             >= 20 bytes (tcp.go:131); else 0;
 *   bit i   = those checks apply and tcp_raw == 0xFFFF (tcp.go:70).
 * mask holds ceil(n/64) words; tcp_raw nullable. */
ORACLE_EXPORT void oracle_go_rx_ipv6_tcp(const uint8_t* base, const uint64_t* offsets, uint64_t n, uint64_t* mask,
                                         uint16_t* tcp_raw) {
    memset(mask, 0, (size_t)((n + 63) / 64) * 8);
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t* p = base + offsets[i];
        const uint64_t len = offsets[i + 1] - offsets[i];
        uint32_t tcpr = 0;
        int valid = 0;
        if (len >= 40) {
            const uint32_t plen = ((uint32_t)p[4] << 8) | p[5];
            if ((p[0] >> 4) == 6 && 40u + plen == len && p[6] == 6 && plen >= 20) {
                uint8_t pseudo[40];
                memcpy(pseudo, p + 8, 16);       /* src: ip.Addr.Raw() */
                memcpy(pseudo + 16, p + 24, 16); /* dst */
                pseudo[32] = 0;
                pseudo[33] = 0;
                pseudo[34] = (uint8_t)(plen >> 8);
                pseudo[35] = (uint8_t)plen;
                pseudo[36] = pseudo[37] = pseudo[38] = 0;
                pseudo[39] = 6;                  /* ip.NextProtoTCP */
                tcpr = oracle_go_checksum(pseudo, 40, p + 40, plen);
                valid = tcpr == 0xFFFFu;
            }
        }
        if (tcp_raw) tcp_raw[i] = (uint16_t)tcpr;
        if (valid) mask[i / 64] |= 1ull << (i % 64);
    }
}

/* ---- synthetic data: splitmix64 stream, counter-based ---- */
static inline uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Byte j of the stream is byte (j % 8) of little-endian word j / 8. */
ORACLE_EXPORT void oracle_splitmix64_fill(uint8_t* buf, uint64_t byte_off, uint64_t nbytes,
                                          uint64_t seed) {
    for (uint64_t j = 0; j < nbytes; j++) {
        uint64_t pos = byte_off + j;
        buf[j] = (uint8_t)(splitmix64_at(seed, pos >> 3) >> (8 * (pos & 7)));
    }
}
