// nsx_loopback — config 1 of BASELINE.json ("64×1500 B TCP segments over
// transport/pipe loopback") and the f4 feed: a sender thread
// serialises TCP segments with the nsx::tcp mirror (checksum field = ~raw over
// the IPv4 pseudo-header, tcp.go:68-71), writes them through an nsx::pipe
// loopback (transport/pipe/pipe.go semantics); the receiver frames exactly
// seg_len bytes per segment (io.ReadFull) and verifies every checksum:
//   --mode host   per-segment nsx_csum16 on arrival (computeChecksum's path)
//   --mode batch  frames land in pinned memory; one nsx_csum_fixed_host call
//                 (GPU) verifies the whole batch — the transport feeding batches.
//   --mode ring-host / ring-gpu
//                 buffered pipe (transport/pipe/buffered.go) whose receive
//                 buffer is the batch (pinned for ring-gpu); the receiver
//                 verifies the frames in place — per segment on the host, or
//                 one GPU batch straight from the pipe's buffer (no copy).
// Prints one JSON line. --dump FILE also writes, per segment, the 12-byte pseudo-header, the seg_len bytes
// sent and the raw sum the receiver computed on the last repetition (u16 LE), so a test can compare every raw
// sum with the oracle's computeChecksum over the same bytes (tests/test_pipe_cpp.py).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "nsx/pipe.hpp"
#include "nsx/tcp.hpp"

int main(int argc, char** argv) {
    int nseg = 64, seg_len = 1500, reps = 200, corrupt = -1;
    std::string mode = "host", dump;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        if (k == "--segments") nseg = std::atoi(argv[i + 1]);
        else if (k == "--seg-len") seg_len = std::atoi(argv[i + 1]);
        else if (k == "--reps") reps = std::atoi(argv[i + 1]);
        else if (k == "--mode") mode = argv[i + 1];
        else if (k == "--corrupt") corrupt = std::atoi(argv[i + 1]);  // flip a bit of segment K
        else if (k == "--dump") dump = argv[i + 1];
    }
    if (seg_len < 20 || corrupt >= nseg || nseg < 1 || reps < 1 || (mode != "host" && mode != "batch" && mode != "ring-host" && mode != "ring-gpu")) {
        std::fprintf(stderr, "usage: nsx_loopback [--segments N] [--seg-len L>=20] [--reps R] [--mode host|batch|ring-host|ring-gpu] [--corrupt K] [--dump FILE]\n");
        return 2;
    }
    // Build the segments once (sender side of tcp.go: field zero, sum, store ~sum).
    std::mt19937_64 rng(0x1071);
    std::vector<std::vector<uint8_t>> wire(nseg), pseudo(nseg);
    std::vector<uint32_t> partial(nseg);
    for (int i = 0; i < nseg; ++i) {
        nsx::tcp::Segment s;
        s.src_port = (uint16_t)rng();
        s.dst_port = 443;
        s.seq_num = (uint32_t)rng();
        s.ack_num = (uint32_t)rng();
        s.control.ack = true;
        s.window = 65535;
        s.data.resize(seg_len - 20);
        for (auto& b : s.data) b = (uint8_t)rng();
        s.offset = s.compute_offset();
        const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2};
        pseudo[i] = nsx::tcp::ipv4_pseudo_header(src, dst, 6, (uint16_t)seg_len);
        for (size_t k = 0; k + 1 < pseudo[i].size(); k += 2) partial[i] += (uint32_t)pseudo[i][k] << 8 | pseudo[i][k + 1];
        s.checksum = nsx_field(s.compute_checksum(pseudo[i]));
        wire[i] = s.bytes();
    }
    if (corrupt >= 0) wire[corrupt][seg_len / 2] ^= 0x10;  // damaged in transit: the receiver must notice
    const size_t batch = (size_t)nseg * seg_len;
    const bool gpu = mode == "batch" || mode == "ring-gpu";
    uint8_t* pinned = nullptr;
    if (gpu) {
        void* p = nullptr;
        const int rc = nsx_alloc_pinned(batch, &p);
        if (rc != NSX_OK) {
            std::printf("{\"error\": \"%s\"}\n", nsx_strerror(rc));
            return 1;
        }
        pinned = static_cast<uint8_t*>(p);
    }
    std::vector<uint8_t> frame(seg_len);
    std::vector<uint16_t> raw(nseg);
    long bad = 0;
    int rc = NSX_OK;
    auto host_verify = [&](int i, const uint8_t* seg) {
        uint16_t sum = 0;
        nsx_csum16(pseudo[i].data(), pseudo[i].size(), seg, seg_len, &sum);
        raw[i] = sum;
        bad += !nsx_verify(sum);
    };
    auto gpu_verify = [&](const uint8_t* frames) {  // one batch call; raw sums come back per segment
        rc = nsx_csum_fixed_host(frames, seg_len, seg_len, nseg, partial.data(), raw.data(), 1);
        for (int i = 0; i < nseg && rc == NSX_OK; ++i) bad += !nsx_verify(raw[i]);
    };
    auto send_all = [&](auto& c1) {
        for (int i = 0; i < nseg; ++i) {
            size_t n = 0;
            if (c1.write(wire[i].data(), wire[i].size(), &n) != nsx::pipe::Err::kOk) return;
        }
    };
    double best = 1e30, total = 0;
    for (int r = 0; r < reps && rc == NSX_OK; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        if (mode == "host" || mode == "batch") {
            // unbuffered rendezvous pipe (pipe.go): frame with read_full
            auto ends = nsx::pipe::make_pipe("client", "server");
            t0 = std::chrono::steady_clock::now();
            std::thread writer([&] { send_all(ends.first); });
            for (int i = 0; i < nseg; ++i) {
                uint8_t* dst = pinned ? pinned + (size_t)i * seg_len : frame.data();
                if (ends.second.read_full(dst, seg_len) != nsx::pipe::Err::kOk) { ++bad; break; }
                if (!pinned) host_verify(i, dst);
            }
            if (pinned) gpu_verify(pinned);
            writer.join();
        } else {
            // buffered pipe (buffered.go) whose receive buffer holds one batch;
            // the receiver verifies the frames in place (peek/consume, no copy)
            auto ends = nsx::pipe::make_buffered_pipe("client", "server", batch, nullptr, pinned);
            t0 = std::chrono::steady_clock::now();
            std::thread writer([&] { send_all(ends.first); });
            const uint8_t* view = nullptr;
            size_t avail = 0;
            if (ends.second.peek(batch, &view, &avail) != nsx::pipe::Err::kOk || avail != batch) {
                ++bad;
            } else if (pinned) {
                gpu_verify(view);
            } else {
                for (int i = 0; i < nseg; ++i) host_verify(i, view + (size_t)i * seg_len);
            }
            ends.second.consume(avail);
            writer.join();
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        best = dt < best ? dt : best;
        total += dt;
    }
    if (rc != NSX_OK) {
        std::printf("{\"error\": \"%s\"}\n", nsx_strerror(rc));
        if (pinned) nsx_free_pinned(pinned);
        return 1;
    }
    if (pinned) nsx_free_pinned(pinned);
    if (!dump.empty()) {
        FILE* f = std::fopen(dump.c_str(), "wb");
        if (!f) return 1;
        for (int i = 0; i < nseg; ++i) {
            const uint8_t r[2] = {(uint8_t)(raw[i] & 0xFF), (uint8_t)(raw[i] >> 8)};
            std::fwrite(pseudo[i].data(), 1, pseudo[i].size(), f);
            std::fwrite(wire[i].data(), 1, wire[i].size(), f);
            std::fwrite(r, 1, 2, f);
        }
        std::fclose(f);
    }
    const double bytes = (double)nseg * seg_len;
    std::printf("{\"config\": \"config1: %d x %dB TCP segments over nsx::pipe loopback\", \"mode\": \"%s\", "
                "\"reps\": %d, \"bad\": %ld, \"corrupt\": %d, \"best_us_per_batch\": %.2f, \"mean_us_per_batch\": %.2f, "
                "\"us_per_segment\": %.3f, \"MB_per_s_best\": %.1f}\n",
                nseg, seg_len, mode.c_str(), reps, bad, corrupt, best * 1e6, total / reps * 1e6, best * 1e6 / nseg,
                bytes / best / 1e6);
    return bad == (corrupt >= 0 ? reps : 0) ? 0 : 1;
}
