// fluere_cli.cpp -- `fluere offline` / `fluere live` drop-in CLI over the C ABI.
//
// Mirrors the offline sub-command of the reference CLI (src/cli.rs:93-138,
// parse_offline_args :347-372, execute_mode src/lib.rs:58-66):
//   fluere offline -f <pcap> [-c <csv>] [-t <timeout ms>] [-M] [-v <0-4>]
// -c is accepted and ignored exactly like the reference
// (offline_fluereflows.rs:27-30); the CSV goes to ./output/<stem>_converted.csv.
//
// and the live sub-command (cli.rs:140-266, live_fluereflow.rs:67-436) with a
// replay capture source instead of a libpcap device (no live devices on this
// path): the capture file's packets arrive in batches cut at interval
// boundaries of their own clock; each boundary is an interval export
// (./output/<csv>_<k>.csv; the reference names files by wall time).
//   fluere live --replay <pcap> [-c <csv>] [-I <interval ms>] [-d <duration ms>] [-t <timeout ms>] [-M]
#include <sys/stat.h>

#include <cerrno>
#include <chrono>
#include <vector>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/fluere_gpu.h"

static int usage() {
    fprintf(stderr,
            "usage: fluere offline -f <file.pcap> [-c <csv>] [-t <timeout_ms>] [-M] [-o <out_dir>] [-v <level>]\n"
            "       fluere live --replay <file.pcap> [-c <csv>] [-I <interval_ms>] [-d <duration_ms>] [-t <timeout_ms>]"
            " [-M] [-o <out_dir>]\n");
    return 2;
}

static uint32_t rd32(const uint8_t* p, bool sw) {
    uint32_t v;
    memcpy(&v, p, 4);
    return sw ? __builtin_bswap32(v) : v;
}

// live: replay a classic pcap as interval batches (packet clock)
static int live_main(int argc, char** argv) {
    std::string file, csv = "output", out_dir = "./output";
    uint64_t timeout = 600000, interval = 1800000, duration = 0;  // cli.rs defaults: 10 min, 30 min, infinite
    int use_mac = 0;
    for (int i = 2; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        const char* v = nullptr;
        if (a == "--replay") { if (!(v = val())) return usage(); file = v; }
        else if (a == "-c" || a == "--csv") { if (!(v = val())) return usage(); csv = v; }
        else if (a == "-I" || a == "--interval") { if (!(v = val())) return usage(); interval = strtoull(v, nullptr, 10); }
        else if (a == "-d" || a == "--duration") { if (!(v = val())) return usage(); duration = strtoull(v, nullptr, 10); }
        else if (a == "-t" || a == "--timeout") { if (!(v = val())) return usage(); timeout = strtoull(v, nullptr, 10); }
        else if (a == "-M" || a == "--useMAC") use_mac = 1;
        else if (a == "-o" || a == "--out-dir") { if (!(v = val())) return usage(); out_dir = v; }
        else return usage();
    }
    if (file.empty()) return usage();
    FILE* fp = fopen(file.c_str(), "rb");
    if (!fp) { fprintf(stderr, "[ERROR] cannot open %s\n", file.c_str()); return 1; }
    std::vector<uint8_t> data;
    uint8_t chunk[1 << 16];
    size_t got;
    while ((got = fread(chunk, 1, sizeof chunk, fp)) > 0) data.insert(data.end(), chunk, chunk + got);
    fclose(fp);
    uint32_t magic = data.size() >= 4 ? rd32(data.data(), false) : 0;
    const bool sw = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
    const bool ns = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
    if (data.size() < 24 || !(magic == 0xa1b2c3d4u || magic == 0xa1b23c4du || sw)) {
        fprintf(stderr, "[ERROR] %s: not a classic pcap\n", file.c_str());
        return 1;
    }
    fluere_opts o{};
    o.timeout_ms = timeout;
    o.use_mac = use_mac;
    o.max_flows = 1 << 20;
    fluere_live* lv = nullptr;
    int rc = fluere_live_open(&o, &lv);
    if (rc) { fprintf(stderr, "[ERROR] fluere_live_open: %d\n", rc); return 1; }
    if (mkdir(out_dir.c_str(), 0755) != 0 && errno != EEXIST) { fprintf(stderr, "[ERROR] mkdir %s\n", out_dir.c_str()); return 1; }
    int k = 0;
    auto write = [&](fluere_record* recs, uint64_t n) {
        const std::string path = out_dir + "/" + csv + "_" + std::to_string(k++) + ".csv";
        const int w = fluere_write_csv(recs, n, path.c_str());
        printf("[INFO] Export %s: %llu flows\n", path.c_str(), (unsigned long long)n);
        fluere_records_free(recs);
        return w;
    };
    std::vector<uint8_t> batch(data.begin(), data.begin() + 24);
    std::vector<uint64_t> boff;  // the batch's record offsets (the ring hands them over with the packets)
    uint64_t off = 24, start = ~0ull, bstart = ~0ull;
    bool stopped = false;
    while (!rc && off + 16 <= data.size()) {
        const uint32_t incl = rd32(&data[off + 8], sw);
        if (incl > 262144 || off + 16 + incl > data.size()) break;
        const uint64_t t = (uint64_t)rd32(&data[off], sw) * 1000000ull + (ns ? rd32(&data[off + 4], sw) / 1000 : rd32(&data[off + 4], sw));
        if (start == ~0ull) start = bstart = t;
        // signed: a timestamp that goes backwards is no elapsed interval
        const int64_t since_start = (int64_t)(t - start), since_batch = (int64_t)(t - bstart);
        boff.push_back(batch.size());
        batch.insert(batch.end(), data.begin() + off, data.begin() + off + 16 + incl);
        off += 16 + incl;
        // both checks follow the packet, the interval export first
        // (live_fluereflow.rs:303-306, then :361-373): the crossing packet
        // belongs to the interval it closes.  (The reference skips both checks
        // after a packet that fails parse_keys / parse_fluereflow; the session
        // runs a due export after the next processed packet, the same point.)
        if (interval && since_batch >= (int64_t)(interval * 1000)) {
            fluere_record* recs = nullptr;
            uint64_t n = 0, no = 0;
            int ex = 0;
            rc = fluere_live_batch_indexed(lv, batch.data(), batch.size(), boff.data(), boff.size(), 1, &recs, &n, &no,
                                           &ex);
            if (!rc && ex) rc = write(recs, n);
            batch.resize(24);
            boff.clear();
            bstart = t;
        }
        if (duration && since_start >= (int64_t)(duration * 1000)) { stopped = true; break; }
    }
    if (!rc && batch.size() > 24) {
        fluere_record* recs = nullptr;
        uint64_t n = 0, no = 0;
        int ex = 0;
        rc = fluere_live_batch_indexed(lv, batch.data(), batch.size(), boff.data(), boff.size(), 0, &recs, &n, &no, &ex);
        if (!rc && ex) rc = write(recs, n);
    }
    if (!rc) {
        fluere_record* recs = nullptr;
        uint64_t n = 0, no = 0;
        rc = fluere_live_finish(lv, stopped ? 1 : 0, &recs, &n, &no);
        if (!rc) rc = write(recs, n);
    }
    fluere_live_close(lv);
    if (rc) fprintf(stderr, "[ERROR] fluere live failed: %d\n", rc);
    return rc ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && strcmp(argv[1], "live") == 0) return live_main(argc, argv);
    if (argc < 2 || strcmp(argv[1], "offline") != 0) return usage();
    std::string file, out_dir = "./output";
    uint64_t timeout = 600000;  // cli.rs: default 10 minutes
    int use_mac = 0, verbose = 2;
    for (int i = 2; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : nullptr; };
        if (a == "-f" || a == "--file") { const char* v = val(); if (!v) return usage(); file = v; }
        else if (a == "-c" || a == "--csv") { if (!val()) return usage(); }
        else if (a == "-t" || a == "--timeout") { const char* v = val(); if (!v) return usage(); timeout = strtoull(v, nullptr, 10); }
        else if (a == "-M" || a == "--useMAC") use_mac = 1;
        else if (a == "-o" || a == "--out-dir") { const char* v = val(); if (!v) return usage(); out_dir = v; }
        else if (a == "-v" || a == "--verbose") { const char* v = val(); if (!v) return usage(); verbose = atoi(v); }
        else return usage();
    }
    if (file.empty()) return usage();
    fluere_stats st{};
    auto t0 = std::chrono::steady_clock::now();
    int rc = fluere_offline_file(file.c_str(), timeout, use_mac, out_dir.c_str(), &st);
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (verbose >= 2) {
        printf("[INFO] Converted in %.6fs (device %.3f ms)\n", s, st.total_ms);
        printf("[INFO] Active flows: %llu\n", (unsigned long long)(st.records - st.ended));
        printf("[INFO] Ended flows: %llu\n", (unsigned long long)st.ended);
    }
    if (rc)
        fprintf(stderr, "[ERROR] fluere offline failed: %d\n", rc);
    return rc ? 1 : 0;
}
