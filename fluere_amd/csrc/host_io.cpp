// host_io.cpp -- egress and the whole `fluere offline` mode.
//
//   fluere_format_csv / fluere_write_csv   <- fluere_exporter
//       (src/utils/fluere_csv_exporter.rs:5-81): csv 1.3 Writer defaults
//       (',' delimiter, '\n' terminator, quote only when necessary -- never
//       for these fields), column order of the header at :10-38, IpAddr via
//       Rust std Display (IPv6: RFC 5952 compression, ::ffff:a.b.c.d).
//   fluere_offline_file                     <- fluereflow_fileparse
//       (src/net/offline_fluereflows.rs:26-196): open the capture, create
//       ./output-style directory, convert, write <stem>_converted.csv.
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <functional>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../../include/fluere_gpu.h"

namespace {

struct Out {
    char* buf;
    uint64_t cap, n;
    void put(const char* s, uint64_t len) {
        if (buf && n + len <= cap) memcpy(buf + n, s, len);
        n += len;
    }
    void put(const char* s) { put(s, strlen(s)); }
    void u(uint64_t v) {
        char t[24];
        int i = 24;
        do { t[--i] = (char)('0' + v % 10); v /= 10; } while (v);
        put(t + i, (uint64_t)(24 - i));
    }
    void hex(unsigned v) {
        char t[8];
        int i = 8;
        do { t[--i] = "0123456789abcdef"[v & 15]; v >>= 4; } while (v);
        put(t + i, (uint64_t)(8 - i));
    }
    // std::net::IpAddr Display
    void ip(uint8_t v6, const uint8_t* b) {
        if (!v6) {
            for (int i = 0; i < 4; i++) { if (i) put(".", 1); u(b[i]); }
            return;
        }
        unsigned seg[8];
        for (int i = 0; i < 8; i++) seg[i] = (unsigned)(b[2 * i] << 8) | b[2 * i + 1];
        bool mapped = seg[0] == 0 && seg[1] == 0 && seg[2] == 0 && seg[3] == 0 && seg[4] == 0 && seg[5] == 0xFFFF;
        if (mapped) {
            put("::ffff:");
            for (int i = 12; i < 16; i++) { if (i > 12) put(".", 1); u(b[i]); }
            return;
        }
        int bs = 0, bl = 0, cs = 0, cl = 0;  // longest zero run, first wins ties
        for (int i = 0; i < 8; i++) {
            if (seg[i] == 0) {
                if (!cl) cs = i;
                if (++cl > bl) { bl = cl; bs = cs; }
            } else cl = 0;
        }
        if (bl > 1) {
            for (int i = 0; i < bs; i++) { if (i) put(":", 1); hex(seg[i]); }
            put("::", 2);
            for (int i = bs + bl; i < 8; i++) { if (i > bs + bl) put(":", 1); hex(seg[i]); }
        } else {
            for (int i = 0; i < 8; i++) { if (i) put(":", 1); hex(seg[i]); }
        }
    }
};

const char* kHeader =
    "source,destination,src_port,dst_port,prot,d_pkts,d_octets,in_pkts,out_pkts,in_bytes,out_bytes,"
    "first,last,min_pkt,max_pkt,min_ttl,max_ttl,fin_cnt,syn_cnt,rst_cnt,psh_cnt,ack_cnt,urg_cnt,"
    "ece_cnt,cwr_cnt,ns_cnt,tos\n";

}  // namespace

// one row (FlowRecord's csv order, fluereflow.rs / exporter)
static void put_row(Out& o, const fluere_record& r) {
    o.ip(r.src_v6, r.source);
    o.put(",", 1);
    o.ip(r.dst_v6, r.destination);
    const uint64_t v[] = {r.src_port, r.dst_port, r.prot, r.d_pkts, r.d_octets, r.in_pkts, r.out_pkts,
                          r.in_bytes, r.out_bytes, r.first, r.last, r.min_pkt, r.max_pkt, r.min_ttl,
                          r.max_ttl, r.cnt[0], r.cnt[1], r.cnt[2], r.cnt[3], r.cnt[4], r.cnt[5],
                          r.cnt[6], r.cnt[7], r.cnt[8], r.tos};
    for (uint64_t x : v) { o.put(",", 1); o.u(x); }
    o.put("\n", 1);
}

// a row is at most two IPv6 texts (39) and 25 numbers of 20 digits, with separators
constexpr uint64_t kRowMax = 2 * 39 + 25 * 20 + 27;

extern "C" uint64_t fluere_format_csv(const fluere_record* recs, uint64_t n, char* buf, uint64_t cap) {
    Out o{buf, cap, 0};
    o.put(kHeader);
    for (uint64_t i = 0; i < n; i++) put_row(o, recs[i]);
    return o.n;
}

// Rows are formatted once, in blocks by threads when there are many, and
// written in order.  A block's buffer is appended whenever it has less than a
// row's bound left; a row that would not fit its bound (cannot happen: the
// bound is exact) is formatted again into a buffer of its own size.
static void format_rows(const fluere_record* recs, uint64_t i0, uint64_t i1, std::string& out) {
    std::vector<char> tmp(256 * kRowMax);
    Out o{tmp.data(), tmp.size(), 0};
    for (uint64_t i = i0; i < i1; i++) {
        if (tmp.size() - o.n < kRowMax) {
            out.append(tmp.data(), o.n);
            o.n = 0;
        }
        const uint64_t at = o.n;
        put_row(o, recs[i]);
        if (o.n > o.cap) {  // (the row did not fit: its bytes past the buffer were not written)
            Out z{nullptr, 0, 0};
            put_row(z, recs[i]);
            std::vector<char> big(z.n);
            Out b{big.data(), big.size(), 0};
            put_row(b, recs[i]);
            out.append(tmp.data(), at);
            out.append(big.data(), b.n);
            o.n = 0;
        }
    }
    out.append(tmp.data(), o.n);
}

extern "C" int fluere_write_csv(const fluere_record* recs, uint64_t n, const char* path) {
    if (!path || (!recs && n)) return FLUERE_E_ARG;
    int T = n >= (1u << 16) ? 8 : 1;
    std::vector<std::string> part(T);
    if (T > 1) {
        // threads; if the runtime cannot start them, the calling thread formats every row
        std::vector<std::thread> th;
        try {
            for (int t = 0; t < T; t++) th.emplace_back(format_rows, recs, n * t / T, n * (t + 1) / T, std::ref(part[t]));
        } catch (const std::exception&) {
            for (auto& x : th) x.join();
            th.clear();
            T = 1;
            part.assign(1, std::string());
        }
        for (auto& x : th) x.join();
    }
    if (T == 1) format_rows(recs, 0, n, part[0]);
    FILE* f = fopen(path, "wb");
    if (!f) return FLUERE_E_IO;
    bool ok = fwrite(kHeader, 1, strlen(kHeader), f) == strlen(kHeader);
    for (const auto& p : part) ok = ok && fwrite(p.data(), 1, p.size(), f) == p.size();
    const int rc = fclose(f);
    return (ok && rc == 0) ? FLUERE_OK : FLUERE_E_IO;
}

static std::string file_stem(const std::string& p) {
    // Path::file_stem(): final component without its last extension;
    // a leading dot alone is not an extension.
    size_t s = p.find_last_of('/');
    std::string name = s == std::string::npos ? p : p.substr(s + 1);
    if (name.empty() || name == "." || name == "..") return "output";
    size_t d = name.find_last_of('.');
    if (d == std::string::npos || d == 0) return name;
    return name.substr(0, d);
}

static int mkdir_p(const std::string& dir) {
    std::string cur;
    for (size_t i = 0; i <= dir.size(); i++) {
        if (i == dir.size() || dir[i] == '/') {
            if (!cur.empty() && mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
        }
        if (i < dir.size()) cur.push_back(dir[i]);
    }
    return 0;
}

extern "C" int fluere_offline_file(const char* pcap_path, uint64_t timeout_ms, int use_mac, const char* out_dir,
                                   fluere_stats* stats) {
    if (!pcap_path) return FLUERE_E_ARG;
    struct stat sb;
    if (stat(pcap_path, &sb) != 0) return FLUERE_E_IO;
    std::string dir = out_dir ? out_dir : "./output";
    if (mkdir_p(dir) != 0) return FLUERE_E_IO;
    std::string out = dir + "/" + file_stem(pcap_path) + "_converted.csv";
    fluere_opts o{};
    o.timeout_ms = timeout_ms;
    o.use_mac = use_mac;
    // flow capacity from the file size (a record is at least 16 bytes; flows
    // rarely exceed one per 64 bytes of capture).  The reference's HashMap has
    // no limit: the first pass grows the context to its census's estimate, and
    // a capture with still more flows reopens with twice the capacity.
    o.max_flows = std::max<uint64_t>(1 << 16, std::min<uint64_t>((uint64_t)sb.st_size / 64, 1 << 22));
    fluere_ctx* c = nullptr;
    fluere_stats st{};
    int rc;
    const bool prof = getenv("FLUERE_HOSTPROF") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {  // FLUERE_HOSTPROF: the call's phases
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[fluere] offline_file %s: %.1f ms\n", what, 1e3 * std::chrono::duration<double>(t - t_last).count());
        t_last = t;
    };
    for (;;) {
        rc = fluere_open(&o, &c);
        if (rc) return rc;
        lap("open");
        rc = fluere_add_pcap_file(c, pcap_path);
        lap("attach");
        if (!rc) rc = fluere_run(c, &st);
        lap("run");
        if (rc != FLUERE_E_TABLE_FULL || o.max_flows >= (1ull << 26)) break;  // (MAX_FLOWS)
        fluere_close(c);
        c = nullptr;
        o.max_flows *= 2;
    }
    if (stats) *stats = st;
    if (rc) { fluere_close(c); return rc; }
    int run_rc = rc;
    fluere_record* recs = nullptr;
    uint64_t nr = 0, ne = 0;
    rc = fluere_get_records(c, &recs, &nr, &ne);
    lap("records");
    if (!rc) rc = fluere_write_csv(recs, nr, out.c_str());
    lap("csv");
    fluere_records_free(recs);
    fluere_close(c);
    lap("close");
    return rc ? rc : run_rc;
}
