// fluere_cli.cpp -- `fluere offline` drop-in CLI over the C ABI.
//
// Mirrors the offline sub-command of the reference CLI (src/cli.rs:93-138,
// parse_offline_args :347-372, execute_mode src/lib.rs:58-66):
//   fluere offline -f <pcap> [-c <csv>] [-t <timeout ms>] [-M] [-v <0-4>]
// -c is accepted and ignored exactly like the reference
// (offline_fluereflows.rs:27-30); the CSV goes to ./output/<stem>_converted.csv.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/fluere_gpu.h"

static int usage() {
    fprintf(stderr,
            "usage: fluere offline -f <file.pcap> [-c <csv>] [-t <timeout_ms>] [-M] [-o <out_dir>] [-v <level>]\n");
    return 2;
}

int main(int argc, char** argv) {
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
