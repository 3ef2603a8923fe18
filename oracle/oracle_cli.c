/* oracle_cli.c -- TEST INFRASTRUCTURE: run the C restatement of the reference
 * `fluere offline` path on a pcap and write its CSV.  Also the CPU baseline:
 * prints the "Converted in" window (offline_fluereflows.rs:49,178).
 *   fluere_oracle -f in.pcap [-t ms] [-M] [-o out.csv] [--repeat k] */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fluere_oracle.h"

int main(int argc, char** argv) {
    const char* file = NULL;
    const char* out = NULL;
    unsigned long long timeout = 600000;
    int use_mac = 0, repeat = 1;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-f") && i + 1 < argc) file = argv[++i];
        else if (!strcmp(argv[i], "-t") && i + 1 < argc) timeout = strtoull(argv[++i], NULL, 10);
        else if (!strcmp(argv[i], "-M")) use_mac = 1;
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
        else if (!strcmp(argv[i], "--repeat") && i + 1 < argc) repeat = atoi(argv[++i]);
        else { fprintf(stderr, "usage: fluere_oracle -f in.pcap [-t ms] [-M] [-o out.csv]\n"); return 2; }
    }
    if (!file) return 2;
    FILE* f = fopen(file, "rb");
    if (!f) { perror(file); return 1; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* buf = malloc((size_t)n + 1);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) { fclose(f); return 1; }
    fclose(f);
    or_result r;
    double best = 1e30;
    for (int k = 0; k < repeat; k++) {
        if (k) or_result_free(&r);
        if (or_offline_buffer(buf, (uint64_t)n, timeout, use_mac, &r)) { fprintf(stderr, "bad pcap\n"); return 1; }
        if (r.loop_seconds < best) best = r.loop_seconds;
    }
    printf("{\"packets\": %llu, \"records\": %llu, \"ended\": %llu, \"loop_seconds\": %.9f}\n",
           (unsigned long long)r.packets, (unsigned long long)r.n, (unsigned long long)r.n_ended, best);
    if (out) {
        uint64_t need = or_format_csv(r.recs, r.n, NULL, 0);
        char* cs = malloc(need);
        or_format_csv(r.recs, r.n, cs, need);
        FILE* o = fopen(out, "wb");
        fwrite(cs, 1, need, o);
        fclose(o);
        free(cs);
    }
    or_result_free(&r);
    free(buf);
    return 0;
}
