// ingest.hip -- host ingress: libpcap's offline walk, the pinned-chunk
// streaming of a capture to HBM, pcapng conversion.
#include "ctx.h"


// libpcap offline walk: stop at the first truncated or
// oversized record.  Returns records, fills offsets (relative to file start).
static int64_t pcap_walk(const uint8_t* f, uint64_t nbytes, uint64_t* offs, uint64_t cap, uint32_t* snap_out,
                         int* swapped_out, int* nsec_out) {
    if (!f || nbytes < 24) return FLUERE_E_PCAP;
    uint32_t magic;
    memcpy(&magic, f, 4);
    int sw = 0, ns = 0;
    if (magic == 0xa1b2c3d4u) {
    } else if (magic == 0xd4c3b2a1u) sw = 1;
    else if (magic == 0xa1b23c4du) ns = 1;
    else if (magic == 0x4d3cb2a1u) { sw = 1; ns = 1; }
    else return FLUERE_E_PCAP;
    auto rd = [&](uint64_t o) { uint32_t v; memcpy(&v, f + o, 4); return sw ? __builtin_bswap32(v) : v; };
    uint32_t snap = rd(16);
    const uint32_t kMax = 262144;
    if (snap == 0 || snap > kMax) snap = kMax;
    if (snap_out) *snap_out = snap;
    if (swapped_out) *swapped_out = sw;
    if (nsec_out) *nsec_out = ns;
    uint64_t off = 24;
    int64_t n = 0;
    while (off + 16 <= nbytes) {
        uint32_t incl = rd(off + 8);
        if (incl > kMax || off + 16 + (uint64_t)incl > nbytes) break;
        if (offs && (uint64_t)n < cap) offs[n] = off;
        n++;
        off += 16 + (uint64_t)incl;
    }
    return n;
}

extern "C" int64_t fluere_pcap_index(const uint8_t* file, uint64_t nbytes, uint64_t* offsets, uint64_t cap) {
    if (file && is_pcapng(file, nbytes)) {  // pcapng: the record count (offsets exist for classic files only)
        if (offsets) return FLUERE_E_ARG;
        std::vector<uint8_t> classic;
        const int rc = pcapng_to_pcap(file, nbytes, classic);
        if (rc) return rc;
        return pcap_walk(classic.data(), classic.size(), nullptr, 0, nullptr, nullptr, nullptr);
    }
    return pcap_walk(file, nbytes, offsets, cap, nullptr, nullptr, nullptr);
}

// ---------------------------------------------------------------------------
// Host ingress.  The capture streams to the device in order through pinned
// staging chunks (the copy of one chunk overlaps filling the next), and the
// record index is built on the host from the staged bytes: libpcap offline
// semantics (stop at the first bad or truncated record).  The record chain is
// a pointer chase (each header gives the next one's offset), latency-bound
// once the bytes have left the cache, so each reader thread walks its own
// chunk as it fills it (in L2-sized pieces), from a record start it
// recognises (a run of plausible headers); the calling thread then only
// checks that the true chain meets the reader's: a chunk whose guessed start
// was wrong is walked from the true position until the chains meet (or to
// its end).  The whole capture lands in one device allocation; batches
// (< 4 GiB each, u32 offsets) are sub-ranges.
// ---------------------------------------------------------------------------
constexpr uint32_t kSnapMax = 262144;
constexpr uint64_t kMaxBatch = (1ull << 32) - (1ull << 20);

// Staging slots: reader threads fill slot k % kIngestSlots with chunk k
// (pread from the file, or a copy of the host buffer) while the calling
// thread indexes the chunks in order and enqueues their H2D copies.
constexpr int kIngestSlots = 8;  // at most; FLUERE_INGEST_SLOTS / _READERS (diagnostics) pick fewer
static uint64_t ingest_chunk() {  // staging chunk bytes (FLUERE_INGEST_CHUNK_MB: diagnostics)
    static const uint64_t v =
        (uint64_t)(getenv("FLUERE_INGEST_CHUNK_MB") ? std::max(1, std::min(64, atoi(getenv("FLUERE_INGEST_CHUNK_MB")))) : 4) << 20;
    return v;
}
static int ingest_slots() {
    static const int v = getenv("FLUERE_INGEST_SLOTS") ? std::max(2, std::min(kIngestSlots, atoi(getenv("FLUERE_INGEST_SLOTS")))) : 8;
    return v;
}
static int ingest_readers() {
    static const int v = getenv("FLUERE_INGEST_READERS") ? std::max(1, std::min(16, atoi(getenv("FLUERE_INGEST_READERS")))) : 8;
    return v;
}
constexpr uint64_t kFillPiece = 512ull << 10;  // a reader fills and walks this much at a time (in L2)
constexpr int kSyncRun = 8;                    // plausible headers in a row that make a record start

// One chunk's record chain as its reader walked it (offsets chunk-relative).
struct ChunkChain {
    std::vector<uint32_t> so;  // record starts
    int64_t start = -1;        // the first record start taken; -1 none yet, -2 none found
    uint64_t next = 0;         // where the chain continues (may lie past the chunk)
    uint64_t scan = 0;         // the record-start search position
    bool stopped = false;      // the chain met a record libpcap's walk stops at
};

struct Ingest {
    fluere_ctx* c;
    uint64_t size = 0;
    uint8_t* d = nullptr;
    uint8_t* pin[kIngestSlots] = {};
    hipEvent_t ev[kIngestSlots] = {};
    bool busy[kIngestSlots] = {};
    int nslots = 2;
    int sw = 0, ns = 0;
    uint32_t snap = kSnapMax;
    uint64_t pos = 24;
    bool stopped = false;
    uint8_t tail[16];
    // the record index: pieces of the chains the readers walked, and of the
    // calling thread's own walk (absolute offsets, seq64), in capture order
    struct Piece {
        int64_t chunk;  // -1: seq64[i0, i0 + n)
        size_t i0, n;
    };
    std::vector<Piece> pieces;
    std::vector<uint64_t> seq64;
    std::vector<ChunkChain> chains;  // per chunk, when the readers walk
    uint64_t nrec = 0;
    uint32_t snap_file = kSnapMax;   // the global header's snaplen (record-start plausibility)
    std::vector<size_t> cut;         // first record of each batch
    std::vector<uint64_t> cut_base;  // byte offset of each batch
    // the capture side's record offsets (fluere_live_batch_indexed): the
    // chunks are only copied; finish() checks the records against them in
    // the source image (independent loads, not the walk's pointer chase)
    const uint8_t* src = nullptr;
    const uint64_t* given = nullptr;
    uint64_t given_n = 0;

    explicit Ingest(fluere_ctx* cc) : c(cc) {}
    ~Ingest() {
        for (int i = 0; i < kIngestSlots; i++)
            if (busy[i]) hipEventSynchronize(ev[i]);  // no copy may read a freed staging chunk
        if (c->reuse_ingest) return;  // the arena keeps them
        for (int i = 0; i < kIngestSlots; i++) {
            if (ev[i]) hipEventDestroy(ev[i]);
            if (pin[i]) hipHostFree(pin[i]);
        }
        if (d) hipFree(d);  // still owned here unless finish() handed it over
    }
    int begin(uint64_t nbytes) {
        if (nbytes < 24) return FLUERE_E_PCAP;
        size = nbytes;
        nslots = ingest_slots();
        const int ns_ = (int)std::min<uint64_t>(nslots, (nbytes + ingest_chunk() - 1) / ingest_chunk());
        const auto ta = std::chrono::steady_clock::now();
        if (c->reuse_ingest) {
            static_assert(kIngestSlots == 8, "arena slots");
            if (nbytes + 256 > c->ar_d_cap) {
                const uint64_t cap = std::max<uint64_t>(nbytes + 256, c->ar_d_cap * 3 / 2);
                hipFree(c->ar_d);
                c->ar_d = nullptr;
                c->ar_d_cap = 0;
                if (hipMalloc(&c->ar_d, cap) != hipSuccess) return FLUERE_E_NOMEM;
                c->ar_d_cap = cap;
            }
            d = c->ar_d;
            for (int i = 0; i < ns_; i++) {
                if (!c->ar_pin[i] && hipHostMalloc(&c->ar_pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess)
                    return FLUERE_E_NOMEM;
                if (!c->ar_ev[i] && hipEventCreateWithFlags(&c->ar_ev[i], hipEventDisableTiming) != hipSuccess)
                    return FLUERE_E_HIP;
                pin[i] = c->ar_pin[i];
                ev[i] = c->ar_ev[i];
            }
            return FLUERE_OK;
        }
        if (hipMalloc(&d, nbytes + 256) != hipSuccess) return FLUERE_E_NOMEM;
        const auto tb = std::chrono::steady_clock::now();
        for (int i = 0; i < ns_; i++) {
            if (hipHostMalloc(&pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess) return FLUERE_E_NOMEM;
            if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return FLUERE_E_HIP;
        }
        if (getenv("FLUERE_HOSTPROF"))
            fprintf(stderr, "[fluere] ingest setup: device buffer %.1f ms, %d pinned slots of %llu MiB %.1f ms\n",
                    1e3 * std::chrono::duration<double>(tb - ta).count(), ns_, (unsigned long long)(ingest_chunk() >> 20),
                    1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count());
        return FLUERE_OK;
    }
    // staging slot for chunk k, free once its previous copy has completed
    uint8_t* slot(uint64_t k) {
        const int i = (int)(k % nslots);
        if (busy[i]) {
            hipEventSynchronize(ev[i]);
            busy[i] = false;
        }
        return pin[i];
    }
    // Every chunk of [0, nbytes): fill(dst, offset, len) brings bytes into a
    // staging slot (reader threads), feed() indexes and copies them in order.
    template <class Fill>
    int run(uint64_t nbytes, Fill fill) {
        const uint64_t nch = (nbytes + ingest_chunk() - 1) / ingest_chunk();
        if (nch <= 1) {  // one chunk: no threads
            for (uint64_t k = 0; k < nch; k++) {
                const uint64_t cs = k * ingest_chunk(), len = std::min(ingest_chunk(), nbytes - cs);
                if (!fill(slot(k), cs, len)) return FLUERE_E_IO;
                const int rc = feed(k, cs, len);
                if (rc) return rc;
            }
            return FLUERE_OK;
        }
        const int NS = nslots, NR = ingest_readers();
        // the global header first: the readers' walks need its byte order
        if (!given) {
            if (!fill(pin[0], 0, 24)) return FLUERE_E_IO;
            if (int rc = global_header(pin[0])) return rc;
            chains.resize(nch);
        }
        std::atomic<int64_t> filled[kIngestSlots];
        for (auto& f : filled) f.store(-1);
        std::atomic<int64_t> fed{-1};
        std::atomic<bool> fail{false}, stop{false};
        auto reader = [&](int t) {
            for (uint64_t k = t; k < nch && !stop.load(); k += NR) {
                const int i = (int)(k % NS);
                // the slot's previous chunk (k - slots) indexed and its copy done
                while ((int64_t)k - NS > fed.load() && !stop.load()) std::this_thread::yield();
                if (stop.load()) return;
                if (k >= (uint64_t)NS && hipEventSynchronize(ev[i]) != hipSuccess) { fail = true; stop = true; return; }
                const uint64_t cs = k * ingest_chunk(), len = std::min(ingest_chunk(), nbytes - cs);
                if (given) {
                    if (!fill(pin[i], cs, len)) { fail = true; stop = true; return; }
                } else {
                    ChunkChain& ch = chains[k];
                    ch.so.reserve(len / 128 + 64);
                    if (k == 0) ch.start = ch.next = 24;
                    for (uint64_t f = 0; f < len; f += kFillPiece) {
                        const uint64_t pl = std::min(kFillPiece, len - f);
                        if (!fill(pin[i] + f, cs + f, pl)) { fail = true; stop = true; return; }
                        chain_walk(pin[i], cs, f + pl, len, ch);
                    }
                }
                filled[i].store((int64_t)k);
            }
        };
        static const bool hostprof = getenv("FLUERE_HOSTPROF") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        double wait_s = 0, feed_s = 0;
        std::vector<std::thread> th;
        for (int t = 0; t < NR; t++) th.emplace_back(reader, t);
        int rc = FLUERE_OK;
        for (uint64_t k = 0; k < nch && !rc; k++) {
            const int i = (int)(k % NS);
            const auto w0 = std::chrono::steady_clock::now();
            while (filled[i].load() != (int64_t)k && !fail.load()) std::this_thread::yield();
            const auto w1 = std::chrono::steady_clock::now();
            if (fail.load()) { rc = FLUERE_E_IO; break; }
            const uint64_t cs = k * ingest_chunk(), len = std::min(ingest_chunk(), nbytes - cs);
            rc = feed(k, cs, len);
            fed.store((int64_t)k);
            wait_s += std::chrono::duration<double>(w1 - w0).count();
            feed_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - w1).count();
        }
        stop = true;
        for (auto& t : th) t.join();
        if (hostprof)
            fprintf(stderr, "[fluere] ingest %llu chunks, %d slots, %d readers: %.1f ms (main waits %.1f, indexes+enqueues %.1f)\n",
                    (unsigned long long)nch, NS, NR,
                    1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), 1e3 * wait_s,
                    1e3 * feed_s);
        return rc;
    }
    uint32_t rd32(const uint8_t* p) const {
        uint32_t v;
        memcpy(&v, p, 4);
        return sw ? __builtin_bswap32(v) : v;
    }
    int global_header(const uint8_t* b) {  // pcap global header (libpcap offline)
        uint32_t magic;
        memcpy(&magic, b, 4);
        if (magic == 0xa1b2c3d4u) {
        } else if (magic == 0xd4c3b2a1u) sw = 1;
        else if (magic == 0xa1b23c4du) ns = 1;
        else if (magic == 0x4d3cb2a1u) { sw = 1; ns = 1; }
        else return FLUERE_E_PCAP;
        snap = rd32(b + 16);
        if (snap == 0 || snap > kSnapMax) snap = kSnapMax;
        snap_file = snap;
        return FLUERE_OK;
    }
    // Is q (chunk-relative, bytes [0, avail) present) the start of kSyncRun
    // plausible record headers in a row?  1 yes, 0 no, -1 not enough bytes
    // yet.  Plausible: caplen within the snaplen and the wire length, a
    // nonzero wire length, a sub-second fraction in range.  Only a speed
    // question: a wrong guess costs the calling thread a walk, never a result.
    int plausible_run(const uint8_t* b, uint64_t q, uint64_t avail, uint64_t len) const {
        const uint32_t frac_max = ns ? 1000000000u : 1000000u;
        for (int d = 0; d < kSyncRun; d++) {
            if (q >= len) return d > 0 ? 1 : 0;  // the run leaves the chunk
            if (q + 16 > avail) return avail == len ? (d > 0 ? 1 : 0) : -1;
            const uint32_t frac = rd32(b + q + 4), incl = rd32(b + q + 8), orig = rd32(b + q + 12);
            if (frac >= frac_max || incl > snap_file || incl > orig || orig == 0 || orig > (1u << 20)) return 0;
            q += 16 + (uint64_t)incl;
        }
        return 1;
    }
    // reader side: extend chunk [cs, cs + len)'s chain over its bytes [0, avail)
    void chain_walk(const uint8_t* b, uint64_t cs, uint64_t avail, uint64_t len, ChunkChain& ch) const {
        if (ch.start == -2) return;
        if (ch.start < 0) {
            // a record starts within the first kSnapMax + 16 bytes of any chunk
            const uint64_t lim = std::min<uint64_t>(len, kSnapMax + 32);
            while (ch.scan < lim) {
                const int r = plausible_run(b, ch.scan, avail, len);
                if (r < 0) return;  // wait for the next piece
                if (r > 0) break;
                ch.scan++;
            }
            if (ch.scan >= lim) { ch.start = -2; return; }
            ch.start = (int64_t)ch.scan;
            ch.next = ch.scan;
        }
        uint64_t p = ch.next;
        while (!ch.stopped && p + 16 <= avail) {
            const uint32_t incl = rd32(b + p + 8);
            if (incl > kSnapMax || cs + p + 16 + (uint64_t)incl > size) {
                ch.stopped = true;
                break;
            }
            ch.so.push_back((uint32_t)p);
            p += 16 + (uint64_t)incl;
        }
        ch.next = p;
    }
    void push_rec(uint64_t off) {
        if (pieces.empty() || pieces.back().chunk >= 0) pieces.push_back({-1, seq64.size(), 0});
        seq64.push_back(off);
        pieces.back().n++;
        nrec++;
    }
    // calling thread: the true chain met chunk k's at its record j (or its end)
    void take_chain(uint64_t k, uint64_t cs, size_t j) {
        const ChunkChain& ch = chains[k];
        const size_t n = ch.so.size() - j;
        const uint64_t end = cs + ch.next;
        if (n) {
            if (end - cut_base.back() > kMaxBatch)  // a 4-GiB batch boundary inside: place it record by record
                for (size_t i = j; i < ch.so.size(); i++) {
                    const uint64_t e = cs + (i + 1 < ch.so.size() ? ch.so[i + 1] : ch.next);
                    if (e - cut_base.back() > kMaxBatch) {
                        cut.push_back(nrec + (i - j));
                        cut_base.push_back(cs + ch.so[i]);
                    }
                }
            pieces.push_back({(int64_t)k, j, n});
            nrec += n;
        }
        pos = end;
        if (ch.stopped) stopped = true;
    }
    // chunk k = bytes [cs, cs + len) of the capture, already in slot(k)
    int feed(uint64_t k, uint64_t cs, uint64_t len) {
        const uint8_t* b = pin[k % nslots];
        if (cs == 0) {
            if (int rc = global_header(b)) return rc;
            cut.push_back(0);
            cut_base.push_back(24);
        }
        const uint64_t ce = cs + len;
        uint8_t h[16];
        const ChunkChain* ch = k < chains.size() && chains[k].start >= 0 ? &chains[k] : nullptr;
        size_t j = 0;
        while (!given && !stopped && pos + 16 <= ce) {
            if (ch && pos >= cs) {  // has the true chain met the reader's?
                const uint64_t r = pos - cs;
                while (j < ch->so.size() && ch->so[j] < r) j++;
                if (j < ch->so.size() ? ch->so[j] == r : r == ch->next) {
                    take_chain(k, cs, j);
                    break;
                }
            }
            const uint8_t* hp;
            if (pos >= cs) {
                hp = b + (pos - cs);
            } else {  // header straddles the previous chunk (its last 16 bytes are in tail)
                for (int j = 0; j < 16; j++) h[j] = pos + j >= cs ? b[pos + j - cs] : tail[16 - (cs - (pos + j))];
                hp = h;
            }
            const uint32_t incl = rd32(hp + 8);
            if (incl > kSnapMax || pos + 16 + (uint64_t)incl > size) {
                stopped = true;
                break;
            }
            if (pos + 16 + incl - cut_base.back() > kMaxBatch) {
                cut.push_back(nrec);
                cut_base.push_back(pos);
            }
            push_rec(pos);
            pos += 16 + (uint64_t)incl;
        }
        if (pos + 16 > size) stopped = true;
        if (len >= 16) memcpy(tail, b + len - 16, 16);
        else {  // short final chunk: shift it into the tail
            memmove(tail, tail + len, 16 - len);
            memcpy(tail + 16 - len, b, len);
        }
        const int i = (int)(k % nslots);
        HIPCHECK(hipMemcpyAsync(d + cs, b, len, hipMemcpyHostToDevice, c->stream));
        HIPCHECK(hipEventRecord(ev[i], c->stream));
        busy[i] = true;
        return FLUERE_OK;
    }
    // libpcap's walk over the given offsets, the same stop rules: record i is
    // taken while it starts where record i - 1 ended and its caplen is one the
    // walk takes.  Each record's test needs only its own header and the one
    // before, so threads test ranges of records at once (independent loads);
    // the first failing record ends the batch.
    void walk_given() {
        const uint64_t n = given_n;
        auto incl_of = [&](uint64_t i) -> uint64_t {
            const uint64_t o = given[i];
            return o + 16 <= size ? rd32(src + o + 8) : ~0ull;
        };
        auto ok = [&](uint64_t i, uint64_t prev_end) {
            const uint64_t o = given[i], incl = incl_of(i);
            return o == prev_end && o + 16 <= size && incl <= kSnapMax && o + 16 + incl <= size;
        };
        const int T = n >= (1u << 16) ? 8 : 1;
        std::vector<uint64_t> first_bad(T, n);
        auto part = [&](int t) {
            const uint64_t i0 = n * t / T, i1 = n * (t + 1) / T;
            uint64_t prev_end = 24;
            if (i0 > 0) {
                const uint64_t pi = incl_of(i0 - 1);
                prev_end = pi == ~0ull ? ~0ull : given[i0 - 1] + 16 + pi;
            }
            for (uint64_t i = i0; i < i1; i++) {
                if (i + 32 < i1 && given[i + 32] + 16 <= size) __builtin_prefetch(src + given[i + 32]);
                if (!ok(i, prev_end)) { first_bad[t] = i; return; }
                prev_end = given[i] + 16 + incl_of(i);
            }
        };
        if (T == 1) {
            part(0);
        } else {
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++) th.emplace_back(part, t);
            for (auto& x : th) x.join();
        }
        const uint64_t m = *std::min_element(first_bad.begin(), first_bad.end());
        pos = 24;
        for (uint64_t i = 0; i < m; i++) {
            const uint64_t end = i + 1 < m ? given[i + 1] : given[i] + 16 + incl_of(i);
            if (end - cut_base.back() > kMaxBatch) {
                cut.push_back(nrec);
                cut_base.push_back(given[i]);
            }
            push_rec(given[i]);
            pos = end;
        }
    }
    // records [g0, g1) of the index, batch-relative
    void fill_rel(uint32_t* out, size_t g0, size_t g1, const std::vector<size_t>& pstart) const {
        if (g0 >= g1) return;
        size_t pi = (size_t)(std::upper_bound(pstart.begin(), pstart.end(), g0) - pstart.begin()) - 1;
        size_t q = (size_t)(std::upper_bound(cut.begin(), cut.end(), g0) - cut.begin()) - 1;
        size_t g = g0;
        while (g < g1) {
            const Piece& P = pieces[pi];
            const size_t e = std::min(g1, pstart[pi + 1]);
            while (g < e) {
                while (q + 1 < cut.size() && cut[q + 1] <= g) q++;
                const size_t lim = q + 1 < cut.size() ? std::min(e, cut[q + 1]) : e;
                const uint64_t sub = cut_base[q];
                size_t i = P.i0 + (g - pstart[pi]);
                if (P.chunk < 0) {
                    for (; g < lim; g++, i++) out[g - g0] = (uint32_t)(seq64[i] - sub);
                } else {
                    const uint32_t* so = chains[P.chunk].so.data();
                    const uint64_t base = (uint64_t)P.chunk * ingest_chunk() - sub;  // mod 2^64
                    for (; g < lim; g++, i++) out[g - g0] = (uint32_t)(base + so[i]);
                }
            }
            pi++;
        }
    }
    // the index as batches of the context (device bytes handed over)
    int finish() {
        const auto tf = std::chrono::steady_clock::now();
        if (given && !cut.empty()) walk_given();
        HIPCHECK(hipMemsetAsync(d + size, 0, 256, c->stream));
        const size_t n = nrec;
        uint32_t* d_offs = nullptr;
        if (c->reuse_ingest) {
            if (std::max<size_t>(n, 1) > c->ar_offs_cap) {
                const uint64_t cap = std::max<uint64_t>(std::max<size_t>(n, 1), c->ar_offs_cap * 3 / 2);
                hipFree(c->ar_offs);
                c->ar_offs = nullptr;
                c->ar_offs_cap = 0;
                if (hipMalloc(&c->ar_offs, cap * 4) != hipSuccess) return FLUERE_E_NOMEM;
                c->ar_offs_cap = cap;
            }
            d_offs = c->ar_offs;
        } else if (hipMalloc(&d_offs, std::max<size_t>(n, 1) * 4) != hipSuccess) {
            return FLUERE_E_NOMEM;
        }
        // batch-relative u32 offsets, written into the staging slots (pinned)
        // a slot's worth at a time, by threads when there are many
        std::vector<size_t> pstart(pieces.size() + 1, 0);
        for (size_t q = 0; q < pieces.size(); q++) pstart[q + 1] = pstart[q] + pieces[q].n;
        const size_t per = ingest_chunk() / 4;
        for (size_t g0 = 0, part = 0; g0 < n; g0 += per, part++) {
            const size_t g1 = std::min(n, g0 + per);
            const int i = (int)(part % nslots);
            if (!pin[i]) {
                if (c->reuse_ingest) {
                    if (!c->ar_pin[i] && hipHostMalloc(&c->ar_pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess)
                        return FLUERE_E_NOMEM;
                    if (!c->ar_ev[i] && hipEventCreateWithFlags(&c->ar_ev[i], hipEventDisableTiming) != hipSuccess)
                        return FLUERE_E_HIP;
                    pin[i] = c->ar_pin[i];
                    ev[i] = c->ar_ev[i];
                } else {
                    if (hipHostMalloc(&pin[i], ingest_chunk(), hipHostMallocDefault) != hipSuccess) return FLUERE_E_NOMEM;
                    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return FLUERE_E_HIP;
                }
            }
            if (busy[i]) HIPCHECK(hipEventSynchronize(ev[i]));
            uint32_t* out = reinterpret_cast<uint32_t*>(pin[i]);
            const int T = g1 - g0 >= (1u << 20) ? 8 : 1;
            if (T == 1) {
                fill_rel(out, g0, g1, pstart);
            } else {
                std::vector<std::thread> th;
                for (int t = 0; t < T; t++) {
                    const size_t a = g0 + (g1 - g0) * t / T, e = g0 + (g1 - g0) * (t + 1) / T;
                    th.emplace_back([this, out, a, e, g0, &pstart] { fill_rel(out + (a - g0), a, e, pstart); });
                }
                for (auto& x : th) x.join();
            }
            HIPCHECK(hipMemcpyAsync(d_offs + g0, out, (g1 - g0) * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHECK(hipEventRecord(ev[i], c->stream));
            busy[i] = true;
        }
        HIPCHECK(hipStreamSynchronize(c->stream));  // staging slots free
        if (getenv("FLUERE_HOSTPROF"))
            fprintf(stderr, "[fluere] ingest finish (%llu records, %zu pieces): %.1f ms\n", (unsigned long long)n,
                    pieces.size(), 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - tf).count());
        for (int i = 0; i < kIngestSlots; i++) busy[i] = false;
        bool first = true;
        for (size_t q = 0; q < cut.size(); q++) {
            const size_t i0 = cut[q], i1 = q + 1 < cut.size() ? cut[q + 1] : n;
            if (i1 == i0) continue;
            const uint64_t base = cut_base[q];
            // the last batch ends with its last indexed record (pos), not at the
            // end of the file: a corrupt tail after a bad record header is not
            // part of any batch (and cannot push it past the 4 GiB offset range)
            const uint64_t endb = q + 1 < cut.size() ? cut_base[q + 1] : pos;
            HostBatch hb;
            hb.own_bytes = first && !c->reuse_ingest ? d : nullptr;  // one allocation for every batch
            hb.own_offs = first && !c->reuse_ingest ? d_offs : nullptr;
            first = false;
            hb.b.bytes = d + base;
            hb.b.offs = d_offs + i0;
            hb.b.nbytes = endb - base;
            hb.b.n = i1 - i0;
            hb.b.first = c->index_base + c->n_total;
            hb.b.snap = snap;
            hb.b.flags = (sw ? 1u : 0u) | (ns ? 2u : 0u);
            c->batches.push_back(hb);
            c->batches_dirty = true;
            c->census_due = true;
            c->n_total += hb.b.n;
        }
        if (c->reuse_ingest) {
            d = nullptr;  // the arena's
        } else if (first) {  // no records: nothing attached
            hipFree(d_offs);
        } else {
            d = nullptr;  // owned by the first batch now
        }
        c->have_results = false;
        return FLUERE_OK;
    }
};

// A classic pcap image with its record offsets known (live batches).
int add_host_pcap_indexed(fluere_ctx* c, const uint8_t* file, uint64_t nbytes, const uint64_t* rec_off,
                                 uint64_t n_recs) {
    Ingest in(c);
    in.src = file;
    in.given = rec_off;
    in.given_n = n_recs;
    int rc = in.begin(nbytes);
    if (rc) return rc;
    rc = in.run(nbytes, [&](uint8_t* dst, uint64_t cs, uint64_t len) {
        memcpy(dst, file + cs, len);
        return true;
    });
    return rc ? rc : in.finish();
}

extern "C" int fluere_add_host_pcap(fluere_ctx* c, const uint8_t* file, uint64_t nbytes) {
    if (!c || !file) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    if (is_pcapng(file, nbytes)) {  // libpcap reads pcapng too (pcapng.h)
        std::vector<uint8_t> classic;
        const int rc = pcapng_to_pcap(file, nbytes, classic);
        if (rc) return rc;
        return fluere_add_host_pcap(c, classic.data(), classic.size());
    }
    Ingest in(c);
    int rc = in.begin(nbytes);
    if (rc) return rc;
    rc = in.run(nbytes, [&](uint8_t* dst, uint64_t cs, uint64_t len) {
        memcpy(dst, file + cs, len);
        return true;
    });
    if (!rc) rc = in.finish();
    return rc ? rc : prepare_capture(c);
}

// File ingress for fluere_offline_file: read() straight into the pinned
// staging chunks (no intermediate copy of the capture in host memory).
extern "C" int fluere_add_pcap_file(fluere_ctx* c, const char* path) {
    if (!c || !path) return FLUERE_E_ARG;
    HIPCHECK(hipSetDevice(c->device));
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return FLUERE_E_IO;
    struct stat stt;
    if (fstat(fd, &stt) != 0) { close(fd); return FLUERE_E_IO; }
    const uint64_t nbytes = (uint64_t)stt.st_size;
    {
        uint8_t head[4] = {0, 0, 0, 0};
        if (nbytes >= 4 && pread(fd, head, 4, 0) == 4 && is_pcapng(head, 4)) {
            // pcapng: read whole, rewrite as a classic image (pcapng.h)
            std::vector<uint8_t> raw(nbytes);
            uint64_t got = 0;
            while (got < nbytes) {
                const ssize_t r = pread(fd, raw.data() + got, nbytes - got, (off_t)got);
                if (r <= 0) { close(fd); return FLUERE_E_IO; }
                got += (uint64_t)r;
            }
            close(fd);
            return fluere_add_host_pcap(c, raw.data(), nbytes);
        }
    }
    Ingest in(c);
    int rc = in.begin(nbytes);
    if (!rc)
        rc = in.run(nbytes, [&](uint8_t* dst, uint64_t cs, uint64_t len) {
            uint64_t got = 0;
            while (got < len) {
                const ssize_t r = pread(fd, dst + got, len - got, (off_t)(cs + got));
                if (r <= 0) return false;
                got += (uint64_t)r;
            }
            return true;
        });
    close(fd);
    if (!rc) rc = in.finish();
    return rc ? rc : prepare_capture(c);
}
