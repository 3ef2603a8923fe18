// pcapng.cpp -- pcapng -> classic pcap image (pcapng.h).
//
// libpcap (pcap-ng.c) semantics as fluere sees them through pcap 2.3 at the
// default microsecond precision (third-party code, not in the reference;
// restated like SURVEY.md Appendix C):
//   * a Section Header Block fixes the byte order (magic 0x1A2B3C4D) and
//     starts a new interface list; major version must be 1;
//   * an Interface Description Block adds an interface: snaplen (0 or above
//     262144 -> 262144), if_tsresol (option 9: 10^-b, or 2^-(b & 0x7f) with
//     the high bit), if_tsoffset (option 14, seconds);
//   * Enhanced (6) and obsolete (2) Packet Blocks: interface, 64-bit time in
//     that interface's units, caplen, original length, data; Simple Packet
//     Blocks (3): no time, caplen = min(len, room in the block, snaplen of
//     interface 0); every other block type is skipped;
//   * time: seconds = t / res + tsoffset, microseconds = (t % res) * 10^6 / res;
//   * the first truncated / malformed block, unknown interface or caplen
//     above 262144 ends the capture (pcap_next_ex fails, fluere's loop stops);
//   * an Enhanced / obsolete Packet Block's caplen above the capture's
//     snapshot length (the first interface's snaplen) is cut to it, like the
//     Simple Packet Block's (unpinned: no reference fixture);
//   * a later Section Header Block in the other byte order ends the capture
//     (libpcap: "sections with different byte orders").
#include "pcapng.h"

#include <cstring>

#include "../../include/fluere_gpu.h"

namespace fl {
namespace {

constexpr uint32_t kMaxSnap = 262144;

struct Reader {
    const uint8_t* f;
    bool sw = false;
    uint32_t u32(uint64_t o) const {
        uint32_t v;
        memcpy(&v, f + o, 4);
        return sw ? __builtin_bswap32(v) : v;
    }
    uint16_t u16(uint64_t o) const {
        uint16_t v;
        memcpy(&v, f + o, 2);
        return sw ? __builtin_bswap16(v) : v;
    }
};

struct Iface {
    uint64_t res = 1000000;
    int64_t off = 0;
    uint32_t snap = kMaxSnap;
};

void put32(std::vector<uint8_t>& o, uint32_t v) {
    const uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
    o.insert(o.end(), b, b + 4);
}

}  // namespace

bool is_pcapng(const uint8_t* f, uint64_t n) {
    uint32_t t;
    if (n < 4) return false;
    memcpy(&t, f, 4);
    return t == 0x0A0D0D0Au;
}

int pcapng_to_pcap(const uint8_t* f, uint64_t n, std::vector<uint8_t>& out) {
    out.clear();
    out.reserve(n + 24);
    // classic global header: microseconds, v2.4, snaplen 262144, Ethernet
    put32(out, 0xa1b2c3d4u);
    put32(out, 2u | (4u << 16));
    put32(out, 0);
    put32(out, 0);
    put32(out, kMaxSnap);
    put32(out, 1);
    Reader R{f};
    std::vector<Iface> ifs;
    bool section = false;
    int first_sw = -1;  // byte order of the first section
    uint64_t pos = 0;
    while (pos + 12 <= n) {
        uint32_t type;
        memcpy(&type, f + pos, 4);  // the SHB type reads the same in both byte orders
        if (type == 0x0A0D0D0Au) {
            uint32_t bom;
            memcpy(&bom, f + pos + 8, 4);
            if (bom == 0x1A2B3C4Du) R.sw = false;
            else if (bom == 0x4D3C2B1Au) R.sw = true;
            else break;
            if (pos + 16 > n || R.u16(pos + 12) != 1) break;
            if (first_sw < 0) first_sw = R.sw ? 1 : 0;
            else if (first_sw != (R.sw ? 1 : 0)) break;
            section = true;
            ifs.clear();
        } else {
            if (!section) break;
            type = R.u32(pos);
        }
        const uint32_t total = R.u32(pos + 4);
        if (total < 12 || (total & 3) || pos + total > n) break;
        const uint64_t b = pos + 8;
        const uint32_t blen = total - 12;
        bool stop = false;
        if (type == 1) {  // Interface Description Block
            if (blen < 8) break;
            Iface x;
            x.snap = R.u32(b + 4);
            if (x.snap == 0 || x.snap > kMaxSnap) x.snap = kMaxSnap;
            for (uint32_t o = 8; o + 4 <= blen;) {
                const uint16_t code = R.u16(b + o), len = R.u16(b + o + 2);
                if (code == 0) break;
                if (o + 4 + len > blen) { stop = true; break; }
                if (code == 9 && len >= 1) {  // if_tsresol
                    const uint8_t v = f[b + o + 4];
                    const uint64_t base = (v & 0x80) ? 2 : 10;
                    uint64_t res = 1;
                    for (int k = 0; k < (v & 0x7f) && !stop; k++) {
                        if (res > UINT64_MAX / base) stop = true;
                        else res *= base;
                    }
                    x.res = res;
                } else if (code == 14 && len >= 8) {  // if_tsoffset
                    const uint64_t lo = R.u32(b + o + 4), hi = R.u32(b + o + 8);
                    x.off = (int64_t)(R.sw ? (lo << 32) | hi : (hi << 32) | lo);
                }
                o += 4 + ((len + 3u) & ~3u);
            }
            if (stop) break;
            ifs.push_back(x);
        } else if (type == 6 || type == 2 || type == 3) {  // EPB, obsolete PB, SPB
            uint32_t ifid = 0, caplen = 0, orig = 0;
            uint64_t t = 0, data = 0;
            if (type == 3) {
                if (blen < 4 || ifs.empty()) break;
                orig = R.u32(b);
                caplen = std::min<uint32_t>(std::min<uint32_t>(orig, blen - 4), ifs[0].snap);
                data = b + 4;
            } else {
                if (blen < 20) break;
                ifid = type == 6 ? R.u32(b) : R.u16(b);
                t = ((uint64_t)R.u32(b + 4) << 32) | R.u32(b + 8);
                caplen = R.u32(b + 12);
                orig = R.u32(b + 16);
                data = b + 20;
                if (ifid >= ifs.size() || caplen > blen - 20) break;
                caplen = std::min<uint32_t>(caplen, ifs[0].snap);
            }
            if (caplen > kMaxSnap) break;
            const Iface& x = ifs[ifid];
            uint64_t sec = 0, usec = 0;
            if (type != 3) {
                sec = t / x.res + (uint64_t)x.off;
                usec = (uint64_t)(((unsigned __int128)(t % x.res) * 1000000u) / x.res);
            }
            put32(out, (uint32_t)sec);
            put32(out, (uint32_t)usec);
            put32(out, caplen);
            put32(out, orig);
            out.insert(out.end(), f + data, f + data + caplen);
        }
        pos += total;
    }
    return out.size() > 24 || section ? FLUERE_OK : FLUERE_E_PCAP;
}

}  // namespace fl
