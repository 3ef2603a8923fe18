// pcapng.h -- pcapng ingress (host): the capture as libpcap's
// pcap_open_offline hands it to fluere (Capture::from_file,
// src/net/offline_fluereflows.rs:44) -- records in block order with
// microsecond timestamps -- rewritten as a classic pcap image, which the
// classic ingest path then streams to the device.
#pragma once
#include <stdint.h>

#include <vector>

namespace fl {
// True when the buffer starts with a pcapng Section Header Block.
bool is_pcapng(const uint8_t* f, uint64_t n);
// The classic (microsecond, little-endian, snaplen 262144, linktype 1) image
// of a pcapng capture; stops at the first block libpcap would fail on.
// FLUERE_OK, or FLUERE_E_PCAP when not even the first section is readable.
int pcapng_to_pcap(const uint8_t* f, uint64_t n, std::vector<uint8_t>& out);
}  // namespace fl
