// rtps_ctx.h — internal view of a parse context for the host-side loops built
// on the public C ABI (rtps_pump.cpp).  Not part of include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

struct rtps_rx_ctx;
hipStream_t rtps_ctx_stream(const rtps_rx_ctx* c);
int rtps_ctx_device(const rtps_rx_ctx* c);
uint32_t rtps_ctx_max_datagrams(const rtps_rx_ctx* c);
// bumped by every rtps_rx_set_readers / set_match_table / set_topics
uint64_t rtps_ctx_readers_version(const rtps_rx_ctx* c);
// The writers an owner table covers: the writer GUIDs of the context's proxies (16 bytes each,
// writer-set order) and, by_topic, a group per writer (the smallest writer index of its group):
// writers whose target readers share a topic cache (a configured topic, or a reader's own) are
// one group; otherwise every writer is its own group.
void rtps_ctx_owner_writers(const rtps_rx_ctx* c, bool by_topic, std::vector<uint8_t>& guids,
                            std::vector<uint32_t>& group);
