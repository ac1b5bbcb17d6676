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
// The keys an owner table covers (16 bytes each): the writer GUIDs of the context's proxies
// (writer-set order) and, by_topic, one ENTITY KEY per entity set (OWNER_EKEY_PREFIX || the
// writer entity id: the records of writers without a proxy that some reader contains by entity
// id), each with a group (the smallest key index of its group): keys whose target readers share
// a topic cache (a configured topic, or a reader's own) are one group; otherwise every key is
// its own group.
constexpr uint8_t OWNER_EKEY_PREFIX = 0xff;  // the 12 prefix bytes of an entity key
void rtps_ctx_owner_keys(const rtps_rx_ctx* c, bool by_topic, std::vector<uint8_t>& keys,
                         std::vector<uint32_t>& group);
// rtps_rx_set_topics configured at least one topic
bool rtps_ctx_topics_configured(const rtps_rx_ctx* c);
// The owner-side exchanges (rtps_rx_shard_*) created on the context: the ingest refuses the
// topic caches while one of them splits a topic cache's writers over its ranks.
struct rtps_shard;
void rtps_ctx_shard_attach(rtps_rx_ctx* c, rtps_shard* s, bool attach);
bool rtps_ctx_topic_split(const rtps_rx_ctx* c);
bool rtps_shard_splits_topics(const rtps_shard* s);  // (rtps_shard.hip)
