// rtps_topic.h — internal interface of the topic caches (rtps_topic.hip) used by the C
// ABI in rtps_rx.hip.  Not installed; see include/rtps_rx.h ("topic caches").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"

struct TopicState;  // per-topic insertion counters + the live (writer GUID, SN) index, batch scratch

TopicState* rtps_topic_state_new(int device);
void rtps_topic_state_free(TopicState* s);
// rtps_rx_set_topics: the topic table and the readers' topics; empties every cache.
// set_first / ent / n_sets: the context's target sets (host view), for the readers' flags.
int rtps_topic_configure(TopicState* s, const rtps_topic* topics, uint32_t n_topics, const rtps_topic_reader* readers,
                         uint32_t n_readers, const uint32_t* set_first, const rtps_target* ent, uint32_t n_sets,
                         hipStream_t st);
// After rtps_rx_set_readers: new readers / proxies (their private topics, which topics
// have one reader); fresh proxies may re-accept changes a topic still holds, so every
// topic checks each delivery against its live changes until those have aged out.
int rtps_topic_readers_changed(TopicState* s, const uint32_t* set_first, const rtps_target* ent, uint32_t n_sets,
                               hipStream_t st);
// Every topic cache emptied (rtps_rx_topic_reset).
int rtps_topic_reset(TopicState* s, hipStream_t st);
// The writer proxies were reset (rtps_rx_ingest_reset): the caches keep their changes, and
// fresh proxies may re-accept what a topic still holds, so every topic checks each delivery
// against its live changes until those have aged out (as after rtps_topic_readers_changed).
int rtps_topic_proxies_reset(TopicState* s, hipStream_t st);
// DDSCache::garbage_collect.
int rtps_topic_gc(TopicState* s, hipStream_t st);
// Topics rtps_rx_set_topics configured (0: every reader slot its own cache).
uint32_t rtps_topic_n_configured(const TopicState* s);
// The topic cache a reader slot's changes go to (its configured topic, else its own).
uint32_t rtps_topic_of_slot(const TopicState* s, uint16_t slot);
// TopicCache::add_change for every delivery of the batch, in order: sets or clears
// RTPS_DELIVERY_CACHED in del[k].flags (asynchronous).
// ovf (device u64, optional): the batch's ingest window overflows; non-zero = some samples were
// accepted without the proxies' duplicate check, so no delivery is stored unchecked ("certain"):
// every one is checked against the topic's live changes.
// gate (device u64, optional): the batch's kernels do nothing unless *gate != 0 when they run
// (queued ahead of the host's knowledge of whether the ingest path they follow runs).
int rtps_topic_apply(TopicState* s, hipStream_t st, const rtps_record* recs, const uint64_t* n_records,
                     uint64_t max_records, rtps_delivery* del, const uint64_t* n_del, uint64_t max_del,
                     const uint64_t* ovf = nullptr, const uint64_t* gate = nullptr);
