// rtps_frag.h — internal interface of the DataFrag reassembly (rtps_frag.hip)
// used by the C ABI in rtps_rx.hip.  Not installed; see include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"
#include "rtps_readers.h"

struct FragState;
// Which DATA_FRAG records a batch assembles and under which reader (rtps_frag.hip, "Assembly keys"):
// mode 0 no readers (every one that passes, one assembler per writer); mode 1 readers whose target
// sets hold at most one reader (looked up in rt, Lifespans in life); mode 2 an expanded batch (one copy
// per target reader, the reader word in reader_id).
struct FragSel {
  uint32_t mode;
  uint32_t any_life;
  ReaderDev rt;
  const int64_t* life;   // [65536] Lifespan of each reader slot in Duration ticks, INT64_MAX: none
  uint64_t recv_ticks;   // the batch's Timestamp::now() as ticks
};  // persistent device state of one context (writers, pending buffers)

// Creates the state lazily on first use (device `device`); returns nullptr on
// allocation failure.
FragState* rtps_frag_state_new(int device);
void rtps_frag_state_free(FragState* s);
// Drops writers and pending buffers (asynchronous on `stream`).
int rtps_frag_state_reset(FragState* s, hipStream_t stream);
// One batch (asynchronous on `stream`); returns an rtps_rx_status code.  sel: the
// records assembled and their reader word.  emap (optional): position -> record of
// the parse, for an expanded batch (the samples' rec_idx go through it).
int rtps_frag_assemble(FragState* s, hipStream_t stream, const uint8_t* arena, uint64_t arena_len,
                       const uint64_t* dgram_off, const rtps_record* records, const uint64_t* n_records,
                       uint64_t max_records, const rtps_frag_out* out, const FragSel& sel, const uint32_t* emap);
// The clock stamped on buffers the next batches create or extend.
void rtps_frag_set_clock(FragState* s, uint64_t now);
void rtps_frag_set_sort(FragState* s, int mode);  // tests: 1 = rocprim device sort always
// Drops the carried buffers last modified before expire_before; the live count
// goes to the device u64 *n_pending (asynchronous on `stream`).
int rtps_frag_gc(FragState* s, hipStream_t stream, uint64_t expire_before, uint64_t* n_pending);
