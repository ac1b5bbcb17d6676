// rtps_cdr.h — internal interface between the C ABI (rtps_rx.hip) and the
// CDR decode kernel (rtps_cdr.hip).  Not installed; see include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"

constexpr uint32_t CDR_MAX_SLOTS = 144;  // op slots + zero gaps + segments (kernel-argument budget)
constexpr uint8_t CDR_SLOT_ZERO = 0;     // gap between op slots
constexpr uint8_t CDR_SLOT_SEG = 0x10;   // merged run of op slots, copied as one block for LE records
constexpr uint8_t CDR_IN_SEG = 1;        // flag: op slot covered by a segment (written here only for
                                         // records that are not decoded little-endian)

// One write-phase slot of the row: `dwords` 4-byte words at out_off.
//
// Segment: a run of >= 2 consecutive ops, all PRIM/ARRAY of 4/8-byte elements
// at wire offsets known on the host (no STRING/SEQ before them), whose row
// slots and wire bytes are both contiguous.  For a little-endian record the run
// is one memcpy of dwords*4 bytes from value + wire_off.
struct CdrSlot {
  uint8_t kind;   // rtps_cdr_op_kind, CDR_SLOT_ZERO or CDR_SLOT_SEG
  uint8_t size;   // primitive size (SEG: 4)
  uint8_t flags;  // CDR_IN_SEG
  uint8_t _r;
  uint16_t op;    // decode op index (position / length table row)
  uint16_t _r2;
  uint32_t out_off;
  uint32_t dwords;
  uint32_t count;  // PRIM 1, ARRAY count; SEG: wire offset of the run in the value
};

struct CdrProg {  // passed by value as a kernel argument (wave-uniform)
  rtps_cdr_op ops[RTPS_CDR_MAX_OPS];
  CdrSlot slots[CDR_MAX_SLOTS];
  uint32_t n_ops;
  uint32_t n_slots;
  uint32_t row_bytes;
  uint32_t lds_per_wave;  // bytes of the per-wave LDS table
};
struct CdrArgs {
  const uint8_t* arena;
  uint64_t arena_len;
  const uint64_t* dgram_off;
  const rtps_record* records;
  const uint64_t* n_records;
  uint64_t max_records;
  uint8_t* rows;
  uint8_t* row_status;
  // list mode (list != nullptr): row k decodes record *(u32*)(list + k * list_stride), for
  // k < min(*n_list, max_list); otherwise row r decodes record r
  const uint8_t* list;
  uint32_t list_stride;
  const uint64_t* n_list;
  uint64_t max_list;
};

// Composite programs (SEQ_BEGIN / ARRAY_BEGIN ... END, include/rtps_rx.h): one lane
// decodes one row, following the program with a stack of open elements.
struct CdrNest {  // kernel argument
  rtps_cdr_op ops[RTPS_CDR_MAX_OPS];
  uint8_t match[RTPS_CDR_MAX_OPS];    // BEGIN k -> its END; END -> its BEGIN
  uint8_t zero_el[RTPS_CDR_MAX_OPS];  // BEGIN k: the element reads no wire bytes (it cannot fail)
  uint32_t n_ops;
  uint32_t row_bytes;
};
// true if the program has composite ops
bool rtps_cdr_is_composite(const rtps_cdr_op* prog, uint32_t n_ops);
// Validates a composite program (op kinds and sizes, slots inside their container and
// not overlapping, BEGIN/END matched, depth <= RTPS_CDR_MAX_DEPTH) and fills N.
bool rtps_cdr_build_nested(const rtps_cdr_op* prog, uint32_t n_ops, uint32_t row_bytes, CdrNest& N);
int rtps_cdr_launch_nested(hipStream_t s, const CdrNest& N, const CdrArgs& a, uint32_t max_blocks);

// Builds the slot list from validated ops (host).  Returns false if slots overlap
// or leave the row.
bool rtps_cdr_build_slots(CdrProg& P);
// Launches the decode; returns 0 or -1 on a launch error.
int rtps_cdr_launch(hipStream_t s, const CdrProg& P, const CdrArgs& a, uint32_t cus);
