// rtps_cdr.h — internal interface between the C ABI (rtps_rx.hip) and the
// CDR decode kernel (rtps_cdr.hip).  Not installed; see include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtps_rx.h"

struct CdrProg {  // passed by value as a kernel argument (wave-uniform)
  rtps_cdr_op ops[RTPS_CDR_MAX_OPS];
  uint32_t n_ops;
  uint32_t row_bytes;
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
};

// Validates nothing (the caller does); returns 0 or -1 on a launch error.
int rtps_cdr_launch(hipStream_t s, const CdrProg& P, const CdrArgs& a, uint32_t max_blocks);
