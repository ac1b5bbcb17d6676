// rtps_ctx.h — internal view of a parse context for the host-side loops built
// on the public C ABI (rtps_pump.cpp).  Not part of include/rtps_rx.h.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

struct rtps_rx_ctx;
hipStream_t rtps_ctx_stream(const rtps_rx_ctx* c);
int rtps_ctx_device(const rtps_rx_ctx* c);
uint32_t rtps_ctx_max_datagrams(const rtps_rx_ctx* c);
