"""Tests of the rejected passes for mixed traffic, which only
diagnostic builds of the library have (-DRTPS_DIAG_PASSES, csrc/diag/mixed_passes.inc).  Not
collected by the default suite (the file name does not match test_*.py); run it against such a
build:
    make -C rustdds-io_uring_amd/csrc variant NAME=passes VDEFS=-DRTPS_DIAG_PASSES
    RTPS_RX_LIB=$PWD/rustdds-io_uring_amd/variants/librtps_rx_passes.so RTPS_RX_DIAG_PASSES=1 \
        python -m pytest tests/diag_mixed_passes.py tests/test_gpu_parity.py -m gpu
"""
import numpy as np
import pytest

import oracle
from test_gpu_parity import rx, _parity  # noqa: F401  (the module's receiver fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lds", [False, True])
@pytest.mark.parametrize("limit", [0, 1])
def test_chained_fallback_to_fix_pass(rx, limit, lds):
    """Chained tiles that stop waiting for their predecessors (forced here with a
    poll limit of 0 or 1) are left to kernel B: the output is still bit-exact, for
    both chained passes (lane walk C: B tiles of 256 datagrams; LDS tiles D: of 32)."""
    import ctypes
    import rtps_rx
    L = rtps_rx.lib()
    L.rtps_rx_debug_set_chain_spin_limit.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    a, o, l = oracle.gen(oracle.WL_C3, 200000)
    rx.set_spec_hint(0)
    rx.debug_set_mixed_pass(lds)
    assert L.rtps_rx_debug_set_chain_spin_limit(rx._h, limit) == 0
    try:
        _parity(rx, a, o, l, f"C3 chained, poll limit {limit}")
        # scratch: u32 flag[4], then u32 info[tile] (INFO_WRITTEN = 1 << 30: written by the chained pass);
        tsz = 32 if lds else 256
        tiles = (len(l) + tsz - 1) // tsz
        words = 2 + (tiles + 1) // 2
        buf = np.zeros(words, dtype=np.uint64)
        L.rtps_rx_debug_scratch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        assert L.rtps_rx_debug_scratch(rx._h, buf.ctypes.data, words) == 0
        info = buf.view(np.uint32)[4:4 + tiles]
        left = int(((info >> 30) & 1 == 0).sum())
        assert left > 0, "no tile was left to kernel B: the fallback was not exercised"
    finally:
        L.rtps_rx_debug_set_chain_spin_limit(rx._h, 1 << 10)
        rx.debug_set_mixed_pass(2)
        rx.set_spec_hint(1)


def test_chained_words_across_sizes_and_epoch_wrap(rx):
    """The chained pass's look-back words are never zeroed: they carry the launch's
    epoch.  Chained batches of different sizes, run across the 32-bit epoch wrap
    (which zeroes everything once), stay bit-exact; item-pass batches in between
    leave the words alone."""
    import ctypes
    import rtps_rx
    L = rtps_rx.lib()
    L.rtps_rx_debug_set_chain_epoch.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    big = oracle.gen(oracle.WL_C3, 70 * 256 + 13)
    small = oracle.gen(oracle.WL_C3, 5 * 256 + 200)
    rx.set_spec_hint(0)
    try:
        assert L.rtps_rx_debug_set_chain_epoch(rx._h, 0xfffffffd) == 0
        for k, (a, o, l) in enumerate([big, small, big, small, big, big]):
            rx.debug_set_mixed_pass(2 if k == 3 else 0)
            _parity(rx, a, o, l, f"C3 chained #{k} ({len(l)} datagrams) across the epoch wrap")
    finally:
        rx.debug_set_mixed_pass(2)
        rx.set_spec_hint(1)


