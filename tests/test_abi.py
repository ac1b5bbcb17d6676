"""C-ABI checks that need no GPU: the library builds, loads and exports
every entry point include/rtps_rx.h declares; the record layout agrees."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rtps_rx.h")
LIB = os.path.join(REPO, "rustdds-io_uring_amd", "librtps_rx.so")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|uint64_t|const char\*)\s+(rtps_(?:rx|udp)_\w+)\s*\(", text, re.M)))


def test_header_declares_api():
    fns = declared_functions()
    for f in ("rtps_rx_create", "rtps_rx_destroy", "rtps_rx_set_stream", "rtps_rx_set_match_table",
              "rtps_rx_parse_batch", "rtps_rx_sync", "rtps_rx_strerror", "rtps_rx_max_records_host",
              "rtps_rx_generate"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(LIB)
    for f in declared_functions():
        assert hasattr(lib, f), f"{f} not exported"


def test_host_helpers_without_gpu():
    import numpy as np
    import rtps_rx
    from rtps_rx.records import max_records
    lib = rtps_rx.lib()
    lens = np.array([0, 19, 20, 24, 1024, 65536, 65537], dtype=np.uint32)
    assert lib.rtps_rx_max_records_host(lens.ctypes.data, len(lens)) == max_records(lens)
    lib.rtps_rx_strerror.restype = ctypes.c_char_p
    assert lib.rtps_rx_strerror(-1) == b"invalid argument"
    # the library's host layout == the oracle's host layout (same generator)
    import oracle
    for wl in (1, 2, 3, 4):
        off, ln, size = rtps_rx.gen_layout(wl, 1000)
        a, o2, l2 = oracle.gen(wl, 1000)
        assert np.array_equal(off, o2) and np.array_equal(ln, l2)


def test_header_compiles_as_c_and_cxx(tmp_path):
    import subprocess
    src = tmp_path / "t.c"
    src.write_text('#include "rtps_rx.h"\nint main(void){return (int)sizeof(rtps_record) - 64;}\n')
    for cc, ext in (("gcc", "c"), ("g++", "cpp")):
        s2 = tmp_path / f"t.{ext}"
        s2.write_text(src.read_text())
        subprocess.run([cc, "-std=c11" if ext == "c" else "-std=c++17", "-I", os.path.join(REPO, "include"),
                        str(s2), "-o", str(tmp_path / f"t_{ext}")], check=True)
        assert subprocess.run([str(tmp_path / f"t_{ext}")]).returncode == 0


def test_product_has_no_oracle_dependency():
    """The product path must not route through the oracle / a CPU fallback."""
    pkg = os.path.join(REPO, "rustdds-io_uring_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(root, f)).read()
                assert "import oracle" not in txt and "rtps_oracle" not in txt, f
