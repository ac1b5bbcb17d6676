"""The C++ host mirror (include/rtps_rx.hpp) builds here; on a GPU it parses a
C3 batch bit-exactly like the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "receiver_check.cpp")
LIBDIR = os.path.join(REPO, "rustdds-io_uring_amd")


def _build(tmp):
    exe = os.path.join(tmp, "receiver_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(REPO, "include"),
                    "-I", "/opt/rocm/include", SRC, "-o", exe, "-L", LIBDIR, "-lrtps_rx",
                    "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"],
                   check=True)
    return exe


def test_cpp_mirror_builds(tmp_path):
    assert os.path.exists(_build(str(tmp_path)))


@pytest.mark.gpu
def test_cpp_mirror_parity(tmp_path):
    exe = _build(str(tmp_path))
    arena, off, ln = oracle.gen(oracle.WL_C3, 5000)
    st, recs, _, _ = oracle.parse(arena, off, ln)
    for name, a in (("arena", arena), ("off", off), ("len", ln), ("status", st), ("records", recs),
                    ("own", np.frombuffer(oracle.OWN_PREFIX, np.uint8))):
        np.ascontiguousarray(a).tofile(os.path.join(tmp_path, f"{name}.bin"))
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
