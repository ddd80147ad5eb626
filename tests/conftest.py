"""Shared test setup: import paths, the `gpu` marker, oracle loaders.

The oracle (oracle/) is the checker only; the product under test is the HIP
library behind roce-sim_amd/roce_icrc.
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


_oracle_lib = None


def oracle_lib():
    """oracle/build/liboracle.so (built by `make -C oracle`)."""
    global _oracle_lib
    if _oracle_lib is None:
        path = ROOT / "oracle" / "build" / "liboracle.so"
        if not path.exists():
            import subprocess
            subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s"], check=True)
        lib = ctypes.CDLL(str(path))
        lib.oracle_icrc_bitwise.restype = ctypes.c_uint32
        lib.oracle_icrc_bitwise.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_icrc_sliced.restype = ctypes.c_uint32
        lib.oracle_icrc_sliced.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_icrc_batch.restype = ctypes.c_int
        lib.oracle_icrc_batch.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
            ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _oracle_lib = lib
    return _oracle_lib


def oracle_batch(buf, offsets=None, lens=None, stride=0, length=0, n=None, nthreads=None):
    """C oracle over a batch; returns (icrc u32[n], ok u8[n])."""
    lib = oracle_lib()
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = offsets.size
    out = np.zeros(n, np.uint32)
    ok = np.zeros(n, np.uint8)
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    rc = lib.oracle_icrc_batch(
        buf.ctypes.data,
        None if offsets is None else offsets.ctypes.data,
        None if lens is None else lens.ctypes.data,
        stride, length, n, out.ctypes.data, ok.ctypes.data, nthreads)
    assert rc == 0
    return out, ok


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on cuda:0 (gpu tests only)."""
    from roce_icrc import IcrcEngine
    e = IcrcEngine(0)
    yield e
    e.close()
