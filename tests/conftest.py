"""Shared fixtures.

Three implementations of the same cmp.h C-ABI are loaded side by side:
  prod   airs-compression_amd/lib/libairscmp.so   (the MI355X product; GPU)
  orc    oracle/liborc.so                          (CPU restatement; checker)
  ref    oracle/_ref/libref.so                     (reference compiled from
         /root/reference; present only where it was built)
"""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "airs-compression_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORC_PATH = os.path.join(ORACLE_DIR, "liborc.so")
REF_PATH = os.path.join(ORACLE_DIR, "_ref", "libref.so")
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def load_pkg():
    if "airs_compression_amd" in sys.modules:
        return sys.modules["airs_compression_amd"]
    spec = importlib.util.spec_from_file_location(
        "airs_compression_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["airs_compression_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def orc(pkg):
    if not os.path.exists(ORC_PATH):
        subprocess.run(["make", "-C", ORACLE_DIR, "liborc.so"], check=True)
    return pkg.CmpLib(ORC_PATH)


@pytest.fixture(scope="session")
def ref(pkg):
    if not os.path.exists(REF_PATH):
        pytest.skip("oracle/_ref/libref.so not built (reference sources absent)")
    return pkg.CmpLib(REF_PATH)


@pytest.fixture(scope="session")
def prod(pkg):
    if not os.path.exists(pkg.LIB_PATH):
        pkg.build()
    return pkg.load()


@pytest.fixture(scope="session")
def orc_ext():
    """Extra (non-cmp.h) entry points of the oracle via ctypes."""
    import ctypes
    lib = ctypes.CDLL(ORC_PATH, mode=ctypes.RTLD_LOCAL)
    lib.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib.orc_synth_i32.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib.orc_select_rice_k.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib.orc_select_rice_k.restype = ctypes.c_uint32
    lib.orc_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    lib.orc_decode.restype = ctypes.c_uint32
    lib.orc_xxh32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    lib.orc_xxh32.restype = ctypes.c_uint32
    lib.orc_checksum_u16.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    lib.orc_checksum_u16.restype = ctypes.c_uint32
    lib.orc_set_counter.argtypes = [ctypes.c_uint64]
    lib.orc_get_counter.restype = ctypes.c_uint64
    lib.drv_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                            ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.drv_run.restype = ctypes.c_uint64
    return lib
