"""The drop-in C-ABI: the shared library loads and exports every function include/siddhi_amd.h declares."""
import ctypes
import os
import re

import siddhi_amd as sa

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "siddhi_amd.h")


def declared_functions():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdg_[a-z_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ["sdg_compile", "sdg_push", "sdg_push_device", "sdg_flush", "sdg_poll", "sdg_advance_time",
              "sdg_destroy"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(sa.library_path())
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_library_is_gfx950_code():
    # the offload bundle inside the .so must target gfx950
    blob = open(sa.library_path(), "rb").read()
    assert b"gfx950" in blob
