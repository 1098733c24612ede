"""CPU checks of the drop-in boundary: the C-ABI library loads and exports exactly what
include/difacto_amd.h declares (no compute call — there is no GPU here)."""
import ctypes

import torch  # noqa: F401  (load torch's HIP runtime first, as difacto_amd._lib does)
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "difacto_amd.h")
LIB = os.path.join(ROOT, "difacto_amd", "libdifacto_amd.so")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int)\s+(dfx_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("dfx_localize", "dfx_fm_predict", "dfx_fm_calcgrad", "dfx_store_pull",
                 "dfx_store_push", "dfx_store_save", "dfx_store_load", "dfx_train_step"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from difacto_amd import _lib
    assert sorted(_lib.EXPORTED) == declared()


DIST_HEADER = os.path.join(ROOT, "include", "difacto_amd_dist.h")
DIST_LIB = os.path.join(ROOT, "difacto_amd", "libdfx_dist.so")


def dist_declared():
    src = open(DIST_HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int)\s+(dfx_\w+)\s*\(", src, re.M)))


def test_dist_library_exports_every_declared_symbol():
    """the split driver's C-ABI (libdfx_dist.so over libdifacto_amd.so and RCCL)"""
    ctypes.CDLL(LIB)
    lib = ctypes.CDLL(DIST_LIB)
    names = dist_declared()
    assert "dfx_split_store_submit" in names and "dfx_dist_rccl_ids" in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from difacto_amd import _lib
    assert sorted(_lib.DIST_EXPORTED) == names
    assert _lib.dist_lib().dfx_dist_rccl_id_bytes() == 128
