"""The C-ABI library loads and exports every symbol include/mapa.h declares; argument checks work without a
GPU (no compute calls here)."""

import ctypes
import os
import re

import pytest

from conftest import REPO


def _declared():
    txt = open(os.path.join(REPO, "include", "mapa.h")).read()
    return sorted(set(re.findall(r"\b(mapa_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def L():
    from mapanything import _native

    return _native.load_library()


def test_exports_every_declared_symbol(L):
    from mapanything import _native

    declared = _declared()
    assert len(declared) >= 18
    for sym in declared:
        assert hasattr(L, sym), f"libmapa.so lacks {sym}"
    assert set(declared) == set(_native.EXPORTED)


def test_version_and_error_channel(L):
    from mapanything import _native

    assert L.mapa_version() >= 1
    d = _native.GemmDesc()
    d.dtype, d.M, d.N, d.K = _native.BF16, 64, 64, 12  # K not a multiple of 8 -> rejected before any launch
    rc = L.mapa_gemm(ctypes.byref(d), None)
    assert rc != 0
    assert b"K=12" in L.mapa_last_error()
    a = _native.AttnDesc()
    assert L.mapa_attention(ctypes.byref(a), None) != 0
    assert b"bad shape" in L.mapa_last_error()


def test_product_path_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mapanything import _native

    with pytest.raises(_native.NativeError):
        _native.lib()
