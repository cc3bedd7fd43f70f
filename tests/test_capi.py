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


def test_descriptor_layouts_match_header(tmp_path):
    """ctypes GemmDesc / AttnDesc field offsets equal the C compiler's offsetof for include/mapa.h (the split
    operand outputs were appended to mapa_gemm_desc; a mismatch would shift every field after it)."""
    import shutil
    import subprocess

    from mapanything import _native

    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    fields = {"mapa_gemm_desc": _native.GemmDesc, "mapa_attn_desc": _native.AttnDesc}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mapa.h"', "int main(void) {"]
    for cname, cls in fields.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "off.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "off"
    subprocess.run([cc, "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {(a, b): int(c) for a, b, c in (ln.split() for ln in out if ln)}
    for cname, cls in fields.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[(cname, fname)] == getattr(cls, fname).offset, (cname, fname)
