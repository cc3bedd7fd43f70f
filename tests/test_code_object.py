"""Resource checks on the gfx950 code objects inside libmapa.so (CPU only: the objects are read from the file).

The main loops of the LDS-DMA kernels wait for their staging with counted `s_waitcnt vmcnt(N)` written by hand
(gemm_big.hip, conv_halo.hip, attention.hip).  A VGPR spill inside such a loop adds scratch memory operations the
count does not know about, so every kernel whose loop relies on a counted wait must use no scratch at all; the
other kernels are allowed none either, so a spill anywhere shows up here first.  Read from the code
object's AMDGPU metadata note (`.private_segment_fixed_size`, `.vgpr_spill_count`) with llvm-readelf."""

import os
import re
import struct
import subprocess

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "map-anything_amd", "mapanything", "_lib", "libmapa.so")
READELF = "/opt/rocm/llvm/bin/llvm-readelf"
OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(data):
    """gfx950 ELF images of every clang offload bundle in the shared object (one bundle per translation unit)."""
    out, pos = [], 0
    while True:
        i = data.find(BUNDLE_MAGIC, pos)
        if i < 0:
            return out
        (count,) = struct.unpack_from("<Q", data, i + 24)
        off = i + 32
        for _ in range(count):
            o, size, tlen = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24: off + 24 + tlen].decode()
            off += 24 + tlen
            if "amdgcn" in triple:
                assert "gfx950" in triple, triple
                out.append(data[i + o: i + o + size])
        pos = i + len(BUNDLE_MAGIC)


@pytest.fixture(scope="module")
def code_object_files(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.skip("libmapa.so not built")
    if not (os.path.exists(READELF) and os.path.exists(OBJDUMP)):
        pytest.skip("llvm-readelf / llvm-objdump not available")
    objs = _code_objects(open(LIB, "rb").read())
    assert objs, "no gfx950 code object in libmapa.so"
    d = tmp_path_factory.mktemp("co")
    paths = []
    for n, co in enumerate(objs):
        p = d / f"co{n}.elf"
        p.write_bytes(co)
        paths.append(p)
    return paths


@pytest.fixture(scope="module")
def kernels(code_object_files):
    res = {}
    for p in code_object_files:
        notes = subprocess.run([READELF, "--notes", str(p)], check=True, capture_output=True, text=True).stdout
        # one metadata map per kernel: .name comes after the resource fields of the same map
        for blk in re.split(r"\n\s+- \.", notes):
            m = re.search(r"\.name:\s+(\S+)", blk)
            if not m or ".private_segment_fixed_size" not in blk:
                continue
            scratch = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1))
            spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", blk).group(1))
            res[m.group(1)] = (scratch, spill)
    return res


def test_every_kernel_metadata_read(kernels):
    names = " ".join(kernels)
    for k in ("gemm_big_kernel", "conv_halo_kernel", "attn_fwd_bf16", "gemm_sk_kernel", "layernorm"):
        assert k in names, f"no {k} in the code objects"
    assert len(kernels) >= 60


def test_no_scratch_in_any_kernel(kernels):
    bad = {k: v for k, v in kernels.items() if v != (0, 0)}
    assert not bad, "kernels with scratch (bytes, vgpr spills): " + "; ".join(f"{k}: {v}" for k, v in bad.items())


def test_no_packed_fp32_instructions(code_object_files):
    """Every object is built with the packed-fp32-ops target feature off (csrc/Makefile): a v_pk_mul_f32 whose two
    halves read each other's source register gave wrong low halves in lanes 48-63 on MI355X (Determinism).
    No v_pk_{add,mul,fma}_f32 may appear in any kernel."""
    bad = []
    for p in code_object_files:
        dis = subprocess.run([OBJDUMP, "-d", str(p)], check=True, capture_output=True, text=True).stdout
        bad += [ln.strip() for ln in dis.splitlines() if re.search(r"\bv_pk_(add|mul|fma)_f32\b", ln)]
    assert not bad, f"{len(bad)} packed f32 instructions, e.g. {bad[:3]}"
