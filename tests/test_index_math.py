"""Bounds-checked CPU build of the kernels' work-assignment index math (SURVEY.md §5 race detection / sanitizers
row): tools/index_check.cpp includes map-anything_amd/csrc/index_math.h — the functions the HIP kernels call to map
a workgroup id to its GEMM tile, stream-K iteration range and slab slot, attention task and K/V chunk, halo-conv
block and conv K column — and checks coverage / bijectivity / bounds over every path shape (up to the 2 738 001-key
configs[4] attention layer) and random ones, built with g++ -fsanitize=address,undefined."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_index_math_under_sanitizers(tmp_path):
    exe = str(tmp_path / "index_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    os.path.join(REPO, "tools", "index_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "index math ok" in r.stdout
