"""Pin the CPU oracle (oracle/mapa_oracle.py) against fixtures produced by the REAL reference
(tests/golden/make_golden.py).  Same synthetic weights, same seeded inputs; fp32 both sides, so the only
differences are ATen op-grouping rounding: tolerance 2e-5 rel-L2 (measured ~1e-6)."""

import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2
from tests_helpers import CASES, VARIANT_CASES, make_views, variant_config

TOL = 2e-5

@pytest.fixture(scope="module")
def oracle(synthetic_sd):
    from oracle.mapa_oracle import MapAnythingOracle

    torch.set_num_threads(min(8, os.cpu_count()))
    return MapAnythingOracle(synthetic_sd)


def _steps(name):
    meta = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))
    return meta[name]["steps_out_tap_dpt"]


def _oracle_for(name, oracle):
    if name not in VARIANT_CASES:
        return oracle, CASES[name]
    from mapanything.models.mapanything.spec import InfoSharingSpec, canonical_spec
    from mapanything.utils.synthetic import synthetic_state_dict
    from oracle.mapa_oracle import MapAnythingOracle

    cfg, case = variant_config(name)
    info = InfoSharingSpec.from_config(cfg["info_sharing_config"])
    return MapAnythingOracle(synthetic_state_dict(canonical_spec(info)), info), case


@pytest.mark.parametrize("name", ["cfg1_224", "mm_224", "mixed_224", "ns_280x392", "one_224", "v2_518",
                                  *VARIANT_CASES])
def test_oracle_matches_reference(oracle, golden, name):
    g = golden(name)
    out_step, tap_step, dpt_step = _steps(name)
    oracle, case = _oracle_for(name, oracle)
    with torch.no_grad():
        preds = oracle.infer(make_views(case))
    taps = oracle.taps
    checked = 0
    for key, ref in g.items():
        if key.startswith("out_"):
            k = key[4:]
            mine = torch.stack([p[k].float() for p in preds], 0).numpy()
            if mine.ndim >= 4 and k not in ("intrinsics", "camera_poses"):
                mine = mine[:, :, ::out_step, ::out_step]
        elif key == "tap_encoder":
            mine = taps["encoder"].numpy()[:, :, ::tap_step, ::tap_step]
        elif key == "tap_fused_nhwc":
            mine = taps["fused_nhwc"].numpy()[:, ::tap_step, ::tap_step, :]
        elif key.startswith("tap_aat_"):  # final + the taps, named by block index
            mine = taps[key[4:]].numpy()[:, :, :, ::tap_step, ::tap_step]
        elif key == "tap_dpt_feature":
            mine = taps["dpt_feature"].numpy()[:, :, ::dpt_step, ::dpt_step]
        else:
            mine = taps[key[4:]].numpy()
        assert mine.shape == ref.shape, (key, mine.shape, ref.shape)
        err = rel_l2(mine, ref)
        assert err < TOL, f"{name}:{key} rel-L2 {err:.3e}"
        checked += 1
    assert checked >= 15


def test_oracle_rope2d_matches_reference_fixture():
    """oracle.rope2d restates the reference's RoPE2D (pos_embed.py:101-155); fixture from the reference itself
    (tests/golden/make_rope_golden.py)."""
    import numpy as np

    from oracle.mapa_oracle import rope2d

    g = np.load(os.path.join(GOLDEN, "golden_rope2d.npz"))
    assert np.array_equal(rope2d(g["grid_tokens"], g["grid_pos"]).numpy(), g["grid_out"])
    for base in (100, 10000):
        got = rope2d(g["rand_tokens"], g["rand_pos"], base=float(base)).numpy()
        assert np.array_equal(got, g[f"rand_out_base{base}"]), base
