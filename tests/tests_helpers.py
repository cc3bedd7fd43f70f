"""Shared helpers for the test-suite (no reference access: the released config is committed as a fixture)."""

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def released_config():
    """configs/inference.json of the reference (committed copy: tests/golden/inference_config.json)."""
    with open(os.path.join(HERE, "golden", "inference_config.json")) as f:
        return json.load(f)
