"""Import harness for the read-only reference at /root/reference (fixture generation ONLY, never on the GPU box).

Recipe of SURVEY.md Appendix A: stub the non-arithmetic imports (omegaconf, torchvision, jaxtyping, cv2,
rerun, trimesh, viser, transformers), replace torch.hub.load with the vendored DINOv2 builder
(mapanything/models/external/dinov2/hub/backbones.py:21-66, pretrained=False: nothing is fetched) and
build `MapAnything(**configs/inference.json)` (model.py:96-231).
"""

import json
import os
import re
import sys
import types

REF = os.environ.get("MAPA_REFERENCE", "/root/reference")


class _Anything(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _AnyObj()


class _AnyObj:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _AnyObj()

    def __getattr__(self, name):
        return _AnyObj()

    def __getitem__(self, item):
        return _AnyObj()

    def __mro_entries__(self, bases):
        return (object,)


def _stub(name, **attrs):
    m = _Anything(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    class _Sub:
        def __getitem__(self, item):
            return object

    _stub("jaxtyping", Float=_Sub(), Int=_Sub(), Bool=_Sub(), Shaped=_Sub())

    class DictConfig(dict):
        pass

    class OmegaConf:
        @staticmethod
        def register_new_resolver(*a, **k):
            pass

        @staticmethod
        def to_container(x, *a, **k):
            return x

    _stub("omegaconf", DictConfig=DictConfig, OmegaConf=OmegaConf)
    tv = _stub("torchvision")
    tvt = _stub("torchvision.transforms", RandomErasing=_AnyObj, Compose=_AnyObj, ToTensor=_AnyObj,
                Normalize=_AnyObj)
    tv.transforms = tvt
    _stub("torchvision.transforms.functional")
    _stub("torchvision.utils")
    for n in ("cv2", "rerun", "trimesh", "viser", "viser.transforms"):
        _stub(n)

    class PretrainedConfig:
        def __init__(self, *a, **k):
            pass

    _stub("transformers")
    _stub("transformers.activations", ACT2FN={})
    _stub("transformers.configuration_utils", PretrainedConfig=PretrainedConfig)


def load_reference():
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import torch

    from mapanything.models.external.dinov2.hub import backbones  # noqa: E402

    torch.hub.load = lambda repo, name, *a, **k: getattr(backbones, name)(pretrained=False)
    from mapanything.models.mapanything.model import MapAnything  # noqa: E402

    return MapAnything


def reference_config():
    txt = open(os.path.join(REF, "configs", "inference.json")).read()
    txt = re.sub(r"//[^\n]*", "", txt)
    return json.loads(txt)


def build_reference_model():
    MapAnything = load_reference()
    model = MapAnything(**reference_config())
    return model.eval()
