"""MI355X-native MapAnything inference engine (drop-in for `mapanything` of facebookresearch/map-anything's
feed-forward path).  `from mapanything.models import MapAnything`."""

__version__ = "0.1.0"
