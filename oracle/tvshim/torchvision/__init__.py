"""Container-only torchvision stand-in used by oracle/gen_golden.py to import the
reference REV model code (REV/models/backbone.py imports torchvision, which is not
installed in this image).  This restates torchvision's ResNet-50 v1.5 structure and
state_dict key names; it is test infrastructure and never ships with the product.
Pinned version statement: REV/README.md:5 asks for torchvision>=0.6 (unpinned);
"0.8.0" is reported so REV/utils/misc.py:21 skips the removed private imports."""
__version__ = "0.8.0"
from . import models, ops  # noqa: F401


def _is_tracing():
    return False
