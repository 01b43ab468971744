from .resnet import resnet50  # noqa: F401
from . import _utils  # noqa: F401
