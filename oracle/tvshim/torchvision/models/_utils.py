from collections import OrderedDict
from torch import nn


class IntermediateLayerGetter(nn.ModuleDict):
    """Keeps the children of `model` up to the last requested layer and returns the
    requested intermediate outputs (torchvision.models._utils semantics)."""

    def __init__(self, model, return_layers):
        wanted = dict(return_layers)
        kept = OrderedDict()
        pending = set(wanted)
        for name, child in model.named_children():
            kept[name] = child
            pending.discard(name)
            if not pending:
                break
        super().__init__(kept)
        self.return_layers = wanted

    def forward(self, x):
        out = OrderedDict()
        for name, module in self.items():
            x = module(x)
            if name in self.return_layers:
                out[self.return_layers[name]] = x
        return out
