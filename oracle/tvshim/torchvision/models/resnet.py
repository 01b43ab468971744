"""ResNet-50 v1.5 (stride on the 3x3 conv of each bottleneck), torchvision key names."""
from torch import nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride, downsample, norm_layer, dilation=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = norm_layer(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=dilation,
                               dilation=dilation, bias=False)
        self.bn2 = norm_layer(width)
        self.conv3 = nn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = norm_layer(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, layers, norm_layer=None, replace_stride_with_dilation=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        dil = replace_stride_with_dilation or [False, False, False]
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self._cin, self._dil = 64, 1
        self.layer1 = self._stage(64, layers[0], 1, False, norm_layer)
        self.layer2 = self._stage(128, layers[1], 2, dil[0], norm_layer)
        self.layer3 = self._stage(256, layers[2], 2, dil[1], norm_layer)
        self.layer4 = self._stage(512, layers[3], 2, dil[2], norm_layer)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(2048, 1000)

    def _stage(self, width, blocks, stride, dilate, norm_layer):
        prev_dil = self._dil
        if dilate:
            self._dil *= stride
            stride = 1
        ds = None
        if stride != 1 or self._cin != width * 4:
            ds = nn.Sequential(nn.Conv2d(self._cin, width * 4, 1, stride=stride, bias=False),
                               norm_layer(width * 4))
        mods = [Bottleneck(self._cin, width, stride, ds, norm_layer, prev_dil)]
        self._cin = width * 4
        for _ in range(1, blocks):
            mods.append(Bottleneck(self._cin, width, 1, None, norm_layer, self._dil))
        return nn.Sequential(*mods)


def resnet50(pretrained=False, progress=True, **kw):
    # pretrained weights cannot be fetched offline; the flag is ignored on purpose
    return ResNet([3, 4, 6, 3], norm_layer=kw.get("norm_layer"),
                  replace_stride_with_dilation=kw.get("replace_stride_with_dilation"))
