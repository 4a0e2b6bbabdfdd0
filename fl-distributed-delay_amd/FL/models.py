"""Drop-in for the reference's FL/models.py (models.py:11-108).

The modules keep the reference's parameter sets, construction order (so torch's default init
under a given seed is identical) and state_dict keys.  They are the parameter containers of the
simulation; the FL hot path never runs their `forward` -- Worker.fwd_bkwd (FL/agents.py) drives
the HIP kernels of libflsim.so on a flat copy of the parameters.  `forward` is kept as the
model definition (e.g. for evaluation helpers).
"""
import math

import torch.nn as nn
import torch.nn.functional as F


class PerformantNet1(nn.Module):
    """models.py:11-47 -- 6 conv3x3(pad 2)+ReLU, 3 maxpool2, dropout .25/.5, 3 linear."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 48, 3, padding=(2, 2))
        self.conv2 = nn.Conv2d(48, 48, 3, padding=(2, 2))
        self.pool1 = nn.MaxPool2d(2, 2)
        self.dropout1 = nn.Dropout(p=0.25)
        self.conv3 = nn.Conv2d(48, 96, 3, padding=(2, 2))
        self.conv4 = nn.Conv2d(96, 96, 3, padding=(2, 2))
        self.conv5 = nn.Conv2d(96, 192, 3, padding=(2, 2))
        self.conv6 = nn.Conv2d(192, 192, 3, padding=(2, 2))
        self.linear1 = nn.Linear(9408, 512)
        self.dropout2 = nn.Dropout(p=0.5)
        self.linear2 = nn.Linear(512, 256)
        self.linear3 = nn.Linear(256, 10)

    def forward(self, x):
        bs = x.shape[0]
        x = F.relu(self.conv2(F.relu(self.conv1(x))))
        x = self.dropout1(self.pool1(x))
        x = F.relu(self.conv4(F.relu(self.conv3(x))))
        x = self.dropout1(self.pool1(x))
        x = F.relu(self.conv6(F.relu(self.conv5(x))))
        x = self.dropout1(self.pool1(x)).view(bs, -1)
        x = self.dropout2(F.relu(self.linear1(x)))
        x = self.dropout2(F.relu(self.linear2(x)))
        return self.linear3(x)


class VGG(nn.Module):
    """models.py:50-75 (configs[4]'s larger CNN; vgg11() runs on the flsim_vgg11_* HIP engine)."""

    def __init__(self, features):
        super().__init__()
        self.features = features
        self.classifier = nn.Sequential(
            nn.Dropout(), nn.Linear(512, 512), nn.ReLU(True),
            nn.Dropout(), nn.Linear(512, 512), nn.ReLU(True), nn.Linear(512, 10))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
                m.bias.data.zero_()

    def forward(self, x):
        return self.classifier(self.features(x).view(x.size(0), -1))


CFG_A = [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"]


def make_layers(cfg, batch_norm=False):
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            conv = nn.Conv2d(c, v, kernel_size=3, padding=1)
            layers += [conv, nn.BatchNorm2d(v), nn.ReLU(inplace=True)] if batch_norm else \
                [conv, nn.ReLU(inplace=True)]
            c = v
    return nn.Sequential(*layers)


cfg = {"A": CFG_A}


def vgg11():
    return VGG(make_layers(CFG_A))


def vgg11_bn():
    return VGG(make_layers(CFG_A, batch_norm=True))
