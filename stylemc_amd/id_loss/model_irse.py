"""ArcFace IR-SE50 backbone (id_loss/model_irse.py:10-49 + helpers.py:29-119 of the reference).

Module names match the reference's state_dict (``input_layer``, ``body.{k}.shortcut_layer`` /
``res_layer``, ``output_layer``) so ``model_ir_se50.pth`` loads unchanged.  Frozen, eval-mode, fp32 on
PyTorch-ROCm (MIOpen convs); 12.59 GFLOP per 112x112 face.
"""
import torch
from torch import nn

# (in_channels, depth, units) for num_layers = 50 / 100 / 152 (helpers.py:29-53)
STAGES = {
    50: [(64, 64, 3), (64, 128, 4), (128, 256, 14), (256, 512, 3)],
    100: [(64, 64, 3), (64, 128, 13), (128, 256, 30), (256, 512, 3)],
    152: [(64, 64, 3), (64, 128, 8), (128, 256, 36), (256, 512, 3)],
}


class PReLU(nn.PReLU):
    """nn.PReLU with the same parameter, but a where-form forward: with the slope frozen its backward is
    the input gradient only (ATen's fused prelu backward also reduces the slope gradient every call)."""

    def forward(self, x):
        return torch.where(x >= 0, x, x * self.weight.view(1, -1, 1, 1))


class Subsample(nn.Module):
    """MaxPool2d(kernel_size=1, stride=s) == every s-th pixel; as a strided view its backward is a cheap
    strided copy instead of ATen's max-pool index scatter."""

    def __init__(self, stride):
        super().__init__()
        self.stride = stride

    def forward(self, x):
        return x if self.stride == 1 else x[:, :, ::self.stride, ::self.stride]


class SEModule(nn.Module):
    def __init__(self, channels, reduction):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(channels, channels // reduction, kernel_size=1, padding=0, bias=False)
        self.relu = nn.ReLU(inplace=True)
        self.fc2 = nn.Conv2d(channels // reduction, channels, kernel_size=1, padding=0, bias=False)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        return x * self.sigmoid(self.fc2(self.relu(self.fc1(self.avg_pool(x)))))


class BottleneckIRSE(nn.Module):
    def __init__(self, in_channel, depth, stride, se=True):
        super().__init__()
        if in_channel == depth:
            self.shortcut_layer = Subsample(stride)
        else:
            self.shortcut_layer = nn.Sequential(nn.Conv2d(in_channel, depth, (1, 1), stride, bias=False),
                                                nn.BatchNorm2d(depth))
        layers = [nn.BatchNorm2d(in_channel), nn.Conv2d(in_channel, depth, (3, 3), (1, 1), 1, bias=False),
                  PReLU(depth), nn.Conv2d(depth, depth, (3, 3), stride, 1, bias=False), nn.BatchNorm2d(depth)]
        if se:
            layers.append(SEModule(depth, 16))
        self.res_layer = nn.Sequential(*layers)

    def forward(self, x):
        return self.res_layer(x) + self.shortcut_layer(x)


class _Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


class Backbone(nn.Module):
    def __init__(self, input_size=112, num_layers=50, mode="ir_se", drop_ratio=0.4, affine=True):
        super().__init__()
        assert input_size in (112, 224) and num_layers in STAGES and mode in ("ir", "ir_se")
        self.input_layer = nn.Sequential(nn.Conv2d(3, 64, (3, 3), 1, 1, bias=False), nn.BatchNorm2d(64),
                                         PReLU(64))
        grid = 7 if input_size == 112 else 14
        self.output_layer = nn.Sequential(nn.BatchNorm2d(512), nn.Dropout(drop_ratio), _Flatten(),
                                          nn.Linear(512 * grid * grid, 512), nn.BatchNorm1d(512, affine=affine))
        units = []
        for cin, depth, n in STAGES[num_layers]:
            units.append(BottleneckIRSE(cin, depth, 2, se=(mode == "ir_se")))
            units += [BottleneckIRSE(depth, depth, 1, se=(mode == "ir_se")) for _ in range(n - 1)]
        self.body = nn.Sequential(*units)
        self.channels_last = False

    def forward(self, x):
        if self.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        x = self.output_layer(self.body(self.input_layer(x)))
        return x / torch.norm(x, 2, 1, True)


def build_irse50(state_dict=None, seed=3, device="cuda"):
    from .. import synthetic
    net = Backbone(input_size=112, num_layers=50, drop_ratio=0.6, mode="ir_se")
    net.load_state_dict(state_dict if state_dict is not None else synthetic.seeded_state_dict(net, seed=seed))
    net = net.eval().requires_grad_(False).to(device)
    if str(device).startswith("cuda"):
        # MIOpen's fp32 convs are NHWC kernels: channels_last avoids a transpose pair around every conv
        net.channels_last = True
        net = net.to(memory_format=torch.channels_last)
    return net
