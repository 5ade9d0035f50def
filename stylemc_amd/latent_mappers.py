"""Per-image latent mapper (latent_mappers.py:68-93): S rows T [B, 8, 512] -> delta [B, 8, 512].

State_dict-compatible with the reference's ``Mapper`` (``course_mapping`` / ``medium_mapping`` ->
``modulation_module_list.{0..4}.fc.{weight,bias}``), so ``mapper_<prompt>.pth`` files written by
train_latent_mapper.py load unchanged (generate_fromS.py:117-122).  What the reference computes:

  SubMapperModulation (latent_mappers.py:35-46): PixelNorm over dim 1 (e4e models/stylegan2/model.py
  PixelNorm: x * rsqrt(mean(x^2, dim=1) + 1e-8) -- on [B, 4, 512] that is the 4-row axis), then 5 x
  ModulationModule (:12-32 with embedding None): Linear(512, 512) -> LayerNorm([4, 512], no affine) ->
  LeakyReLU(neg_slope).  Mapper (:68-93): rows 0-3 through ``course_mapping``, rows 4-7 through
  ``medium_mapping``.  (The gamma/beta branches are commented out in the reference and never built.)

Small dense MLPs (8 x 512 per image): PyTorch-ROCm ops, off the synthesis hot path.
"""
import torch
import torch.nn.functional as F
from torch import nn


class ModulationModule(nn.Module):
    def __init__(self, layernum, neg_slope=0.01):
        super().__init__()
        self.layernum = layernum
        self.fc = nn.Linear(512, 512)
        self.neg_slope = neg_slope

    def forward(self, x):
        x = F.layer_norm(self.fc(x), [self.layernum, 512], eps=1e-5)
        return F.leaky_relu(x, self.neg_slope)


class SubMapperModulation(nn.Module):
    def __init__(self, layernum=4, neg_slope=0.01):
        super().__init__()
        self.layernum = layernum
        self.modulation_module_list = nn.ModuleList([ModulationModule(layernum, neg_slope) for _ in range(5)])

    def forward(self, x):
        x = x * torch.rsqrt(torch.mean(x ** 2, dim=1, keepdim=True) + 1e-8)
        for m in self.modulation_module_list:
            x = m(x)
        return x


class Mapper(nn.Module):
    def __init__(self, neg_slope=0.01):
        super().__init__()
        self.course_mapping = SubMapperModulation(neg_slope=neg_slope)
        self.medium_mapping = SubMapperModulation(neg_slope=neg_slope)

    def forward(self, x, embedding=None):
        return torch.cat([self.course_mapping(x[:, :4, :]), self.medium_mapping(x[:, 4:8, :])], dim=1)
