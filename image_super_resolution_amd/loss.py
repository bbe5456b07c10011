"""Drop-in for utils/loss.py: gen_loss (perceptual + adversarial) and L1Loss.

The VGG feature extractor is vgg.TruncatedVGG19 (HIP forward + input
gradient); the feature-space L1/MSE and the BCE-with-logits terms are tiny
reductions over [N, 512, h/16, w/16] features and [N, 1] logits and stay on
PyTorch-ROCm ops.
"""
from __future__ import annotations

import torch
from torch import nn

from .vgg import TruncatedVGG19


class L1Loss(nn.Module):
    """utils/loss.py:32-39: sum(loss_weight * mean|a - b|).  The reference builds
    the weight as a Parameter of an int tensor, which fails on construction
    (`Parameter` of a LongTensor cannot require grad); here it is a float
    Parameter with the same value and key."""

    def __init__(self, lossweight=1):
        super().__init__()
        self.loss_weight = nn.parameter.Parameter(torch.tensor([float(lossweight)]))
        self.criterion = nn.L1Loss()

    def forward(self, inputs, ground_truth):
        return torch.sum(torch.mul(self.loss_weight, self.criterion(inputs, ground_truth)))


class gen_loss:
    """utils/loss.py:7-29."""

    def __init__(self, vgg_i=5, vgg_j=4, beta=1e-3, device='cuda', beforeAct=False, vgg_weights=None):
        self.vgg_net = TruncatedVGG19(vgg_i, vgg_j, beforeAct, weights=vgg_weights).to(device)
        for x in self.vgg_net.parameters():
            x.requires_grad = False
        self.vgg_net.eval()
        self.mse = L1Loss().to(device) if beforeAct else nn.MSELoss()
        self.bce = nn.BCEWithLogitsLoss()
        self.beta = beta

    def calc_contentLoss(self, sr_imgs: torch.Tensor, hr_imgs: torch.Tensor, sr_discriminated: torch.Tensor,
                         hr_features: torch.Tensor | None = None):
        """`hr_features`: vgg_net(hr_imgs) computed ahead, or a callable returning it once ready
        (trainer.train_srgan runs it on a second stream beside the VGG(sr) forward; `sr_discriminated`
        may be such a callable too); None computes it here as the reference does."""
        sr_imgs_in_vgg_space = self.vgg_net(sr_imgs)
        if callable(sr_discriminated):  # likewise made on a second stream (trainer.train_srgan)
            sr_discriminated = sr_discriminated()
        if hr_features is None:
            hr_features = self.vgg_net(hr_imgs)
        elif callable(hr_features):
            hr_features = hr_features()
        hr_imgs_in_vgg_space = hr_features.detach()
        content_loss = self.mse(sr_imgs_in_vgg_space, hr_imgs_in_vgg_space)
        adversarial_loss = self.bce(sr_discriminated, torch.ones_like(sr_discriminated))
        perceptual_loss = content_loss + self.beta * adversarial_loss
        return perceptual_loss, adversarial_loss, content_loss

    def calc_advLoss(self, sr_discriminated: torch.Tensor, hr_discriminated: torch.Tensor):
        return (self.bce(sr_discriminated, torch.zeros_like(sr_discriminated))
                + self.bce(hr_discriminated, torch.ones_like(hr_discriminated)))
