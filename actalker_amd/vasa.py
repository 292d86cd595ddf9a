"""VASA expression / head-pose encoders (the remainder): drop-in counterparts of
the reference's ResNet-GroupNorm encoders, run once per clip before the loop in modes 1 / 2.

  HeadPose_train   src/dataset/vasa_feature_v2.py:9-22    (Inference.py:159-163; ResNet18_GN, 6 outputs)
  ResNet18_GN      vasa_feature_v2.py:25-60               (BasicBlock :63-85, GroupNorm(32, C))
  HeadExpression   vasa_feature_v2.py:108-122             (Inference.py:147-157; ResNet50-GN, 512 outputs)
  ResNet_GN        vasa_feature_v2.py:168-206             (Bottleneck :125-160, GroupNorm(groups=1, C))
  vasa_prompts     Inference.py:486-500                   (expression + pose -> VASA prompt tokens)

Same class names, constructor arguments and parameter names as the reference (``state_dict`` loads with
``strict=True``; Inference.py:154 / :160 load the VASA checkpoint into them). The image tensors are
what the reference's ``vasa_transform`` produces (test_preprocess.py:184-200: 256x256, [0, 1]); the
cv2 / PIL cropping before it is preprocessing, out of scope here.

Compute runs in libactalker_hip.so on token-major NHWC rows: the 7x7 / stride-2 stems as an explicit
im2col (Cin = 3) + MFMA GEMM, every 3x3 conv on the implicit-GEMM MFMA kernel (stride 1 / 2), 1x1 convs
as dense GEMMs (stride 2 through a row gather of the even pixels), GroupNorm with ReLU and the block's
residual add fused into the normalisation's apply pass, the stem max-pool on its own kernel, the global
average pool as a per-image row mean, fc as a GEMM with fp32 output.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn as nn

from . import ops
from .modules import Conv2d, GroupNorm, Linear, Packed, _bf


def _even_pixel_index(H: int, W: int, stride: int, device) -> torch.Tensor:
    """Row indices (within one image) of the pixels a 1x1 / stride-s conv reads."""
    ys = torch.arange(0, H, stride)
    xs = torch.arange(0, W, stride)
    return (ys[:, None] * W + xs[None, :]).reshape(-1).to(device=device, dtype=torch.int32)


def _conv1x1(conv: Conv2d, x: torch.Tensor, B: int, H: int, W: int, stride: int) -> torch.Tensor:
    if stride != 1:
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        sub = torch.empty((B * Ho * Wo, x.shape[1]), device=x.device, dtype=torch.bfloat16)
        ops.gather_rows(x, _even_pixel_index(H, W, stride, x.device), B, H * W, sub, Ho * Wo)
        x = sub
    return ops.gemm(x, conv.w1(), bias=conv.b())


def _gn(norm: GroupNorm, x: torch.Tensor, rows_per_image: int, relu: bool, residual=None) -> torch.Tensor:
    g, b = norm.gb()
    return ops.groupnorm(x, g, b, norm.eps, rows_per_image, groups=norm.num_groups, relu=relu, residual=residual)


class _Stem(Conv2d):
    """7x7 / stride 2 / pad 3 conv on 3 channels: im2col (K = 147, padded to 152) + GEMM."""

    def wk(self):
        def f():
            w = self.weight.detach().permute(0, 2, 3, 1).reshape(self.out_channels, -1)   # (Cout, 7*7*3), k = tap*3 + c
            kp = (w.shape[1] + 7) // 8 * 8
            return _bf(torch.nn.functional.pad(w, (0, kp - w.shape[1])))
        return self._pk("wk", f)

    def run(self, x, B, H, W):
        k, s, p = self.kernel_size[0], self.stride[0], self.padding[0]
        cols = ops.im2col(x, B, H, W, k, k, s, p)
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        return ops.gemm(cols, self.wk(), bias=self.b()), Ho, Wo


class _EncoderBase(nn.Module):
    def invalidate_kernel_cache(self):
        for m in self.modules():
            if hasattr(m, "_acth_invalidate"):
                m._acth_invalidate()

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        self.invalidate_kernel_cache()
        return r

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        r = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.invalidate_kernel_cache()
        return r


# ------------------------------------------------------------------------------------------ ResNet18-GN
class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = GroupNorm(32, planes)
        self.conv2 = Conv2d(planes, planes * self.expansion, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = GroupNorm(32, planes * self.expansion)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes * self.expansion:
            self.shortcut = nn.Sequential(
                Conv2d(in_planes, planes * self.expansion, kernel_size=1, stride=stride, bias=False),
                GroupNorm(32, planes * self.expansion))
        self.stride = stride

    def run(self, x, B, H, W):
        s = self.stride
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        h = ops.conv3x3(x, self.conv1.w3(), B, H, W, stride=s)
        h = _gn(self.bn1, h, Ho * Wo, relu=True)
        h = ops.conv3x3(h, self.conv2.w3(), B, Ho, Wo)
        if len(self.shortcut) == 0:
            sc = x
        else:
            sc = _gn(self.shortcut[1], _conv1x1(self.shortcut[0], x, B, H, W, s), Ho * Wo, relu=False)
        # out = relu(bn2(conv2(.)) + shortcut(x)): residual add + ReLU fused into the GN apply
        return _gn(self.bn2, h, Ho * Wo, relu=True, residual=sc), Ho, Wo


class ResNet18_GN(_EncoderBase):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.in_planes = 64
        self.conv1 = _Stem(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = GroupNorm(32, 64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(BasicBlock, 64, 2, stride=1)
        self.layer2 = self._make_layer(BasicBlock, 128, 2, stride=2)
        self.layer3 = self._make_layer(BasicBlock, 256, 2, stride=2)
        self.layer4 = self._make_layer(BasicBlock, 512, 2, stride=2)
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = Linear(512 * BasicBlock.expansion, num_classes)

    def _make_layer(self, block, planes, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _resnet_forward(self, x, self.bn1, self.avg_pool)


# ------------------------------------------------------------------------------------------ ResNet50-GN
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64):
        super().__init__()
        width = int(planes * (base_width / 64.)) * groups
        if groups != 1:
            raise ValueError("grouped 3x3 convolutions are not used by the VASA encoders (groups=1)")
        self.conv1 = Conv2d(inplanes, width, kernel_size=1, bias=False)
        self.gn1 = GroupNorm(groups, width)
        self.conv2 = Conv2d(width, width, kernel_size=3, stride=stride, padding=1, bias=False, groups=groups)
        self.gn2 = GroupNorm(groups, width)
        self.conv3 = Conv2d(width, planes * self.expansion, kernel_size=1, bias=False)
        self.gn3 = GroupNorm(groups, planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def run(self, x, B, H, W):
        s = self.stride
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        h = _gn(self.gn1, ops.gemm(x, self.conv1.w1()), H * W, relu=True)
        h = _gn(self.gn2, ops.conv3x3(h, self.conv2.w3(), B, H, W, stride=s), Ho * Wo, relu=True)
        h = ops.gemm(h, self.conv3.w1())
        if self.downsample is None:
            res = x
        else:
            res = _gn(self.downsample[1], _conv1x1(self.downsample[0], x, B, H, W, s), Ho * Wo, relu=False)
        return _gn(self.gn3, h, Ho * Wo, relu=True, residual=res), Ho, Wo


class ResNet_GN(_EncoderBase):
    def __init__(self, block, layers, num_classes=1000, groups=1, base_width=64):
        super().__init__()
        self.inplanes = 64
        self.conv1 = _Stem(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.gn1 = GroupNorm(groups, 64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0], groups=groups, base_width=base_width)
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2, groups=groups, base_width=base_width)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2, groups=groups, base_width=base_width)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2, groups=groups, base_width=base_width)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1, groups=1, base_width=64):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                GroupNorm(groups, planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, groups, base_width)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=groups, base_width=base_width))
        return nn.Sequential(*layers)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _resnet_forward(self, x, self.gn1, self.avgpool)


def resnet50_gn(**kwargs):
    return ResNet_GN(Bottleneck, [3, 4, 6, 3], **kwargs)


def _resnet_forward(net, x: torch.Tensor, stem_norm: GroupNorm, pool: nn.Module) -> torch.Tensor:
    """(B, 3, H, W) image -> (B, num_classes) fp32 logits, every op on the HIP kernels."""
    if not x.is_cuda:
        raise RuntimeError("actalker_amd VASA encoders run on the MI355X HIP kernels only; move them to a GPU")
    B, _, H, W = x.shape
    with torch.no_grad():
        t = ops.nchw_to_tokens(x.float())                                  # (B*H*W, 3) bf16
        h, H, W = net.conv1.run(t, B, H, W)
        h = _gn(stem_norm, h, H * W, relu=True)
        mp = net.maxpool
        h = ops.maxpool2d(h, B, H, W, mp.kernel_size, mp.stride, mp.padding)
        H, W = (H + 2 * mp.padding - mp.kernel_size) // mp.stride + 1, (W + 2 * mp.padding - mp.kernel_size) // mp.stride + 1
        for layer in (net.layer1, net.layer2, net.layer3, net.layer4):
            for blk in layer:
                h, H, W = blk.run(h, B, H, W)
        pooled = ops.frame_mean(h, B, H * W, 1)                             # AdaptiveAvgPool2d((1, 1))
        return ops.gemm(pooled, net.fc.w(), bias=net.fc.b(), out_f32=True)


# ------------------------------------------------------------------------------------------ heads
class HeadPose_train(_EncoderBase):
    def __init__(self):
        super().__init__()
        self.head_pose_net = ResNet18_GN(num_classes=6)

    def forward(self, x: torch.Tensor) -> Dict[str, torch.Tensor]:
        head_pose = self.head_pose_net(x)
        rotation = torch.sigmoid(head_pose[:, :3]) * 360. - 180
        translation = torch.sigmoid(head_pose[:, 3:]) * 4. - 2
        return {"rotation": rotation, "translation": translation}


class HeadExpression(_EncoderBase):
    def __init__(self, out_feat_dim=1024):
        super().__init__()
        self.resnet50 = resnet50_gn(num_classes=out_feat_dim)

    def forward(self, source_image: torch.Tensor) -> torch.Tensor:
        return self.resnet50(source_image)


def vasa_prompts(expression_model: HeadExpression, pose_model: HeadPose_train, vasa_linear, crop_face: torch.Tensor,
                 pose_image: torch.Tensor):
    """Inference.py:486-500: expression (512) + [rotation, translation * 0] -> vasa_linear(512 -> 1018) ++
    pose (6) = 1024-wide VASA prompts, and the unconditional prompts vasa_linear(0) ++ 0.
    ``crop_face`` / ``pose_image``: (N, 3, 256, 256) in [0, 1] (the pose image is mapped to [-1, 1] here,
    as at Inference.py:491)."""
    feat = expression_model(crop_face)
    pose = pose_model(pose_image * 2 - 1.0)
    full = torch.cat([feat.float(), pose["rotation"], pose["translation"] * 0.], dim=-1)
    prompts, pose_fea = full[..., :-6], full[..., -6:]
    uncond = vasa_linear(torch.zeros_like(prompts))
    prompts = vasa_linear(prompts)
    prompts = torch.cat([prompts.float(), pose_fea], dim=-1)
    uncond = torch.cat([uncond.float(), torch.zeros_like(pose_fea)], dim=-1)
    return prompts, uncond
