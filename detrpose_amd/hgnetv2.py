"""HGNetv2 backbone: constructor and parameter layout of src/nn/backbone/hgnetv2.py.

The classes here hold parameters under the reference's names so a reference
checkpoint loads unchanged (1208 keys for DETRPose-L). They do not compute: the
forward is planned over HIP kernels by detrpose_amd.engine (NHWC, BN folded into the
conv, concats written in place). Constructor arguments match HGNetv2.__init__
(hgnetv2.py:478-570); `pretrained=True` is rejected because it downloads weights.
"""
from __future__ import annotations

import torch
from torch import nn


class FrozenBatchNorm2d(nn.Module):
    """Buffers of hgnetv2.py:24-65 (weight, bias, running_mean, running_var)."""

    def __init__(self, num_features, eps=1e-5):
        super().__init__()
        self.register_buffer("weight", torch.ones(num_features))
        self.register_buffer("bias", torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.eps = eps
        self.num_features = num_features

    def _load_from_state_dict(self, state_dict, prefix, *args, **kw):
        state_dict.pop(prefix + "num_batches_tracked", None)
        super()._load_from_state_dict(state_dict, prefix, *args, **kw)


class LearnableAffineBlock(nn.Module):
    """hgnetv2.py:68-79: y = scale * x + bias (scalars)."""

    def __init__(self, scale_value=1.0, bias_value=0.0):
        super().__init__()
        self.scale = nn.Parameter(torch.tensor([scale_value]))
        self.bias = nn.Parameter(torch.tensor([bias_value]))


class ConvBNAct(nn.Module):
    """hgnetv2.py:82-134 (padding=(k-1)//2; 'same' padding is unused by B0-B6)."""

    def __init__(self, in_chs, out_chs, kernel_size, stride=1, groups=1, padding="", use_act=True, use_lab=False,
                 freeze_norm=True):
        super().__init__()
        if padding == "same":
            raise NotImplementedError("padding='same' is not used by the HGNetv2 B0-B6 architectures")
        self.kernel_size, self.stride, self.groups = kernel_size, stride, groups
        self.use_act, self.use_lab = use_act, use_lab
        self.conv = nn.Conv2d(in_chs, out_chs, kernel_size, stride, padding=(kernel_size - 1) // 2, groups=groups,
                              bias=False)
        self.bn = FrozenBatchNorm2d(out_chs) if freeze_norm else nn.BatchNorm2d(out_chs)
        self.lab = LearnableAffineBlock() if (use_act and use_lab) else nn.Identity()


class LightConvBNAct(nn.Module):
    """hgnetv2.py:137-166: 1x1 (no act) then depthwise k x k + ReLU."""

    def __init__(self, in_chs, out_chs, kernel_size, groups=1, use_lab=False, freeze_norm=True):
        super().__init__()
        self.conv1 = ConvBNAct(in_chs, out_chs, 1, use_act=False, use_lab=use_lab, freeze_norm=freeze_norm)
        self.conv2 = ConvBNAct(out_chs, out_chs, kernel_size, groups=out_chs, use_act=True, use_lab=use_lab,
                               freeze_norm=freeze_norm)


class StemBlock(nn.Module):
    """hgnetv2.py:169-220."""

    def __init__(self, in_chs, mid_chs, out_chs, use_lab=False, freeze_norm=True):
        super().__init__()
        kw = dict(use_lab=use_lab, freeze_norm=freeze_norm)
        self.stem1 = ConvBNAct(in_chs, mid_chs, 3, stride=2, **kw)
        self.stem2a = ConvBNAct(mid_chs, mid_chs // 2, 2, stride=1, **kw)
        self.stem2b = ConvBNAct(mid_chs // 2, mid_chs, 2, stride=1, **kw)
        self.stem3 = ConvBNAct(mid_chs * 2, mid_chs, 3, stride=2, **kw)
        self.stem4 = ConvBNAct(mid_chs, out_chs, 1, stride=1, **kw)


class HG_Block(nn.Module):
    """hgnetv2.py:243-329 with agg='se' (the only aggregation HG_Stage builds, 344)."""

    def __init__(self, in_chs, mid_chs, out_chs, layer_num, kernel_size=3, residual=False, light_block=False,
                 use_lab=False, agg="se", drop_path=0.0, freeze_norm=True):
        super().__init__()
        if agg != "se":
            raise NotImplementedError("only agg='se' is reachable from HGNetv2 (hgnetv2.py:344, 514-524)")
        self.residual = residual
        self.light_block = light_block
        self.layers = nn.ModuleList()
        for i in range(layer_num):
            cin = in_chs if i == 0 else mid_chs
            if light_block:
                self.layers.append(LightConvBNAct(cin, mid_chs, kernel_size, use_lab=use_lab, freeze_norm=freeze_norm))
            else:
                self.layers.append(ConvBNAct(cin, mid_chs, kernel_size, stride=1, use_lab=use_lab,
                                             freeze_norm=freeze_norm))
        total = in_chs + layer_num * mid_chs
        self.aggregation = nn.Sequential(
            ConvBNAct(total, out_chs // 2, 1, stride=1, use_lab=use_lab, freeze_norm=freeze_norm),
            ConvBNAct(out_chs // 2, out_chs, 1, stride=1, use_lab=use_lab, freeze_norm=freeze_norm))


class HG_Stage(nn.Module):
    """hgnetv2.py:332-383."""

    def __init__(self, in_chs, mid_chs, out_chs, block_num, layer_num, downsample=True, light_block=False,
                 kernel_size=3, use_lab=False, agg="se", drop_path=0.0, freeze_norm=True):
        super().__init__()
        if downsample:
            self.downsample = ConvBNAct(in_chs, in_chs, 3, stride=2, groups=in_chs, use_act=False, use_lab=use_lab,
                                        freeze_norm=freeze_norm)
        else:
            self.downsample = nn.Identity()
        self.blocks = nn.Sequential(*[
            HG_Block(in_chs if i == 0 else out_chs, mid_chs, out_chs, layer_num, residual=i > 0,
                     kernel_size=kernel_size, light_block=light_block, use_lab=use_lab, agg=agg,
                     freeze_norm=freeze_norm)
            for i in range(block_num)])


class HGNetv2(nn.Module):
    """hgnetv2.py:386-593. arch_configs restated from 398-476."""

    arch_configs = {
        "B0": {"stem_channels": [3, 16, 16],
               "stage_config": {"stage1": [16, 16, 64, 1, False, False, 3, 3],
                                "stage2": [64, 32, 256, 1, True, False, 3, 3],
                                "stage3": [256, 64, 512, 2, True, True, 5, 3],
                                "stage4": [512, 128, 1024, 1, True, True, 5, 3]}},
        "B1": {"stem_channels": [3, 24, 32],
               "stage_config": {"stage1": [32, 32, 64, 1, False, False, 3, 3],
                                "stage2": [64, 48, 256, 1, True, False, 3, 3],
                                "stage3": [256, 96, 512, 2, True, True, 5, 3],
                                "stage4": [512, 192, 1024, 1, True, True, 5, 3]}},
        "B2": {"stem_channels": [3, 24, 32],
               "stage_config": {"stage1": [32, 32, 96, 1, False, False, 3, 4],
                                "stage2": [96, 64, 384, 1, True, False, 3, 4],
                                "stage3": [384, 128, 768, 3, True, True, 5, 4],
                                "stage4": [768, 256, 1536, 1, True, True, 5, 4]}},
        "B3": {"stem_channels": [3, 24, 32],
               "stage_config": {"stage1": [32, 32, 128, 1, False, False, 3, 5],
                                "stage2": [128, 64, 512, 1, True, False, 3, 5],
                                "stage3": [512, 128, 1024, 3, True, True, 5, 5],
                                "stage4": [1024, 256, 2048, 1, True, True, 5, 5]}},
        "B4": {"stem_channels": [3, 32, 48],
               "stage_config": {"stage1": [48, 48, 128, 1, False, False, 3, 6],
                                "stage2": [128, 96, 512, 1, True, False, 3, 6],
                                "stage3": [512, 192, 1024, 3, True, True, 5, 6],
                                "stage4": [1024, 384, 2048, 1, True, True, 5, 6]}},
        "B5": {"stem_channels": [3, 32, 64],
               "stage_config": {"stage1": [64, 64, 128, 1, False, False, 3, 6],
                                "stage2": [128, 128, 512, 2, True, False, 3, 6],
                                "stage3": [512, 256, 1024, 5, True, True, 5, 6],
                                "stage4": [1024, 512, 2048, 2, True, True, 5, 6]}},
        "B6": {"stem_channels": [3, 48, 96],
               "stage_config": {"stage1": [96, 96, 192, 2, False, False, 3, 6],
                                "stage2": [192, 192, 512, 3, True, False, 3, 6],
                                "stage3": [512, 384, 1024, 6, True, True, 5, 6],
                                "stage4": [1024, 768, 2048, 3, True, True, 5, 6]}},
    }

    def __init__(self, name, use_lab=False, return_idx=(1, 2, 3), freeze_stem_only=True, freeze_at=-1,
                 freeze_norm=True, pretrained=False, local_model_dir="weight/hgnetv2/", for_pgi=False,
                 freeze_network=False):
        super().__init__()
        if pretrained:
            raise ValueError("pretrained=True downloads weights (hgnetv2.py:548); load a state_dict instead")
        self.name = name
        self.use_lab = use_lab
        self.return_idx = list(return_idx)
        stem = self.arch_configs[name]["stem_channels"]
        cfg = self.arch_configs[name]["stage_config"]
        self._out_strides = [4, 8, 16, 32]
        self._out_channels = [cfg[k][2] for k in cfg]
        self.num_channels = self._out_channels[4 - len(self.return_idx):]
        self.stem = StemBlock(stem[0], stem[1], stem[2], use_lab=use_lab, freeze_norm=freeze_norm)
        self.stages = nn.ModuleList()
        for k in cfg:
            cin, mid, cout, nblk, down, light, ks, nl = cfg[k]
            self.stages.append(HG_Stage(cin, mid, cout, nblk, nl, down, light, ks, use_lab, freeze_norm=freeze_norm))
        if freeze_network:
            for p in self.parameters():
                p.requires_grad = False

    def forward(self, x):
        raise NotImplementedError("run the full model through DETRPose.forward (HIP engine)")
