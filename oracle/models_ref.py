"""ORACLE (test infrastructure only): fp32 PyTorch-CPU restatement of the
reference speaker backbones, written against a plain state_dict.

Each function cites the reference code it restates.  Pinned by
tests/golden/*.npz (generated from the reference modules themselves).
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
BN_EPS = 1e-5  # nn.BatchNorm default


def _bn(x: Tensor, sd: Dict[str, Tensor], p: str) -> Tensor:
    # eval-mode BatchNorm{1,2}d: (x - rm) / sqrt(rv + eps) * w + b
    shape = [1, -1] + [1] * (x.dim() - 2)
    rm, rv = sd[p + ".running_mean"].view(shape), sd[p + ".running_var"].view(shape)
    y = (x - rm) / torch.sqrt(rv + BN_EPS)
    if (p + ".weight") in sd:
        y = y * sd[p + ".weight"].view(shape) + sd[p + ".bias"].view(shape)
    return y


# ---------------------------------------------------------------- pooling ---
def tstp(x: Tensor) -> Tensor:
    """TSTP.forward — pooling_layers.py:78-85 (unbiased var, +1e-7)."""
    mean = x.mean(dim=-1).flatten(start_dim=1)
    std = torch.sqrt(torch.var(x, dim=-1) + 1e-7).flatten(start_dim=1)
    return torch.cat((mean, std), 1)


def astp(x: Tensor, sd: Dict[str, Tensor], p: str, glob: bool) -> Tensor:
    """ASTP.forward — pooling_layers.py:119-144."""
    if x.dim() == 4:
        x = x.reshape(x.shape[0], x.shape[1] * x.shape[2], x.shape[3])
    if glob:
        mean = x.mean(dim=-1, keepdim=True).expand_as(x)
        std = torch.sqrt(torch.var(x, dim=-1, keepdim=True) + 1e-7).expand_as(x)
        x_in = torch.cat((x, mean, std), dim=1)
    else:
        x_in = x
    a = torch.tanh(F.conv1d(x_in, sd[p + ".linear1.weight"], sd[p + ".linear1.bias"]))
    a = torch.softmax(F.conv1d(a, sd[p + ".linear2.weight"], sd[p + ".linear2.bias"]), dim=2)
    mu = torch.sum(a * x, dim=2)
    var = torch.sum(a * x * x, dim=2) - mu * mu
    return torch.cat([mu, torch.sqrt(var.clamp(min=1e-7))], dim=1)


# ------------------------------------------------------------------ ECAPA ---
def _conv_relu_bn(x, sd, p, padding=0, dilation=1):
    """Conv1dReluBn — ecapa_tdnn.py:85-106 (conv -> ReLU -> BN)."""
    y = F.conv1d(x, sd[p + ".conv.weight"], sd.get(p + ".conv.bias"), padding=padding, dilation=dilation)
    return _bn(F.relu(y), sd, p + ".bn")


def _res2(x, sd, p, dilation, scale=8):
    """Res2Conv1dReluBn — ecapa_tdnn.py:29-78."""
    width = x.shape[1] // scale
    spx = torch.split(x, width, 1)
    out = []
    sp = spx[0]
    for i in range(scale - 1):
        if i >= 1:
            sp = sp + spx[i]
        sp = F.conv1d(sp, sd[f"{p}.convs.{i}.weight"], sd.get(f"{p}.convs.{i}.bias"),
                      padding=dilation, dilation=dilation)
        sp = _bn(F.relu(sp), sd, f"{p}.bns.{i}")
        out.append(sp)
    out.append(spx[scale - 1])
    return torch.cat(out, dim=1)


def _se(x, sd, p):
    """SE_Connect — ecapa_tdnn.py:113-126."""
    s = x.mean(dim=2)
    s = F.relu(F.linear(s, sd[p + ".linear1.weight"], sd[p + ".linear1.bias"]))
    s = torch.sigmoid(F.linear(s, sd[p + ".linear2.weight"], sd[p + ".linear2.bias"]))
    return x * s.unsqueeze(2)


def _se_res2block(x, sd, p, dilation):
    """SE_Res2Block — ecapa_tdnn.py:133-157: x + SE(conv(Res2(conv(x))))."""
    y = _conv_relu_bn(x, sd, p + ".se_res2block.0")
    y = _res2(y, sd, p + ".se_res2block.1", dilation)
    y = _conv_relu_bn(y, sd, p + ".se_res2block.2")
    y = _se(y, sd, p + ".se_res2block.3")
    return x + y


def ecapa_frame_level(feats: Tensor, sd: Dict[str, Tensor]):
    """ECAPA_TDNN._get_frame_level_feat — ecapa_tdnn.py:208-220."""
    x = feats.permute(0, 2, 1)
    out1 = _conv_relu_bn(x, sd, "layer1", padding=2)
    out2 = _se_res2block(out1, sd, "layer2", 2)
    out3 = _se_res2block(out2, sd, "layer3", 3)
    out4 = _se_res2block(out3, sd, "layer4", 4)
    out = F.conv1d(torch.cat([out2, out3, out4], dim=1), sd["conv.weight"], sd["conv.bias"])
    return out, out4, (out1, out2, out3, out4)


def ecapa_forward(feats: Tensor, sd: Dict[str, Tensor], glob: bool, emb_bn: bool = False):
    """ECAPA_TDNN.forward — ecapa_tdnn.py:227-234. Returns (out4, embed)."""
    out, out4, _ = ecapa_frame_level(feats, sd)
    pooled = astp(F.relu(out), sd, "pool", glob)
    e = F.linear(_bn(pooled, sd, "bn"), sd["linear.weight"], sd["linear.bias"])
    if emb_bn:
        e = _bn(e, sd, "bn2")
    return out4, e


# ----------------------------------------------------------------- ResNet ---
RESNET_BLOCKS = {
    "ResNet18": ("basic", [2, 2, 2, 2]), "ResNet34": ("basic", [3, 4, 6, 3]),
    "ResNet50": ("bottleneck", [3, 4, 6, 3]), "ResNet101": ("bottleneck", [3, 4, 23, 3]),
    "ResNet152": ("bottleneck", [3, 8, 36, 3]), "ResNet221": ("bottleneck", [6, 16, 48, 3]),
    "ResNet293": ("bottleneck", [10, 20, 64, 3]),
}


def _basic(x, sd, p, stride):
    """BasicBlock.forward — resnet.py:35-69."""
    out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], stride=stride, padding=1), sd, p + ".bn1"))
    out = _bn(F.conv2d(out, sd[p + ".conv2.weight"], padding=1), sd, p + ".bn2")
    sc = x
    if (p + ".shortcut.0.weight") in sd:
        sc = _bn(F.conv2d(x, sd[p + ".shortcut.0.weight"], stride=stride), sd, p + ".shortcut.1")
    return F.relu(out + sc)


def _bottleneck(x, sd, p, stride):
    """Bottleneck.forward — resnet.py:72-107."""
    out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"]), sd, p + ".bn1"))
    out = F.relu(_bn(F.conv2d(out, sd[p + ".conv2.weight"], stride=stride, padding=1), sd, p + ".bn2"))
    out = _bn(F.conv2d(out, sd[p + ".conv3.weight"]), sd, p + ".bn3")
    sc = x
    if (p + ".shortcut.0.weight") in sd:
        sc = _bn(F.conv2d(x, sd[p + ".shortcut.0.weight"], stride=stride), sd, p + ".shortcut.1")
    return F.relu(out + sc)


def resnet_forward(feats: Tensor, sd: Dict[str, Tensor], arch: str, two_emb_layer: bool = False):
    """ResNet.forward — resnet.py:171-204 (TSTP pooling). Returns (aux, embed)."""
    kind, nblocks = RESNET_BLOCKS[arch]
    blk = _basic if kind == "basic" else _bottleneck
    x = feats.permute(0, 2, 1).unsqueeze(1)
    out = F.relu(_bn(F.conv2d(x, sd["conv1.weight"], padding=1), sd, "bn1"))
    for li, n in enumerate(nblocks):
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            out = blk(out, sd, f"layer{li + 1}.{bi}", stride)
    stats = tstp(out)
    e = F.linear(stats, sd["seg_1.weight"], sd["seg_1.bias"])
    if two_emb_layer:
        o = _bn(F.relu(e), sd, "seg_bn_1")
        return e, F.linear(o, sd["seg_2.weight"], sd["seg_2.bias"])
    return torch.tensor(0.0), e


# ------------------------------------------------------------ SimAM-ResNet ---
SIMAM_BLOCKS = {"SimAM_ResNet34_ASP": [3, 4, 6, 3], "SimAM_ResNet100_ASP": [6, 16, 24, 3]}


def _simam(x: Tensor, lam: float = 1e-4) -> Tensor:
    """SimAMBasicBlock.SimAM — samresnet.py:64-69: energy over the F*T positions,
    variance with the (n - 1) divisor."""
    n = x.shape[2] * x.shape[3] - 1
    d = (x - x.mean(dim=(2, 3), keepdim=True)) ** 2
    v = d.sum(dim=(2, 3), keepdim=True) / n
    return x * torch.sigmoid(d / (4 * (v + lam)) + 0.5)


def _simam_block(x, sd, p, stride):
    """SimAMBasicBlock.forward — samresnet.py:56-62."""
    out = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], stride=stride, padding=1), sd, p + ".bn1"))
    out = _simam(_bn(F.conv2d(out, sd[p + ".conv2.weight"], padding=1), sd, p + ".bn2"))
    sc = x
    if (p + ".downsample.0.weight") in sd:
        sc = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=stride), sd, p + ".downsample.1")
    return F.relu(out + sc)


def asp(x: Tensor, sd: Dict[str, Tensor], p: str) -> Tensor:
    """ASP.forward — pooling_layers.py:166-173: (B,C,F,T) -> (B,C*F,T), attention
    Conv1d -> ReLU -> BN -> Conv1d -> softmax over T, clamp 1e-5."""
    x = x.reshape(x.shape[0], -1, x.shape[-1])
    h = _bn(F.relu(F.conv1d(x, sd[p + ".0.weight"], sd[p + ".0.bias"])), sd, p + ".2")
    w = torch.softmax(F.conv1d(h, sd[p + ".3.weight"], sd[p + ".3.bias"]), dim=2)
    mu = torch.sum(x * w, dim=2)
    sg = torch.sqrt((torch.sum(x * x * w, dim=2) - mu * mu).clamp(min=1e-5))
    return torch.cat((mu, sg), 1)


def simam_forward(feats: Tensor, sd: Dict[str, Tensor], arch: str) -> Tensor:
    """SimAM_ResNet*_ASP.forward — samresnet.py:135-143 (returns the embedding)."""
    x = feats.permute(0, 2, 1).unsqueeze(1)
    out = F.relu(_bn(F.conv2d(x, sd["front.conv1.weight"], padding=1), sd, "front.bn1"))
    for li, n in enumerate(SIMAM_BLOCKS[arch]):
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            out = _simam_block(out, sd, f"front.layer{li + 1}.{bi}", stride)
    return F.linear(asp(out, sd, "pooling.attention"), sd["bottleneck.weight"], sd["bottleneck.bias"])


def forward(arch: str, feats: Tensor, sd: Dict[str, Tensor], emb_bn: bool = False, two_emb_layer: bool = False):
    """Registry dispatch — speaker_model.py:30-57 (prefix match).  Always (aux, embed)."""
    if arch.startswith("SimAM_ResNet"):
        return None, simam_forward(feats, sd, arch)
    if arch.startswith("ECAPA_TDNN"):
        return ecapa_forward(feats, sd, glob="GLOB" in arch, emb_bn=emb_bn)
    if arch.startswith("ResNet"):
        return resnet_forward(feats, sd, arch, two_emb_layer)
    raise KeyError(arch)
