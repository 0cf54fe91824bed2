"""Architecture registry: names, hyper-parameters and state_dict layout.

Mirrors `get_speaker_model(name)(**model_args)` (wespeaker/models/speaker_model.py:30-57)
for the backbones on the north-star path, and reproduces the exact state_dict
key/shape list of the reference modules so an `avg_model.pt` trained with the
reference loads unchanged (`load_checkpoint(strict=False)`,
wespeaker/utils/checkpoint.py:20-27).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple

ParamList = List[Tuple[str, Tuple[int, ...]]]

ECAPA_ARCHS = {
    # name: (channels, global_context_att) — ecapa_tdnn.py:237-274
    "ECAPA_TDNN_c512": (512, False),
    "ECAPA_TDNN_GLOB_c512": (512, True),
    "ECAPA_TDNN_c1024": (1024, False),
    "ECAPA_TDNN_GLOB_c1024": (1024, True),
}
RESNET_ARCHS = {
    # name: (block, num_blocks) — resnet.py:207-260
    "ResNet18": ("basic", (2, 2, 2, 2)),
    "ResNet34": ("basic", (3, 4, 6, 3)),
    "ResNet50": ("bottleneck", (3, 4, 6, 3)),
    "ResNet101": ("bottleneck", (3, 4, 23, 3)),
    "ResNet152": ("bottleneck", (3, 8, 36, 3)),
    "ResNet221": ("bottleneck", (6, 16, 48, 3)),
    "ResNet293": ("bottleneck", (10, 20, 64, 3)),
}

SIMAM_ARCHS = {
    # name: num_blocks of SimAMBasicBlock — samresnet.py:115-121, 124-166
    "SimAM_ResNet34_ASP": (3, 4, 6, 3),
    "SimAM_ResNet100_ASP": (6, 16, 24, 3),
}


@dataclass
class ModelSpec:
    arch: str
    feat_dim: int = 80
    embed_dim: int = 192
    pooling_func: str = "ASTP"
    emb_bn: bool = False
    two_emb_layer: bool = False
    m_channels: int = 32
    extra: dict = field(default_factory=dict)

    @property
    def family(self) -> str:
        if self.arch.startswith("ECAPA_TDNN"):
            return "ecapa"
        if self.arch.startswith("ResNet"):
            return "resnet"
        if self.arch.startswith("SimAM_ResNet"):
            return "simam"
        raise KeyError(self.arch)


def make_spec(arch: str, **model_args) -> ModelSpec:
    """`get_speaker_model(arch)(**model_args)` analogue (speaker_model.py:30-57).

    Unknown names raise (the reference prints and exit(1)s, speaker_model.py:55-57).
    """
    if arch not in ECAPA_ARCHS and arch not in RESNET_ARCHS and arch not in SIMAM_ARCHS:
        raise KeyError(f"{arch} not found !!! (supported: "
                       f"{sorted(ECAPA_ARCHS) + sorted(RESNET_ARCHS) + sorted(SIMAM_ARCHS)})")
    kw = dict(model_args)
    if arch in SIMAM_ARCHS:
        # SimAM_ResNet*_ASP(in_planes=64, embed_dim=256, acoustic_dim=80, dropout=0)
        spec = ModelSpec(arch=arch, feat_dim=int(kw.pop("acoustic_dim", 80)),
                         embed_dim=int(kw.pop("embed_dim", 256)), pooling_func="ASP",
                         m_channels=int(kw.pop("in_planes", 64)))
        kw.pop("dropout", None)  # eval: nn.Dropout is the identity
        spec.extra = kw
        return spec
    spec = ModelSpec(arch=arch,
                     feat_dim=int(kw.pop("feat_dim", 80 if arch.startswith("ECAPA") else 40)),
                     embed_dim=int(kw.pop("embed_dim", 192 if arch.startswith("ECAPA") else 128)),
                     pooling_func=kw.pop("pooling_func", "ASTP" if arch.startswith("ECAPA") else "TSTP"),
                     emb_bn=bool(kw.pop("emb_bn", False)),
                     two_emb_layer=bool(kw.pop("two_emb_layer", False)))
    if spec.family == "ecapa" and spec.pooling_func != "ASTP":
        raise NotImplementedError("ECAPA path implements ASTP pooling (the north-star config)")
    if spec.family == "resnet" and spec.pooling_func != "TSTP":
        raise NotImplementedError("ResNet path implements TSTP pooling (the north-star config)")
    spec.extra = kw
    return spec


def _bn(p: str, c: int) -> ParamList:
    return [(p + ".weight", (c,)), (p + ".bias", (c,)), (p + ".running_mean", (c,)),
            (p + ".running_var", (c,)), (p + ".num_batches_tracked", ())]


def ecapa_params(spec: ModelSpec) -> ParamList:
    """state_dict layout of ECAPA_TDNN (ecapa_tdnn.py:160-206)."""
    C, glob = ECAPA_ARCHS[spec.arch]
    w = C // 8
    out: ParamList = [("layer1.conv.weight", (C, spec.feat_dim, 5)), ("layer1.conv.bias", (C,))]
    out += _bn("layer1.bn", C)
    for li in (2, 3, 4):
        p = f"layer{li}.se_res2block"
        out += [(f"{p}.0.conv.weight", (C, C, 1)), (f"{p}.0.conv.bias", (C,))] + _bn(f"{p}.0.bn", C)
        for i in range(7):
            out += [(f"{p}.1.convs.{i}.weight", (w, w, 3)), (f"{p}.1.convs.{i}.bias", (w,))]
        for i in range(7):
            out += _bn(f"{p}.1.bns.{i}", w)
        out += [(f"{p}.2.conv.weight", (C, C, 1)), (f"{p}.2.conv.bias", (C,))] + _bn(f"{p}.2.bn", C)
        out += [(f"{p}.3.linear1.weight", (128, C)), (f"{p}.3.linear1.bias", (128,)),
                (f"{p}.3.linear2.weight", (C, 128)), (f"{p}.3.linear2.bias", (C,))]
    out += [("conv.weight", (1536, 3 * C, 1)), ("conv.bias", (1536,))]
    out += [("pool.linear1.weight", (128, 1536 * (3 if glob else 1), 1)), ("pool.linear1.bias", (128,)),
            ("pool.linear2.weight", (1536, 128, 1)), ("pool.linear2.bias", (1536,))]
    out += _bn("bn", 3072)
    out += [("linear.weight", (spec.embed_dim, 3072)), ("linear.bias", (spec.embed_dim,))]
    if spec.emb_bn:
        out += _bn("bn2", spec.embed_dim)
    return out


def resnet_params(spec: ModelSpec) -> ParamList:
    """state_dict layout of ResNet (resnet.py:110-169)."""
    kind, nblocks = RESNET_ARCHS[spec.arch]
    m = spec.m_channels
    exp = 1 if kind == "basic" else 4
    out: ParamList = [("conv1.weight", (m, 1, 3, 3))] + _bn("bn1", m)
    in_planes = m
    for li, n in enumerate(nblocks):
        planes = m * (2 ** li)
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            p = f"layer{li + 1}.{bi}"
            if kind == "basic":
                out += [(p + ".conv1.weight", (planes, in_planes, 3, 3))] + _bn(p + ".bn1", planes)
                out += [(p + ".conv2.weight", (planes, planes, 3, 3))] + _bn(p + ".bn2", planes)
            else:
                out += [(p + ".conv1.weight", (planes, in_planes, 1, 1))] + _bn(p + ".bn1", planes)
                out += [(p + ".conv2.weight", (planes, planes, 3, 3))] + _bn(p + ".bn2", planes)
                out += [(p + ".conv3.weight", (planes * 4, planes, 1, 1))] + _bn(p + ".bn3", planes * 4)
            if stride != 1 or in_planes != exp * planes:
                out += [(p + ".shortcut.0.weight", (exp * planes, in_planes, 1, 1))]
                out += _bn(p + ".shortcut.1", exp * planes)
            in_planes = planes * exp
    stats_dim = int(spec.feat_dim / 8) * m * 8 * exp
    out += [("seg_1.weight", (spec.embed_dim, stats_dim * 2)), ("seg_1.bias", (spec.embed_dim,))]
    if spec.two_emb_layer:
        out += [("seg_bn_1.running_mean", (spec.embed_dim,)), ("seg_bn_1.running_var", (spec.embed_dim,)),
                ("seg_bn_1.num_batches_tracked", ()),
                ("seg_2.weight", (spec.embed_dim, spec.embed_dim)), ("seg_2.bias", (spec.embed_dim,))]
    return out


def simam_params(spec: ModelSpec) -> ParamList:
    """state_dict layout of SimAM_ResNet*_ASP (samresnet.py:72-166, ASP pooling_layers.py:151-164)."""
    m = spec.m_channels
    out: ParamList = [("front.conv1.weight", (m, 1, 3, 3))] + _bn("front.bn1", m)
    in_planes = m
    for li, n in enumerate(SIMAM_ARCHS[spec.arch]):
        planes = m * (2 ** li)
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            p = f"front.layer{li + 1}.{bi}"
            out += [(p + ".conv1.weight", (planes, in_planes, 3, 3))] + _bn(p + ".bn1", planes)
            out += [(p + ".conv2.weight", (planes, planes, 3, 3))] + _bn(p + ".bn2", planes)
            if stride != 1 or in_planes != planes:
                out += [(p + ".downsample.0.weight", (planes, in_planes, 1, 1))] + _bn(p + ".downsample.1", planes)
            in_planes = planes
    cf = m * 8 * int(spec.feat_dim / 8)
    out += [("pooling.attention.0.weight", (128, cf, 1)), ("pooling.attention.0.bias", (128,))]
    out += _bn("pooling.attention.2", 128)
    out += [("pooling.attention.3.weight", (cf, 128, 1)), ("pooling.attention.3.bias", (cf,))]
    out += [("bottleneck.weight", (spec.embed_dim, 2 * cf)), ("bottleneck.bias", (spec.embed_dim,))]
    return out


def param_list(spec: ModelSpec) -> ParamList:
    if spec.family == "ecapa":
        return ecapa_params(spec)
    if spec.family == "simam":
        return simam_params(spec)
    return resnet_params(spec)


def simam_gflop_per_utt(spec: ModelSpec, T: int) -> float:
    """Algorithmic FLOPs (2 x MACs) of one SimAM-ResNet forward over T frames."""
    m, F, t = spec.m_channels, spec.feat_dim, T
    macs = F * t * m * 9  # stem
    cin = m
    for li, n in enumerate(SIMAM_ARCHS[spec.arch]):
        planes = m * (2 ** li)
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            Fo, To = (F - 1) // stride + 1, (t - 1) // stride + 1
            macs += Fo * To * planes * (cin * 9 + planes * 9)
            if stride != 1 or cin != planes:
                macs += Fo * To * planes * cin
            F, t, cin = Fo, To, planes
    cf = cin * F
    macs += t * (cf * 128 * 2) + 2 * cf * spec.embed_dim
    return 2.0 * macs / 1e9


def resnet_gflop_per_utt(spec: ModelSpec, T: int) -> float:
    """Algorithmic FLOPs (2 x MACs) of one ResNet forward over T frames (resnet.py:35-204):
    stem, every block's convs (+ projection shortcuts), the pooled-statistics embedding."""
    kind, nblocks = RESNET_ARCHS[spec.arch]
    m, F, t = spec.m_channels, spec.feat_dim, T
    exp = 1 if kind == "basic" else 4
    macs = F * t * m * 9  # stem 3x3, 1 -> m
    cin = m
    for li, n in enumerate(nblocks):
        p = m * (2 ** li)
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            Fo, To = (F - 1) // s + 1, (t - 1) // s + 1
            if kind == "basic":
                macs += Fo * To * p * (cin * 9 + p * 9)
            else:
                macs += F * t * cin * p + Fo * To * (p * p * 9 + p * 4 * p)
            if s != 1 or cin != exp * p:
                macs += Fo * To * cin * exp * p
            F, t, cin = Fo, To, exp * p
    macs += 2 * cin * F * spec.embed_dim + (spec.embed_dim ** 2 if spec.two_emb_layer else 0)
    return 2.0 * macs / 1e9


def ecapa_gflop_per_utt(spec: ModelSpec, T: int) -> float:
    """Algorithmic FLOPs (2 x MACs) of one ECAPA forward over T frames."""
    C, glob = ECAPA_ARCHS[spec.arch]
    w = C // 8
    macs = spec.feat_dim * 5 * C * T                       # layer1
    macs += 3 * (2 * C * C * T + 7 * w * w * 3 * T + 2 * C * 128)  # blocks
    macs += 3 * C * 1536 * T                                # conv
    # pool.linear1: GLOB's mean/std context columns are constant over T and
    # are folded into a per-utterance bias, so both variants run
    # a 1536-deep contraction per frame.
    macs += 1536 * 128 * T + (2 * 1536 * 128 if glob else 0)
    macs += 128 * 1536 * T                                  # pool.linear2
    macs += 3072 * spec.embed_dim
    return 2.0 * macs / 1e9


# ---------------------------------------------------------------- HuBERT ---
# s3prl HuBERT-base upstream as wrapped by wespeaker/frontend/s3prl.py:23-93.
# Canonical keys are the fairseq names s3prl loads, under the prefix the
# reference checkpoint uses (`model.add_module("frontend", ...)`,
# bin/extract.py:49-55 -> S3PRLUpstream.upstream.model).
HUBERT_PREFIX = "frontend.upstream.upstream.model."
HUBERT_BASE = dict(conv_dim=512, conv_kernel=(10, 3, 3, 3, 3, 2, 2), conv_stride=(5, 2, 2, 2, 2, 2, 2),
                   hidden=768, layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16)


def hubert_params(cfg=HUBERT_BASE, prefix: str = HUBERT_PREFIX) -> ParamList:
    c, h = cfg["conv_dim"], cfg["hidden"]
    out: ParamList = []
    for i, k in enumerate(cfg["conv_kernel"]):
        out.append((f"feature_extractor.conv_layers.{i}.0.weight", (c, 1 if i == 0 else c, k)))
        if i == 0:
            out += [("feature_extractor.conv_layers.0.2.weight", (c,)),
                    ("feature_extractor.conv_layers.0.2.bias", (c,))]
    out += [("layer_norm.weight", (c,)), ("layer_norm.bias", (c,)),
            ("post_extract_proj.weight", (h, c)), ("post_extract_proj.bias", (h,)),
            ("encoder.pos_conv.0.bias", (h,)), ("encoder.pos_conv.0.weight_g", (1, 1, cfg["pos_k"])),
            ("encoder.pos_conv.0.weight_v", (h, h // cfg["pos_groups"], cfg["pos_k"])),
            ("encoder.layer_norm.weight", (h,)), ("encoder.layer_norm.bias", (h,))]
    for li in range(cfg["layers"]):
        p = f"encoder.layers.{li}."
        for proj in ("k_proj", "v_proj", "q_proj", "out_proj"):
            out += [(p + f"self_attn.{proj}.weight", (h, h)), (p + f"self_attn.{proj}.bias", (h,))]
        out += [(p + "self_attn_layer_norm.weight", (h,)), (p + "self_attn_layer_norm.bias", (h,)),
                (p + "fc1.weight", (cfg["ffn"], h)), (p + "fc1.bias", (cfg["ffn"],)),
                (p + "fc2.weight", (h, cfg["ffn"])), (p + "fc2.bias", (h,)),
                (p + "final_layer_norm.weight", (h,)), (p + "final_layer_norm.bias", (h,))]
    out = [(prefix + n, s) for n, s in out]
    out.append(("frontend.featurizer.weights", (cfg["layers"] + 1,)))
    return out


def hubert_num_frames(num_samples: int, cfg=HUBERT_BASE) -> int:
    t = num_samples
    for k, s in zip(cfg["conv_kernel"], cfg["conv_stride"]):
        t = (t - k) // s + 1
    return t


def s3prl_num_frames(num_samples: int, downsample_rate: int = 320) -> int:
    """len(range(0, W, 320)) — s3prl's length match target."""
    return (num_samples + downsample_rate - 1) // downsample_rate


def hubert_gflop_per_utt(num_samples: int, cfg=HUBERT_BASE) -> float:
    """Algorithmic FLOPs (2 x MACs) of the HuBERT-base front end on one utterance."""
    c, h, L = cfg["conv_dim"], cfg["hidden"], cfg["layers"]
    t = num_samples
    macs = 0
    for i, (k, s) in enumerate(zip(cfg["conv_kernel"], cfg["conv_stride"])):
        t = (t - k) // s + 1
        macs += t * c * k * (1 if i == 0 else c)
    macs += t * c * h                                               # post_extract_proj
    macs += t * h * (h // cfg["pos_groups"]) * cfg["pos_k"]         # grouped pos_conv
    per_layer = t * h * 3 * h + 2 * t * t * h + t * h * h + 2 * t * h * cfg["ffn"]
    return 2.0 * (macs + L * per_layer) / 1e9
