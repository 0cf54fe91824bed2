"""ORACLE (test infrastructure only): fp32 torch-CPU restatement of the
HuBERT-base SSL front end as used by the reference through s3prl
(wespeaker/frontend/s3prl.py:23-93; s3prl is a third-party dependency,
requirements.txt `s3prl` unpinned, NOT installed here).

Restated algorithm (fairseq HuBERT as loaded by s3prl's `hubert` upstream,
identical to transformers' HubertModel with feat_extract_norm="group",
do_stable_layer_norm=False):
  conv0 (1->512, k10, s5, no bias) -> GroupNorm(512 groups) -> GELU ->
  6 x [conv (512->512, k3/3/3/3/2/2, s2, no bias) -> GELU]            (B, T, 512)
  LayerNorm(512) -> Linear(512 -> 768)
  x + GELU(SamePad(weight-norm grouped conv k128 g16 pad 64)(x)) -> LayerNorm
  12 x post-LN layers: x = LN(x + MHA(x)); x = LN(x + fc2(GELU(fc1(x))))
  hidden states = [input of layer 0] + [output of each layer]  (13)
s3prl glue restated from s3prl>=0.4 `s3prl/nn/upstream.py` S3PRLUpstream.forward
(published source; cannot be verified offline), called at
wespeaker/frontend/s3prl.py:80-82:
  * MIN_SECOND = 0.05: when the longest waveform is shorter than
    0.05 * 16000 = 800 samples, the batch is zero-padded to 800 samples BEFORE
    the upstream (so conv0's GroupNorm sees the padding);
  * length match: every hidden state is matched to len(range(0, W_padded, 320))
    frames by repeating its last frame (or trimming), then trimmed to
    (W_original - 1) // 320 + 1 frames;
  * Featurizer (normalize=False): sum_l softmax(weights)_l * h_l.
**Parity unpinned against the reference** (s3prl absent, weights download by
URL).  `hubert_hidden_states` is pinned against transformers' HubertModel
(offline proxy) by tests/golden/hubert_proxy.npz.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F

from wespeaker_hubert_amd.arch import HUBERT_BASE, HUBERT_PREFIX, s3prl_num_frames

Tensor = torch.Tensor


def _ln(x, sd, p, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def pos_conv_weight(g: Tensor, v: Tensor) -> Tensor:
    """weight_norm(dim=2): w = g * v / ||v|| with the norm over dims (0, 1)."""
    n = torch.sqrt((v.double() ** 2).sum(dim=(0, 1), keepdim=True)).float()
    return g * v / n


def hubert_hidden_states(wav: Tensor, sd: Dict[str, Tensor], prefix: str = HUBERT_PREFIX,
                         cfg=HUBERT_BASE) -> List[Tensor]:
    P = prefix
    x = wav.unsqueeze(1)
    for i, (k, s) in enumerate(zip(cfg["conv_kernel"], cfg["conv_stride"])):
        x = F.conv1d(x, sd[P + f"feature_extractor.conv_layers.{i}.0.weight"], stride=s)
        if i == 0:
            x = F.group_norm(x, x.shape[1], sd[P + "feature_extractor.conv_layers.0.2.weight"],
                             sd[P + "feature_extractor.conv_layers.0.2.bias"], 1e-5)
        x = F.gelu(x)
    x = x.transpose(1, 2)
    x = _ln(x, sd, P + "layer_norm")
    x = F.linear(x, sd[P + "post_extract_proj.weight"], sd[P + "post_extract_proj.bias"])
    w = pos_conv_weight(sd[P + "encoder.pos_conv.0.weight_g"], sd[P + "encoder.pos_conv.0.weight_v"])
    pc = F.conv1d(x.transpose(1, 2), w, sd[P + "encoder.pos_conv.0.bias"], padding=cfg["pos_k"] // 2,
                  groups=cfg["pos_groups"])
    if cfg["pos_k"] % 2 == 0:
        pc = pc[:, :, :-1]
    x = x + F.gelu(pc).transpose(1, 2)
    x = _ln(x, sd, P + "encoder.layer_norm")
    hs = [x]
    H = cfg["heads"]
    B, T, D = x.shape
    dh = D // H
    for li in range(cfg["layers"]):
        p = P + f"encoder.layers.{li}."
        q = F.linear(x, sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.q_proj.bias"])
        k = F.linear(x, sd[p + "self_attn.k_proj.weight"], sd[p + "self_attn.k_proj.bias"])
        v = F.linear(x, sd[p + "self_attn.v_proj.weight"], sd[p + "self_attn.v_proj.bias"])
        q = q.view(B, T, H, dh).transpose(1, 2)
        k = k.view(B, T, H, dh).transpose(1, 2)
        v = v.view(B, T, H, dh).transpose(1, 2)
        a = torch.softmax(torch.matmul(q, k.transpose(2, 3)) * dh ** -0.5, dim=-1)
        o = torch.matmul(a, v).transpose(1, 2).reshape(B, T, D)
        o = F.linear(o, sd[p + "self_attn.out_proj.weight"], sd[p + "self_attn.out_proj.bias"])
        x = _ln(x + o, sd, p + "self_attn_layer_norm")
        f = F.linear(F.gelu(F.linear(x, sd[p + "fc1.weight"], sd[p + "fc1.bias"])), sd[p + "fc2.weight"],
                     sd[p + "fc2.bias"])
        x = _ln(x + f, sd, p + "final_layer_norm")
        hs.append(x)
    return hs


def match_length(h: Tensor, num_samples: int, downsample_rate: int = 320) -> Tensor:
    """s3prl S3PRLUpstream._match_length: replicate the last frame / trim."""
    tgt = s3prl_num_frames(num_samples, downsample_rate)
    T = h.shape[1]
    if T < tgt:
        h = torch.cat([h, h[:, -1:].expand(-1, tgt - T, -1)], dim=1)
    return h[:, :tgt]


MIN_SECOND = 0.05     # s3prl/nn/upstream.py
SAMPLE_RATE = 16000


def s3prl_upstream(wav: Tensor, sd: Dict[str, Tensor]) -> List[Tensor]:
    """S3PRLUpstream.forward on an equal-length batch (B, W): the 13 length-matched
    hidden states, each (B, len(range(0, W, 320)), 768), with the MIN_SECOND
    zero pad of short batches."""
    W = wav.shape[1]
    min_len = int(MIN_SECOND * SAMPLE_RATE)
    x = F.pad(wav, (0, min_len - W)) if W < min_len else wav
    tgt = s3prl_num_frames(W)
    return [match_length(h, x.shape[1])[:, :tgt] for h in hubert_hidden_states(x, sd)]


def s3prl_frontend(wav: Tensor, sd: Dict[str, Tensor]) -> Tensor:
    """S3prlFrontend.forward (multilayer_feature=True, layer=-1, frozen)."""
    hs = s3prl_upstream(wav, sd)
    w = torch.softmax(sd["frontend.featurizer.weights"], dim=-1)
    return sum(w[i] * h for i, h in enumerate(hs))
