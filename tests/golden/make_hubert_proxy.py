"""Golden fixture for the HuBERT-base front end from transformers' HubertModel
(offline third-party PROXY for s3prl's fairseq HuBERT; s3prl is absent and its
weights download by URL, so reference parity is unpinned — DESIGN.md §3).

Synthetic weights are generated under the canonical fairseq/s3prl names
(wespeaker_hubert_amd.arch.hubert_params), mapped onto the transformers module,
and the 13 hidden states are recorded.  Run: python tests/golden/make_hubert_proxy.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from wespeaker_hubert_amd.arch import HUBERT_PREFIX, hubert_params  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict  # noqa: E402

P = HUBERT_PREFIX


def fairseq_to_hf(name: str) -> str:
    n = name[len(P):]
    n = n.replace("feature_extractor.conv_layers.0.2.", "feature_extractor.conv_layers.0.layer_norm.")
    for i in range(7):
        n = n.replace(f"feature_extractor.conv_layers.{i}.0.", f"feature_extractor.conv_layers.{i}.conv.")
    if n.startswith("layer_norm."):
        n = "feature_projection." + n
    n = n.replace("post_extract_proj.", "feature_projection.projection.")
    n = n.replace("encoder.pos_conv.0.bias", "encoder.pos_conv_embed.conv.bias")
    n = n.replace("encoder.pos_conv.0.weight_g", "encoder.pos_conv_embed.conv.parametrizations.weight.original0")
    n = n.replace("encoder.pos_conv.0.weight_v", "encoder.pos_conv_embed.conv.parametrizations.weight.original1")
    n = n.replace(".self_attn_layer_norm.", ".layer_norm.").replace(".self_attn.", ".attention.")
    n = n.replace(".fc1.", ".feed_forward.intermediate_dense.").replace(".fc2.", ".feed_forward.output_dense.")
    return n


def main():
    from transformers import HubertConfig, HubertModel
    torch.manual_seed(0)
    model = HubertModel(HubertConfig()).eval()
    plist = [(n, s) for n, s in hubert_params() if n.startswith(P)]
    sd = synth_state_dict(41, plist)
    hf = model.state_dict()
    new = {}
    for n, v in sd.items():
        k = fairseq_to_hf(n)
        assert k in hf, k
        assert tuple(hf[k].shape) == tuple(v.shape), (k, hf[k].shape, v.shape)
        new[k] = torch.from_numpy(v)
    missing = [k for k in hf if k not in new]
    assert missing == ["masked_spec_embed"], missing
    new["masked_spec_embed"] = hf["masked_spec_embed"]
    model.load_state_dict(new, strict=True)
    rec = {}
    for tag, n in (("short", 8000), ("s1", 16000)):
        wav = synth_audio(51 if tag == "short" else 52, 2, n, int16_scale=False)
        with torch.no_grad():
            out = model(torch.from_numpy(wav), output_hidden_states=True)
        hs = out.hidden_states
        assert len(hs) == 13
        rec[f"{tag}_wav_seed"] = np.int64(51 if tag == "short" else 52)
        rec[f"{tag}_num_samples"] = np.int64(n)
        rec[f"{tag}_layer_sums"] = np.array([h.double().sum().item() for h in hs])
        rec[f"{tag}_layer_abs"] = np.array([h.double().abs().sum().item() for h in hs])
        if tag == "short":
            rec["short_hs0"] = hs[0].numpy()
            rec["short_hs6"] = hs[6].numpy()
            rec["short_hs12"] = hs[12].numpy()
        else:
            rec["s1_hs12"] = hs[12][:, :8].numpy()
        print(tag, hs[12].shape, float(hs[12].abs().max()))
    rec["weight_seed"] = np.int64(41)
    np.savez_compressed(os.path.join(HERE, "hubert_proxy.npz"), **rec)


if __name__ == "__main__":
    main()
