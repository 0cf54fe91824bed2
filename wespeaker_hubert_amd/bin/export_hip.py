"""Export a wespeaker model directory (config.yaml + avg_model.pt) to the
safetensors file the C++ runtime backend loads (runtime/speaker_model_hip.h) —
the HIP sibling of the reference's bin/export_onnx.py / export_mnn.py.

    python -m wespeaker_hubert_amd.bin.export_hip --config exp/config.yaml \
        --checkpoint exp/avg_model.pt --output exp/final.safetensors

The state_dict goes through the same intake as load_model_pt (names checked
against the architecture's layout, training-only heads dropped with the
reference's warnings); the file holds the reference's tensor names with f32
data and metadata arch / feat_dim / embed_dim / emb_bn / two_emb_layer.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np
import torch
import yaml

from ..speaker_model import get_speaker_model


def export(config: str, checkpoint: str, output: str) -> str:
    from safetensors.numpy import save_file
    with open(config, "r") as f:
        cfg = yaml.safe_load(f)
    model = get_speaker_model(cfg["model"])(**cfg["model_args"])
    state = torch.load(checkpoint, map_location="cpu", weights_only=True)
    missing, _ = model.load_state_dict(state, strict=False)
    needed = [n for n in missing if not n.endswith("num_batches_tracked")]
    if needed:
        raise RuntimeError(f"checkpoint lacks {len(needed)} tensors, e.g. {needed[:3]}")
    arch, feat_dim, embed_dim, emb_bn, two_emb = model._create_args()
    tensors = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in model._host.items()}
    meta = {"arch": str(arch), "feat_dim": str(int(feat_dim)), "embed_dim": str(int(embed_dim)),
            "emb_bn": str(int(emb_bn)), "two_emb_layer": str(int(two_emb)), "format": "wespeaker_hubert_amd/1"}
    save_file(tensors, output, metadata=meta)
    return output


def main(argv=None):
    p = argparse.ArgumentParser(description="export a model for the C++ HIP runtime backend")
    p.add_argument("--config", required=True)
    p.add_argument("--checkpoint", required=True)
    p.add_argument("--output", required=True)
    a = p.parse_args(argv)
    print(export(a.config, a.checkpoint, a.output))


if __name__ == "__main__":
    sys.exit(main())
