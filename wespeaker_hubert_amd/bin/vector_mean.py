"""Per-speaker mean embeddings (cohort) — drop-in for tools/vector_mean.py:
  --spk2utt F --xvector_scp S --spk_xvector_ark A   (sums on the GPU, f64)."""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from ..kaldi_io import WriteHelper, load_scp_sequential, validate_path
from ..scoring import group_sums


def compute_vector_mean(spk2utt, xvector_scp, spk_xvector_ark, device="cuda"):
    spk2utts = {}
    with open(spk2utt, "r", encoding="utf-8") as f:
        for line in f:
            tok = line.strip().split(" ")
            if tok and tok[0]:
                spk2utts[tok[0]] = tok[1:]
    utt2emb = dict(load_scp_sequential(xvector_scp))
    spks = list(spk2utts.keys())
    rows, groups = [], []
    for gi, spk in enumerate(spks):
        for utt in spk2utts[spk]:
            rows.append(utt2emb[utt])
            groups.append(gi)
    x = torch.from_numpy(np.stack(rows).astype(np.float32)).to(device)
    acc, cnt = group_sums(x, np.asarray(groups, np.int32), len(spks))
    means = (acc / cnt.unsqueeze(1)).cpu().numpy().astype(np.float32)
    validate_path(spk_xvector_ark)
    ark = os.path.abspath(spk_xvector_ark)
    with WriteHelper("ark,scp:" + ark + "," + ark[:-3] + "scp") as w:
        for spk, m in zip(spks, means):
            w(spk, m)


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="compute the mean of vector")
    ap.add_argument("--spk2utt", type=str, default="")
    ap.add_argument("--xvector_scp", type=str, default="")
    ap.add_argument("--spk_xvector_ark", type=str, default="")
    a = ap.parse_args()
    compute_vector_mean(a.spk2utt, a.xvector_scp, a.spk_xvector_ark)
