"""Cosine trial scoring — drop-in for wespeaker/bin/score.py (fire CLI):
  python -m wespeaker_hubert_amd.bin.score --exp_dir E --eval_scp_path S \
      --cal_mean True --cal_mean_dir D trials...
Mean vector (score.py:25-35) and per-trial cosines (score.py:38-72) run on the GPU."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

from ..kaldi_io import load_scp_matrix
from ..scoring import group_sums, trials_cosine_score
from . import _fire


def calculate_mean_from_kaldi_vec(scp_path, device="cuda"):
    _, embs = load_scp_matrix(scp_path)
    x = torch.from_numpy(np.ascontiguousarray(embs, dtype=np.float32)).to(device)
    acc, cnt = group_sums(x, np.zeros(len(embs), np.int32), 1)
    return (acc[0] / cnt[0]).cpu().numpy().astype(embs.dtype)


def main(exp_dir, eval_scp_path, cal_mean, cal_mean_dir, *trials):
    if not cal_mean:
        mean_vec = None
    else:
        scp_path = os.path.join(cal_mean_dir, "xvector.scp")
        mean_vec = calculate_mean_from_kaldi_vec(scp_path)
        np.save(os.path.join(cal_mean_dir, "mean_vec.npy"), mean_vec)
    emb = load_scp_matrix(eval_scp_path)
    store = os.path.join(exp_dir, "scores")
    return trials_cosine_score(emb, trials, store, mean_vec)


if __name__ == "__main__":
    pos, kw = _fire.parse(sys.argv[1:])
    main(kw.pop("exp_dir"), kw.pop("eval_scp_path"), kw.pop("cal_mean", False), kw.pop("cal_mean_dir", None),
         *[str(p) for p in pos])
