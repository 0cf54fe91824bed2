"""AS-Norm / S-Norm — drop-in for wespeaker/bin/score_norm.py (fire CLI):
  --score_norm_method asnorm --top_n 300 --trial_score_file --score_norm_file
  --cohort_emb_scp --eval_emb_scp [--mean_vec_path]"""
from __future__ import annotations

import sys

import numpy as np

from ..kaldi_io import load_scp_matrix
from ..scoring import score_norm
from . import _fire


def main(score_norm_method, top_n, trial_score_file, score_norm_file, cohort_emb_scp, eval_emb_scp,
         mean_vec_path=None):
    mean_vec = np.load(mean_vec_path) if mean_vec_path else None
    cohort = load_scp_matrix(cohort_emb_scp)
    evals = load_scp_matrix(eval_emb_scp)
    score_norm(score_norm_method, int(top_n), trial_score_file, score_norm_file, cohort, evals, mean_vec)


if __name__ == "__main__":
    _, kw = _fire.parse(sys.argv[1:])
    main(**kw)
