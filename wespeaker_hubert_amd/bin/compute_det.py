"""DET curve — drop-in for wespeaker/bin/compute_det.py (local/score.sh:54,
score_norm.sh:66, score_calibration.sh:111): for every scores file
`<enroll> <test> <score> target|nontarget`, writes `<file>.det.png`."""
from __future__ import annotations

import sys

import numpy as np

from ..scoring import compute_pmiss_pfa_rbst, plot_det_curve
from . import _fire


def compute_det(scores_file: str, det_file: str) -> None:
    scores, labels = [], []
    with open(scores_file) as f:
        for line in f:
            tok = line.strip().split()
            scores.append(float(tok[2]))
            labels.append(tok[3] == "target")
    fnr, fpr = compute_pmiss_pfa_rbst(np.hstack(scores), np.hstack(labels))
    plot_det_curve(fnr, fpr, det_file)
    print("DET curve saved in {}".format(det_file))


def main(*scores_files):
    for f in scores_files:
        compute_det(str(f), str(f) + ".det.png")


if __name__ == "__main__":
    pos, _ = _fire.parse(sys.argv[1:])
    main(*pos)
