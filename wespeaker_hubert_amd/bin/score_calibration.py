"""QMF score calibration — drop-in for wespeaker/bin/score_calibration.py (fire CLI,
three sub-commands, as run by the voxceleb recipes after `score_norm.py`):

  gather_calibration_factors --wav_dur_scp --max_dur --score_norm_file
                             --calibration_factor_file [--drop_duration]
  train_calibration_model    --calibration_factor_file --save_model_path
  infer_calibration          --calibration_factor_file --save_model_path
                             --calibration_score_file

The quality-measure features are the AS-Norm side outputs that
`score_norm.py` writes next to each normalised score (embedding magnitudes and
the two cohort means, score_norm.py:107-115), plus the two utterance durations.
A linear model on [score, quality measures] is fitted by minimising Cllr with
L-BFGS (score_calibration.py:66-139).  This is host-side float64 work over one
small feature row per trial; it runs on the CPU exactly as the reference does.
"""
from __future__ import annotations

import math
import os
import sys
from typing import List, Tuple

import numpy as np
import torch

from . import _fire


def _table(path: str) -> List[List[str]]:
    with open(path, "r", encoding="utf-8") as f:
        return [ln.strip().split() for ln in f if ln.strip()]


def _sorted_pair(a: float, b: float) -> str:
    """min, max, max - min, max / min with 4 decimals (score_calibration.py:38-43)."""
    lo, hi = (a, b) if a <= b else (b, a)
    return "{:.4f} {:.4f} {:.4f} {:.4f}".format(lo, hi, hi - lo, hi / lo)


def gather_calibration_factors(wav_dur_scp, max_dur, score_norm_file, calibration_factor_file,
                               drop_duration=False):
    """score_calibration.py:30-63: one line per trial,
    `enroll test label score [dur x4] mag x4 cohort_mean x4`."""
    if not os.path.exists(score_norm_file):
        raise AssertionError("score norm file ({}) does not exist !!!".format(score_norm_file))
    dur = {}
    if not drop_duration:
        dur = {r[0]: min(float(r[1]), float(max_dur)) for r in _table(wav_dur_scp)}
    with open(calibration_factor_file, "w", encoding="utf-8") as fout:
        for r in _table(score_norm_file):
            dur_str = "" if drop_duration else _sorted_pair(dur[r[0]], dur[r[1]])
            fout.write("{} {} {} {} {} {} {}\n".format(
                r[0], r[1], r[3], r[2], dur_str, _sorted_pair(float(r[4]), float(r[5])),
                _sorted_pair(float(r[6]), float(r[7]))))


def _read_factors(path: str) -> Tuple[List[List[str]], np.ndarray]:
    rows = _table(path)
    x = np.array([[float(v) for v in r[3:]] for r in rows], dtype=np.float64)
    return rows, x


def cllr(target_llrs: torch.Tensor, nontarget_llrs: torch.Tensor) -> torch.Tensor:
    """score_calibration.py:76-87: mean of -log sigmoid over both classes, in bits."""
    return 0.5 * (torch.log1p(torch.exp(-target_llrs)).mean() +
                  torch.log1p(torch.exp(nontarget_llrs)).mean()) / math.log(2)


def _linear(dim: int) -> torch.nn.Linear:
    # LinearModel init (score_calibration.py:68-71) happens in float32 and the model is
    # converted with .double() afterwards (:113): the start point is float32(1/dim).
    lin = torch.nn.Linear(dim, 1)
    with torch.no_grad():
        lin.weight.fill_(1.0 / dim)
        lin.bias.zero_()
    return lin.double()


def train_calibration_model(calibration_factor_file, save_model_path, max_epochs: int = 50):
    """score_calibration.py:90-139: L-BFGS (lr 0.01, torch defaults) on Cllr, at
    most `max_epochs` optimizer steps, stopping once a step improves the best
    loss by less than 1e-4.  Saves {'linear.weight', 'linear.bias'}."""
    rows, x = _read_factors(calibration_factor_file)
    tgt = np.array([r[2] in ("tgt", "target") for r in rows])
    xt = torch.from_numpy(x[tgt])
    xn = torch.from_numpy(x[~tgt])
    lin = _linear(x.shape[1])
    opt = torch.optim.LBFGS(lin.parameters(), lr=0.01)

    def closure():
        opt.zero_grad()
        loss = cllr(lin(xt), lin(xn))
        loss.backward()
        return loss

    best = 1e6
    for _ in range(int(max_epochs)):
        loss = float(opt.step(closure))
        if best - loss < 1e-4:
            break
        best = min(best, loss)
    torch.save({"linear.weight": lin.weight.detach().clone(), "linear.bias": lin.bias.detach().clone()},
               save_model_path)


def load_calibration_model(save_model_path) -> torch.nn.Linear:
    """infer_calibration loads the float64 weights into the still-float32 module and
    converts it afterwards (score_calibration.py:154-157): scores use float32-rounded
    weights in float64 arithmetic."""
    sd = torch.load(save_model_path, map_location="cpu", weights_only=True)
    w = sd["linear.weight"]
    lin = torch.nn.Linear(w.shape[1], 1)
    lin.load_state_dict({"weight": w, "bias": sd["linear.bias"]})
    return lin.double()


def infer_calibration(calibration_factor_file, save_model_path, calibration_score_file):
    """score_calibration.py:142-164: `enroll test calibrated_score label` per trial."""
    rows, x = _read_factors(calibration_factor_file)
    lin = load_calibration_model(save_model_path)
    with torch.no_grad():
        out = lin(torch.from_numpy(x)).reshape(-1).tolist()
    with open(calibration_score_file, "w", encoding="utf-8") as fout:
        for r, s in zip(rows, out):
            fout.write("{} {} {} {}\n".format(r[0], r[1], s, r[2]))


COMMANDS = {f.__name__: f for f in (gather_calibration_factors, train_calibration_model, infer_calibration)}

if __name__ == "__main__":
    pos, kw = _fire.parse(sys.argv[1:])
    if not pos or pos[0] not in COMMANDS:
        raise SystemExit(f"usage: score_calibration.py {{{','.join(COMMANDS)}}} --flags ...")
    COMMANDS[pos[0]](*pos[1:], **kw)
