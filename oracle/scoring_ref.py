"""ORACLE (test infrastructure only): numpy restatement of the reference's
cosine / AS-Norm scoring and EER / minDCF metrics.  Pinned by
tests/golden/scoring.npz (made from the reference functions themselves).
"""
from __future__ import annotations

import numpy as np


def get_mean_std(emb: np.ndarray, cohort: np.ndarray, top_n: int):
    """bin/score_norm.py:26-36 — L2-normalise, S = E C^T, sort desc, top_n, mean, std(ddof=0)."""
    emb = emb / np.sqrt(np.sum(emb ** 2, axis=1, keepdims=True))
    cohort = cohort / np.sqrt(np.sum(cohort ** 2, axis=1, keepdims=True))
    s = np.matmul(emb, cohort.T)
    top = -np.sort(-s, axis=1)[:, :top_n]
    return np.mean(top, axis=1), np.std(top, axis=1)


def cosine(e1: np.ndarray, e2: np.ndarray) -> float:
    """sklearn cosine_similarity as used by bin/score.py:64-65 (float64 accumulate)."""
    a = e1.astype(np.float64).ravel()
    b = e2.astype(np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


def asnorm(score, e_mu, e_sd, t_mu, t_sd):
    """bin/score_norm.py:105-107."""
    return 0.5 * ((score - e_mu) / e_sd + (score - t_mu) / t_sd)


def compute_pmiss_pfa_rbst(scores, labels, weights=None):
    """utils/score_metrics.py:58-76."""
    idx = np.argsort(scores)
    labels = labels[idx]
    weights = np.ones(labels.shape, dtype="f8") if weights is None else weights[idx]
    tgt = weights * (labels == 1).astype("f8")
    imp = weights * (labels == 0).astype("f8")
    fnr = np.cumsum(tgt) / np.sum(tgt)
    fpr = 1 - np.cumsum(imp) / np.sum(imp)
    return fnr, fpr


def compute_eer(fnr, fpr, scores=None):
    """utils/score_metrics.py:79-93."""
    d = fnr - fpr
    x1 = np.flatnonzero(d >= 0)[0]
    x2 = np.flatnonzero(d < 0)[-1]
    a = (fnr[x1] - fpr[x1]) / (fpr[x2] - fpr[x1] - (fnr[x2] - fnr[x1]))
    eer = fnr[x1] + a * (fnr[x2] - fnr[x1])
    if scores is not None:
        return eer, np.sort(scores)[x1]
    return eer


def compute_c_norm(fnr, fpr, p_target, c_miss=1, c_fa=1):
    """utils/score_metrics.py:96-105."""
    c_det = min(c_miss * fnr * p_target + c_fa * fpr * (1 - p_target))
    c_def = min(c_miss * p_target, c_fa * (1 - p_target))
    return c_det / c_def
