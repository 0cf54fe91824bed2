"""Cosine / AS-Norm scoring on the GPU, plus the reference's score-file formats.

Mirrors wespeaker/bin/score.py (trials_cosine_score, calculate_mean_from_kaldi_vec),
wespeaker/bin/score_norm.py (get_mean_std, AS-Norm / S-Norm main),
tools/vector_mean.py (compute_vector_mean) and the EER/minDCF metrics of
wespeaker/utils/score_metrics.py used by bin/compute_metrics.py.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def l2_normalize(x: torch.Tensor, sub: Optional[torch.Tensor] = None) -> torch.Tensor:
    x = x.float().contiguous()
    y = torch.empty_like(x)
    R, D = x.shape
    subp = sub.float().contiguous().data_ptr() if sub is not None else None
    _lib.check(_lib.load().wsp_l2_normalize(x.data_ptr(), subp, y.data_ptr(), R, D, _stream(x)),
               "wsp_l2_normalize")
    return y


def asnorm_stats(emb: torch.Tensor, cohort: torch.Tensor, top_n: int,
                 mean_vec: Optional[torch.Tensor] = None) -> Tuple[np.ndarray, np.ndarray]:
    """get_mean_std (score_norm.py:26-36) on (emb - mean_vec), (cohort - mean_vec)."""
    e = l2_normalize(emb, mean_vec)
    c = l2_normalize(cohort, mean_vec)
    Ne, D = e.shape
    Nc = c.shape[0]
    if top_n < 1:
        raise ValueError(f"top_n={top_n} must be >= 1")
    top_n = min(int(top_n), Nc)  # score_norm.py:33 slices [:, :top_n]: an oversized top_n is the whole cohort
    nbytes = ctypes.c_size_t()
    _lib.check(_lib.load().wsp_asnorm_workspace_bytes(Ne, Nc, D, ctypes.byref(nbytes)), "asnorm ws")
    ws = torch.empty(nbytes.value, dtype=torch.uint8, device=e.device)
    mu = torch.empty(Ne, dtype=torch.float64, device=e.device)
    sd = torch.empty(Ne, dtype=torch.float64, device=e.device)
    _lib.check(_lib.load().wsp_asnorm_stats(e.data_ptr(), Ne, c.data_ptr(), Nc, D, int(top_n), mu.data_ptr(),
                                            sd.data_ptr(), ws.data_ptr(), ws.numel(), _stream(e)),
               "wsp_asnorm_stats")
    return mu.cpu().numpy(), sd.cpu().numpy()


def cosine_pairs(E: torch.Tensor, idx_a, idx_b) -> np.ndarray:
    E = E.float().contiguous()
    ia = torch.as_tensor(np.asarray(idx_a, dtype=np.int32), device=E.device)
    ib = torch.as_tensor(np.asarray(idx_b, dtype=np.int32), device=E.device)
    out = torch.empty(ia.numel(), dtype=torch.float64, device=E.device)
    _lib.check(_lib.load().wsp_cosine_pairs(E.data_ptr(), E.shape[1], ia.data_ptr(), ib.data_ptr(), ia.numel(),
                                            out.data_ptr(), _stream(E)), "wsp_cosine_pairs")
    return out.cpu().numpy()


def group_sums(x: torch.Tensor, groups, n_groups: int) -> Tuple[torch.Tensor, torch.Tensor]:
    x = x.float().contiguous()
    g = torch.as_tensor(np.asarray(groups, dtype=np.int32), device=x.device)
    acc = torch.zeros(n_groups, x.shape[1], dtype=torch.float64, device=x.device)
    cnt = torch.zeros(n_groups, dtype=torch.float64, device=x.device)
    _lib.check(_lib.load().wsp_row_mean_accum(x.data_ptr(), g.data_ptr(), x.shape[0], x.shape[1],
                                              acc.data_ptr(), cnt.data_ptr(), _stream(x)), "wsp_row_mean_accum")
    return acc, cnt


def group_means(x: torch.Tensor, groups, n_groups: int) -> np.ndarray:
    acc, cnt = group_sums(x, groups, n_groups)
    return (acc / cnt.clamp(min=1).unsqueeze(1)).cpu().numpy()


# ------------------------------------------------------------- metrics ---
def compute_pmiss_pfa_rbst(scores, labels, weights=None):
    """score_metrics.py:58-76."""
    idx = np.argsort(scores)
    labels = np.asarray(labels)[idx]
    weights = np.ones(labels.shape, dtype="f8") if weights is None else np.asarray(weights)[idx]
    tgt = weights * (labels == 1).astype("f8")
    imp = weights * (labels == 0).astype("f8")
    return np.cumsum(tgt) / np.sum(tgt), 1 - np.cumsum(imp) / np.sum(imp)


def compute_eer(fnr, fpr, scores=None):
    """score_metrics.py:79-93."""
    d = fnr - fpr
    x1 = np.flatnonzero(d >= 0)[0]
    x2 = np.flatnonzero(d < 0)[-1]
    a = (fnr[x1] - fpr[x1]) / (fpr[x2] - fpr[x1] - (fnr[x2] - fnr[x1]))
    eer = fnr[x1] + a * (fnr[x2] - fnr[x1])
    if scores is not None:
        return eer, np.sort(scores)[x1]
    return eer


def compute_c_norm(fnr, fpr, p_target, c_miss=1, c_fa=1):
    """score_metrics.py:96-105."""
    c_det = min(c_miss * fnr * p_target + c_fa * fpr * (1 - p_target))
    return c_det / min(c_miss * p_target, c_fa * (1 - p_target))


def plot_det_curve(fnr, fpr, save_path: str) -> None:
    """score_metrics.py:119-160: the DET curve on normal-deviate axes with the EER
    point marked, saved to `save_path` (matplotlib, non-interactive backend)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from scipy.stats import norm
    ticks = [0.0001, 0.0002, 0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.4]
    plt.plot(norm.ppf(fpr), norm.ppf(fnr), "r")
    plt.xticks(norm.ppf(ticks), [str(x * 100) for x in ticks])
    plt.yticks(norm.ppf(ticks), [str(x * 100) for x in ticks])
    plt.xlim(norm.ppf([0.00051, 0.5]))
    plt.ylim(norm.ppf([0.00051, 0.5]))
    plt.xlabel("false-alarm rate [%]", fontsize=12)
    plt.ylabel("false-reject rate [%]", fontsize=12)
    eer = compute_eer(fnr, fpr)
    plt.plot(norm.ppf(eer), norm.ppf(eer), "o")
    plt.annotate("EER = %.2f%%" % (eer * 100), xy=(norm.ppf(eer), norm.ppf(eer)), xycoords="data",
                 xytext=(norm.ppf(eer + 0.05), norm.ppf(eer + 0.05)), textcoords="data",
                 arrowprops=dict(arrowstyle="-|>", connectionstyle="arc3, rad=+0.2", fc="w"), size=12,
                 va="center", ha="center", bbox=dict(boxstyle="round4", fc="w"))
    plt.grid()
    plt.savefig(save_path)
    plt.clf()


# --------------------------------------------------------- file drivers ---
def read_trials(path: str) -> List[List[str]]:
    with open(path, "r", encoding="utf8") as f:
        return [t for t in (ln.split() for ln in f) if t]


def as_table(emb) -> Tuple[List[str], np.ndarray, Dict[str, int]]:
    """Embeddings as (keys, [n][D] float32 matrix, key -> row): a {key: vector} dict or a
    (keys, matrix) pair from kaldi_io.load_scp_matrix (later duplicates win, as in a dict)."""
    if isinstance(emb, tuple):
        keys, mat = emb
        index = {k: i for i, k in enumerate(keys)}
        return list(keys), np.ascontiguousarray(mat, dtype=np.float32), index
    keys = list(emb.keys())
    return keys, np.stack([emb[k] for k in keys]).astype(np.float32), {k: i for i, k in enumerate(keys)}


def trials_cosine_score(emb, trials: Sequence[str], store_dir: str,
                        mean_vec: Optional[np.ndarray] = None, device: str = "cuda") -> List[str]:
    """bin/score.py:38-72 on the GPU; writes `<trial>.score` with `{:.5f}` scores.  `emb`: a
    {key: vector} dict or a (keys, matrix) pair (as_table)."""
    _, mat, kidx = as_table(emb)
    E = torch.from_numpy(mat).to(device)
    if mean_vec is not None:
        E = E - torch.from_numpy(np.asarray(mean_vec, dtype=np.float32)).to(device)
    out_paths = []
    os.makedirs(store_dir, exist_ok=True)
    for trial in trials:
        lines = read_trials(trial)
        ia = [kidx[s[0]] for s in lines]
        ib = [kidx[s[1]] for s in lines]
        sc = cosine_pairs(E, ia, ib)
        path = os.path.join(store_dir, os.path.basename(trial) + ".score")
        with open(path, "w") as w:
            w.write("".join(f"{s[0]} {s[1]} {v:.5f} {s[2]}\n" if len(s) == 3 else f"{s[0]} {s[1]} {v:.5f}\n"
                            for s, v in zip(lines, np.asarray(sc, np.float64).tolist())))
        out_paths.append(path)
    return out_paths


def score_norm(score_norm_method: str, top_n: int, trial_score_file: str, score_norm_file: str,
               cohort, eval_emb, mean_vec: Optional[np.ndarray] = None, device: str = "cuda") -> None:
    """bin/score_norm.py:54-115 (asnorm / snorm) with the statistics on the GPU.  `cohort` /
    `eval_emb`: {key: vector} dicts or (keys, matrix) pairs (as_table)."""
    rows = read_trials(trial_score_file)
    enroll = sorted(set(r[0] for r in rows))
    test = sorted(set(r[1] for r in rows))
    _, emat, eidx = as_table(eval_emb)
    mv = np.zeros(emat.shape[1], np.float32) if mean_vec is None else np.asarray(mean_vec, np.float32)
    _, cmat, _ = as_table(cohort)
    C = torch.from_numpy(cmat).to(device)
    if score_norm_method == "snorm":
        top_n = C.shape[0]
    elif score_norm_method != "asnorm":
        raise ValueError(score_norm_method)
    mvt = torch.from_numpy(mv).to(device)
    Ee = emat[[eidx[k] for k in enroll]]
    Et = emat[[eidx[k] for k in test]]
    e_mu, e_sd = asnorm_stats(torch.from_numpy(Ee).to(device), C, top_n, mvt)
    t_mu, t_sd = asnorm_stats(torch.from_numpy(Et).to(device), C, top_n, mvt)
    ei = {k: i for i, k in enumerate(enroll)}
    ti = {k: i for i, k in enumerate(test)}
    e_mag = np.linalg.norm(Ee - mv, axis=1)
    t_mag = np.linalg.norm(Et - mv, axis=1)
    # whole-trial-list arithmetic in the per-row order of score_norm.py:103-111 (float64, so
    # every value and every formatted line equals the per-row form), one write
    n = len(rows)
    ia = np.fromiter((ei[r[0]] for r in rows), np.int64, n)
    ib = np.fromiter((ti[r[1]] for r in rows), np.int64, n)
    s = np.fromiter((float(r[2]) for r in rows), np.float64, n)
    ns = 0.5 * ((s - e_mu[ia]) / e_sd[ia] + (s - t_mu[ib]) / t_sd[ib])
    with open(score_norm_file, "w", encoding="utf-8") as fout:
        fout.write("".join(
            f"{r[0]} {r[1]} {v:.5f} {r[3]} {ma:.4f} {mb:.4f} {ua:.4f} {ub:.4f}\n"
            for r, v, ma, mb, ua, ub in zip(rows, ns.tolist(), e_mag[ia].tolist(), t_mag[ib].tolist(),
                                            e_mu[ia].tolist(), t_mu[ib].tolist())))


def compute_metrics(scores_file: str, p_target=0.01, c_miss=1, c_fa=1) -> Tuple[float, float]:
    """bin/compute_metrics.py:25-50 -> (EER %, minDCF)."""
    with open(scores_file) as f:
        rows = [t for t in (ln.split() for ln in f) if t]
    # the same float(tok[2]) / tok[3] == "target" per line as the reference, in two list passes
    scores = np.array([float(t[2]) for t in rows], dtype=np.float64)
    labels = np.array([t[3] == "target" for t in rows], dtype=bool)
    fnr, fpr = compute_pmiss_pfa_rbst(scores, labels)
    eer, _ = compute_eer(fnr, fpr, scores)
    return 100 * eer, compute_c_norm(fnr, fpr, p_target, c_miss, c_fa)
