"""Per-speaker mean embeddings (cohort) — drop-in for tools/vector_mean.py:
  --spk2utt F --xvector_scp S --spk_xvector_ark A   (sums on the GPU, f64).

Under torchrun (WORLD_SIZE > 1) every rank sums its contiguous shard of the
utterance rows (dist.shard_bounds, the split of tools/extract_embedding.sh) and
the per-speaker f64 sums / counts are combined with ONE all-reduce
(dist.allreduce_sums: RCCL over xGMI for "nccl") — the cohort-statistics
collective of the north-star pipeline; rank 0 writes the ark/scp."""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from .. import dist as wdist
from ..kaldi_io import WriteHelper, load_scp_matrix, validate_path
from ..scoring import group_sums


def compute_vector_mean(spk2utt, xvector_scp, spk_xvector_ark, device="cuda"):
    spk2utts = {}
    with open(spk2utt, "r", encoding="utf-8") as f:
        for line in f:
            tok = line.strip().split(" ")
            if tok and tok[0]:
                spk2utts[tok[0]] = tok[1:]
    keys, mat = load_scp_matrix(xvector_scp)
    uidx = {k: i for i, k in enumerate(keys)}
    spks = list(spk2utts.keys())
    rows, groups = [], []
    for gi, spk in enumerate(spks):
        for utt in spk2utts[spk]:
            rows.append(uidx[utt])
            groups.append(gi)
    rank, world = wdist.world()
    lo, hi = wdist.shard_bounds(len(rows), rank, world)
    dim = mat.shape[1]
    if hi > lo:
        x = torch.from_numpy(np.ascontiguousarray(mat[rows[lo:hi]], dtype=np.float32)).to(device)
        acc, cnt = group_sums(x, np.asarray(groups[lo:hi], np.int32), len(spks))
    else:
        acc = torch.zeros(len(spks), dim, dtype=torch.float64, device=device)
        cnt = torch.zeros(len(spks), dtype=torch.float64, device=device)
    wdist.allreduce_sums(acc, cnt)
    means = (acc / cnt.unsqueeze(1)).cpu().numpy().astype(np.float32)
    if rank != 0:
        return means
    validate_path(spk_xvector_ark)
    ark = os.path.abspath(spk_xvector_ark)
    with WriteHelper("ark,scp:" + ark + "," + ark[:-3] + "scp") as w:
        for spk, m in zip(spks, means):
            w(spk, m)
    return means


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="compute the mean of vector")
    ap.add_argument("--spk2utt", type=str, default="")
    ap.add_argument("--xvector_scp", type=str, default="")
    ap.add_argument("--spk_xvector_ark", type=str, default="")
    a = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % torch.cuda.device_count())
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    compute_vector_mean(a.spk2utt, a.xvector_scp, a.spk_xvector_ark,
                        device=torch.device("cuda", torch.cuda.current_device()))
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
