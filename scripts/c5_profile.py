"""Host-side profile of C5's scoring stages (development tool): synthetic eval / cohort files as
scripts/bench_c5.py prepares them, then bin/score, vector_mean, bin/score_norm and the metrics
under cProfile on the GPU box.  Writes the timings and the top functions by own time to stdout.

    python scripts/c5_profile.py [--top 30]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts"))

import bench_c5  # noqa: E402
from wespeaker_hubert_amd.bin import score as bin_score  # noqa: E402
from wespeaker_hubert_amd.bin import score_norm as bin_score_norm  # noqa: E402
from wespeaker_hubert_amd.bin.vector_mean import compute_vector_mean  # noqa: E402
from wespeaker_hubert_amd.kaldi_io import WriteHelper  # noqa: E402
from wespeaker_hubert_amd.scoring import compute_metrics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    root = tempfile.mkdtemp(prefix="wsp_c5p_")
    try:
        paths = bench_c5._prepare_files(root, 4874, 10000, 37611, 192, 0)
        rng = np.random.default_rng(3)
        ark = os.path.join(paths["eval_dir"], "xvector_000.ark")
        with WriteHelper("ark,scp:" + ark + "," + ark[:-3] + "scp") as w:
            for i in range(4874):
                w(f"e{i:05d}", rng.standard_normal(192).astype(np.float32))
        eval_scp = os.path.join(paths["eval_dir"], "xvector.scp")
        os.rename(ark[:-3] + "scp", eval_scp)
        score_file = os.path.join(paths["exp"], "scores", os.path.basename(paths["trials"]) + ".score")
        norm_file = score_file + ".asnorm"
        spk_ark = os.path.join(paths["cohort_dir"], "spk_xvector.ark")

        def stages():
            t = {}
            t0 = time.perf_counter()
            bin_score.main(paths["exp"], eval_scp, True, paths["cohort_dir"], paths["trials"])
            torch.cuda.synchronize(dev)
            t["score"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            compute_vector_mean(paths["spk2utt"], paths["cohort_scp"], spk_ark, device=dev)
            torch.cuda.synchronize(dev)
            t["vector_mean"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            bin_score_norm.main("asnorm", 300, score_file, norm_file, spk_ark[:-3] + "scp", eval_scp,
                                os.path.join(paths["cohort_dir"], "mean_vec.npy"))
            torch.cuda.synchronize(dev)
            t["score_norm"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            compute_metrics(norm_file)
            t["metrics"] = time.perf_counter() - t0
            return {k: round(v, 4) for k, v in t.items()}

        stages()
        print("warm", stages(), flush=True)
        print("warm", stages(), flush=True)
        pr = cProfile.Profile()
        pr.enable()
        stages()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
        print(s.getvalue())
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
