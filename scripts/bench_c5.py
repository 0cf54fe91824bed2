"""C5 (BASELINE.json configs[4]): the vox1-O-shaped pipeline on synthetic data, through the
product's own file path (examples/voxceleb/v2/run.sh:104-123 stage by stage):

  extract     eval utterances split contiguously over ranks (tools/extract_embedding.sh:40-42),
              fbank + model on each rank (audio resident in HBM before the clock), each rank
              writing xvector_<rank>.ark/scp (kaldi ark, as bin/extract.py), rank 0 concatenating
              the scps in rank order (extract_embedding.sh:66-73);
  score       bin/score.py with cal_mean: the cohort set's mean vector (score.py:25-35), then the
              cosine of every trial -> scores/<trials>.score ({:.5f}, score.py:38-72);
  vector_mean bin/vector_mean.py: 10k cohort speaker means from the cohort xvector.scp + spk2utt,
              every rank summing its shard, ONE f64 all-reduce (RCCL over xGMI), rank 0 writing
              spk_xvector.ark/scp (tools/vector_mean.py:24-53);
  score_norm  bin/score_norm.py: AS-Norm (top 300) of every trial against the cohort means
              (score_norm.py:54-115) -> <trials>.score.asnorm;
  metrics     bin/compute_metrics.py's EER / minDCF(0.01) on the normalised score file.

The cohort set's utterance embeddings (2 per speaker) and the trial list are synthetic data
files prepared before the clock, as the recipe's earlier stages would have left them.
`run_c5` is the `configs.C5` sub-record of bench.py; run standalone as

    python scripts/bench_c5.py            (1 GPU)
    torchrun --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_c5.py
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from wespeaker_hubert_amd import dist as wdist  # noqa: E402
from wespeaker_hubert_amd.bin import score as bin_score  # noqa: E402
from wespeaker_hubert_amd.bin import score_norm as bin_score_norm  # noqa: E402
from wespeaker_hubert_amd.bin.vector_mean import compute_vector_mean  # noqa: E402
from wespeaker_hubert_amd.frontend import compute_fbank  # noqa: E402
from wespeaker_hubert_amd.kaldi_io import WriteHelper  # noqa: E402
from wespeaker_hubert_amd.scoring import compute_metrics  # noqa: E402
from wespeaker_hubert_amd.speaker_model import HipSpeakerModel  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict  # noqa: E402

STAGES = ("extract", "score", "vector_mean", "score_norm", "metrics")


def _prepare_files(root: str, eval_utts: int, cohort: int, trials: int, D: int, rank: int) -> dict:
    """Synthetic inputs of the scoring stages (rank 0 writes, every rank reads)."""
    paths = {"cohort_dir": os.path.join(root, "cohort"), "eval_dir": os.path.join(root, "eval"),
             "trials": os.path.join(root, "vox1_O_cleaned.kaldi"), "exp": os.path.join(root, "exp")}
    paths["cohort_scp"] = os.path.join(paths["cohort_dir"], "xvector.scp")
    paths["spk2utt"] = os.path.join(paths["cohort_dir"], "spk2utt")
    if rank == 0:
        for d in (paths["cohort_dir"], paths["eval_dir"], paths["exp"]):
            os.makedirs(d, exist_ok=True)
        rng = np.random.default_rng(7)
        spk = rng.standard_normal((cohort, D)).astype(np.float32)
        with WriteHelper("ark,scp:" + os.path.join(paths["cohort_dir"], "xvector.ark") + "," + paths["cohort_scp"]) as w:
            for s in range(cohort):
                for u in range(2):
                    w(f"c{s:05d}-{u}", spk[s] + 0.5 * rng.standard_normal(D).astype(np.float32))
        with open(paths["spk2utt"], "w") as f:
            for s in range(cohort):
                f.write(f"c{s:05d} c{s:05d}-0 c{s:05d}-1\n")
        r = np.random.default_rng(99)
        a, b = r.integers(0, eval_utts, trials), r.integers(0, eval_utts, trials)
        tgt = r.random(trials) < 0.5
        with open(paths["trials"], "w") as f:
            for i in range(trials):
                f.write(f"e{a[i]:05d} e{b[i]:05d} {'target' if tgt[i] else 'nontarget'}\n")
    return paths


def run_c5(arch: str = "ECAPA_TDNN_c1024", dev=None, world: int = 1, rank: int = 0, dist=None,
           eval_utts: int = 4874, seconds: float = 5.0, cohort: int = 10000, trials: int = 37611,
           top_n: int = 300, batch: int = 256, warmup: int = 1) -> dict:
    dev = dev or torch.device("cuda", torch.cuda.current_device())
    D = 192

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()

    root = tempfile.mkdtemp(prefix="wsp_c5_") if rank == 0 else None
    if dist is not None:  # every rank works in rank 0's directory (one host)
        obj = [root]
        dist.broadcast_object_list(obj, src=0)
        root = obj[0]
    try:
        paths = _prepare_files(root, eval_utts, cohort, trials, D, rank)
        model = HipSpeakerModel(arch, feat_dim=80, embed_dim=D)
        model.load_state_dict(synth_state_dict(1234, model.state_dict_layout()))
        model.to(dev)
        N = int(seconds * 16000)
        lo, hi = wdist.shard_bounds(eval_utts, rank, world)
        # this rank's shard of the eval audio, resident in HBM before the clock starts
        wavs = [(b0, torch.from_numpy(synth_audio(1000 + b0, min(batch, hi - b0), N)).to(dev))
                for b0 in range(lo, hi, batch)]
        barrier()
        trial_name = os.path.basename(paths["trials"])
        score_file = os.path.join(paths["exp"], "scores", trial_name + ".score")
        norm_file = score_file + ".asnorm"
        spk_ark = os.path.join(paths["cohort_dir"], "spk_xvector.ark")

        def run_once():
            t = {}
            barrier()
            t0 = time.perf_counter()
            # ---- extract: per-rank ark/scp, rank 0 concatenates the scps in rank order
            ark = os.path.join(paths["eval_dir"], f"xvector_{rank:03d}.ark")
            with torch.no_grad(), WriteHelper("ark,scp:" + ark + "," + ark[:-3] + "scp") as w:
                for b0, wav in wavs:
                    emb = model.embed(compute_fbank(wav, scale=1.0, cmn=True)).cpu().numpy()
                    for i in range(emb.shape[0]):
                        w(f"e{b0 + i:05d}", emb[i])
            barrier()
            if rank == 0:
                with open(os.path.join(paths["eval_dir"], "xvector.scp"), "w") as out:
                    for r in range(world):
                        with open(os.path.join(paths["eval_dir"], f"xvector_{r:03d}.scp")) as f:
                            out.write(f.read())
            barrier()
            t1 = time.perf_counter()
            t["extract"] = t1 - t0
            eval_scp = os.path.join(paths["eval_dir"], "xvector.scp")
            if rank == 0:
                # ---- bin/score.py with cal_mean: the cohort set's mean vector, then the cosine of
                # every trial (mean-subtracted) -> scores/<trials>.score
                bin_score.main(paths["exp"], eval_scp, True, paths["cohort_dir"], paths["trials"])
                torch.cuda.synchronize(dev)
                t["score"] = time.perf_counter() - t1
            barrier()
            # ---- cohort speaker means: every rank sums its shard, one all-reduce
            t3 = time.perf_counter()
            compute_vector_mean(paths["spk2utt"], paths["cohort_scp"], spk_ark, device=dev)
            barrier()
            t4 = time.perf_counter()
            t["vector_mean"] = t4 - t3
            if rank == 0:
                bin_score_norm.main("asnorm", top_n, score_file, norm_file, spk_ark[:-3] + "scp", eval_scp,
                                    os.path.join(paths["cohort_dir"], "mean_vec.npy"))
                torch.cuda.synchronize(dev)
                t5 = time.perf_counter()
                t["score_norm"] = t5 - t4
                eer, min_dcf = compute_metrics(norm_file)
                t["metrics"] = time.perf_counter() - t5
                t["eer_pct"], t["min_dcf"] = float(eer), float(min_dcf)
            barrier()
            t["total"] = time.perf_counter() - t0
            return t

        for _ in range(warmup):  # kernel code objects, top-n workspace, RCCL's first all-reduce, file caches
            run_once()
        t = run_once()
        with open(norm_file) as f:
            n_scored = sum(1 for _ in f) if rank == 0 else None
        del model, wavs
        torch.cuda.empty_cache()
    finally:
        if dist is not None:
            dist.barrier()
        if rank == 0:
            shutil.rmtree(root, ignore_errors=True)
    if rank != 0:
        return {}
    return {"metric": "vox1-O-shaped pipeline seconds (extract + mean vector + cosine trials + cohort means with one "
                      "all-reduce + AS-Norm + EER/minDCF), through the product's file path",
            "value": round(t["total"], 4), "unit": "s", "higher_is_better": False, "n_gpus": world,
            "stages_s": {k: round(t[k], 4) for k in STAGES},
            "eval_emb_per_s": round(eval_utts / t["extract"], 1),
            "trials_scored": n_scored, "eer_pct": t["eer_pct"], "min_dcf": t["min_dcf"],
            "warmup_passes": warmup,
            "config": {"arch": arch, "eval_utts": eval_utts, "seconds": seconds, "cohort_speakers": cohort,
                       "cohort_utts": 2 * cohort, "trials": trials, "top_n": top_n, "batch": batch},
            "data": "synthetic eval audio, synthetic cohort embeddings / trial list (random labels: EER ~50 %)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ECAPA_TDNN_c1024")
    ap.add_argument("--eval-utts", type=int, default=4874)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--cohort", type=int, default=10000)
    ap.add_argument("--trials", type=int, default=37611)
    ap.add_argument("--top-n", type=int, default=300)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=1, help="untimed passes of the whole pipeline first")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    r = run_c5(a.arch, dev, world, rank, dist, a.eval_utts, a.seconds, a.cohort, a.trials, a.top_n, a.batch,
               a.warmup)
    if rank == 0:
        print(json.dumps(r), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
