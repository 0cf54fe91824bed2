"""The recipe drop-in (compat/wespeaker): a recipe directory whose `wespeaker`
symlink points at compat/wespeaker runs the reference command lines unchanged
(local/score.sh:46-50 `python wespeaker/bin/compute_metrics.py ...`,
tools/extract_embedding.sh:51 `python -u wespeaker/bin/extract.py ...`)."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _recipe(tmp_path):
    os.symlink(os.path.join(REPO, "compat", "wespeaker"), tmp_path / "wespeaker")
    return tmp_path


def test_compute_metrics_runs_from_a_recipe_symlink(tmp_path):
    d = _recipe(tmp_path)
    rng = np.random.default_rng(0)
    with open(d / "vox1_O_cleaned.kaldi.score", "w") as f:
        for i in range(400):
            tgt = i % 2 == 0
            s = rng.normal(0.6 if tgt else 0.1, 0.15)
            f.write(f"e{i} t{i} {s:.5f} {'target' if tgt else 'nontarget'}\n")
    out = subprocess.run([sys.executable, "wespeaker/bin/compute_metrics.py", "--p_target", "0.01", "--c_fa", "1",
                          "--c_miss", "1", "vox1_O_cleaned.kaldi.score"], cwd=d, capture_output=True, text=True,
                         check=True).stdout
    from wespeaker_hubert_amd.scoring import compute_metrics
    eer, dcf = compute_metrics(str(d / "vox1_O_cleaned.kaldi.score"), 0.01, 1, 1)
    assert "---- vox1_O_cleaned.kaldi.score -----" in out
    assert f"EER = {eer:.3f}" in out and f"= {dcf:.3f}" in out


def test_every_recipe_entry_point_has_a_launcher():
    # every wespeaker/bin script the recipes' extraction / scoring stages call
    # (tools/extract_embedding.sh, local/score.sh, score_norm.sh, score_calibration.sh)
    for m in ("extract", "score", "score_norm", "compute_metrics", "compute_det", "score_calibration"):
        assert os.path.isfile(os.path.join(REPO, "compat", "wespeaker", "bin", m + ".py"))
        assert os.path.isfile(os.path.join(REPO, "wespeaker_hubert_amd", "bin", m + ".py"))


def test_import_wespeaker_exports_the_reference_names(tmp_path):
    d = _recipe(tmp_path)
    out = subprocess.run([sys.executable, "-c", "import wespeaker; print(wespeaker.load_model.__module__, "
                          "callable(wespeaker.load_model_pt))"], cwd=d, capture_output=True, text=True,
                         check=True).stdout
    assert out.split() == ["wespeaker_hubert_amd", "True"]


def test_compute_det_writes_the_det_plot(tmp_path):
    """local/score.sh:54 `python wespeaker/bin/compute_det.py <scores>` -> <scores>.det.png."""
    d = _recipe(tmp_path)
    rng = np.random.default_rng(1)
    with open(d / "trials.score", "w") as f:
        for i in range(300):
            tgt = i % 3 == 0
            f.write(f"e{i} t{i} {rng.normal(0.5 if tgt else 0.0, 0.2):.5f} {'target' if tgt else 'nontarget'}\n")
    out = subprocess.run([sys.executable, "wespeaker/bin/compute_det.py", "trials.score"], cwd=d, capture_output=True,
                         text=True, check=True).stdout
    png = d / "trials.score.det.png"
    assert "DET curve saved in trials.score.det.png" in out
    assert png.is_file() and png.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"
