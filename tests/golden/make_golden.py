"""Generate golden fixtures from the REFERENCE implementation (survey container only).

Run once in the container where `/root/reference` exists:

    python tests/golden/make_golden.py

It imports the reference's own model / pooling / scoring code read-only from
`/root/reference/wespeaker` (package-init bypass documented in SURVEY.md §8(c):
`wespeaker/__init__.py` imports silero_vad/torchaudio/kaldiio which are absent),
loads seeded synthetic weights produced by `wespeaker_hubert_amd.synthetic`
(keyed by parameter name), runs the reference forward on seeded inputs and
stores ONLY inputs-seeds, input checksums and outputs as `.npz` fixtures.  No
reference source is copied; nothing under `/root/reference` is needed to *use*
the fixtures (GPU box included).

Reference call sites exercised:
  * ECAPA_TDNN_*           wespeaker/models/ecapa_tdnn.py:160-274
  * ResNet34 / ResNet293   wespeaker/models/resnet.py:110-260
  * ASTP / TSTP            wespeaker/models/pooling_layers.py:67-148
  * get_mean_std           wespeaker/bin/score_norm.py:26-36
  * compute_pmiss_pfa_rbst / compute_eer / compute_c_norm
                           wespeaker/utils/score_metrics.py:58-105
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from wespeaker_hubert_amd.synthetic import synth_feats, synth_state_dict  # noqa: E402

REF = "/root/reference"


def _import_reference():
    pkg = types.ModuleType("wespeaker")
    pkg.__path__ = [os.path.join(REF, "wespeaker")]
    sys.modules["wespeaker"] = pkg
    # import-only stubs: score_norm imports fire + kaldiio at module level but
    # get_mean_std never touches them; diar/extract_emb imports
    # kaldiio + onnxruntime at module level, its subsegment() uses numpy only.
    for stub in ("fire", "kaldiio", "onnxruntime"):
        if stub not in sys.modules:
            sys.modules[stub] = types.ModuleType(stub)
    from wespeaker.models import ecapa_tdnn, pooling_layers, resnet, samresnet  # noqa
    _import_reference.samresnet = samresnet
    from wespeaker.bin import score_norm  # noqa
    from wespeaker.utils import score_metrics  # noqa
    return ecapa_tdnn, resnet, pooling_layers, score_norm, score_metrics


def load_synth(model, seed, residual_tame=False):
    shapes = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    sd = synth_state_dict(seed, shapes, residual_tame=residual_tame)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    model.eval()
    return model


# (fixture name, ctor, ctor kwargs, weight seed, input seed, B, T, residual_tame)
MODEL_CASES = [
    ("ecapa_c512_b2_t200", "ECAPA_TDNN_c512", dict(feat_dim=80, embed_dim=192), 11, 101, 2, 200, False),
    ("ecapa_c512_b1_t301", "ECAPA_TDNN_c512", dict(feat_dim=80, embed_dim=192), 11, 102, 1, 301, False),
    ("ecapa_glob_c512_b2_t200", "ECAPA_TDNN_GLOB_c512", dict(feat_dim=80, embed_dim=192), 12, 103, 2, 200, False),
    ("ecapa_glob_c512_embbn_b2_t123", "ECAPA_TDNN_GLOB_c512",
     dict(feat_dim=80, embed_dim=256, emb_bn=True), 13, 104, 2, 123, False),
    ("ecapa_c1024_b2_t498", "ECAPA_TDNN_c1024", dict(feat_dim=80, embed_dim=192), 14, 105, 2, 498, False),
    ("ecapa_glob_c1024_b1_t150", "ECAPA_TDNN_GLOB_c1024", dict(feat_dim=80, embed_dim=192), 15, 106, 1, 150, False),
    ("ecapa_glob_c512_ssl768_b2_t250", "ECAPA_TDNN_GLOB_c512", dict(feat_dim=768, embed_dim=192), 16, 107, 2, 250, False),
    ("resnet34_b2_t200", "ResNet34", dict(feat_dim=80, embed_dim=256), 21, 201, 2, 200, True),
    ("resnet293_b1_t160", "ResNet293", dict(feat_dim=80, embed_dim=256), 22, 202, 1, 160, True),
    # hub "english" backbone (cli/hub.py:88) and the two-embedding-layer head (resnet.py:158-161,196-201)
    ("resnet221_b1_t120", "ResNet221", dict(feat_dim=80, embed_dim=256), 23, 203, 1, 120, True),
    ("resnet34_2emb_b2_t150", "ResNet34", dict(feat_dim=80, embed_dim=256, two_emb_layer=True), 24, 204, 2, 150, True),
    # samresnet.py:124-166 (hub "vblinkp"/"vblinkf" backbone); ctor takes acoustic_dim
    ("simam34_b2_t200", "SimAM_ResNet34_ASP", dict(acoustic_dim=80, embed_dim=256), 31, 301, 2, 200, True),
    ("simam34_inpl32_b1_t97", "SimAM_ResNet34_ASP", dict(in_planes=32, acoustic_dim=40, embed_dim=128),
     32, 302, 1, 97, True),
    ("simam100_b1_t123", "SimAM_ResNet100_ASP", dict(acoustic_dim=80, embed_dim=256), 33, 303, 1, 123, True),
]


def make_models(out, only=None):
    ecapa_tdnn, resnet, _, _, _ = _import_reference()
    for name, ctor, kw, wseed, iseed, B, T, tame in MODEL_CASES:
        if only and not any(o in name for o in only):
            continue
        mod = ecapa_tdnn if ctor.startswith("ECAPA") else (
            _import_reference.samresnet if ctor.startswith("SimAM") else resnet)
        torch.manual_seed(0)
        model = load_synth(getattr(mod, ctor)(**kw), wseed, residual_tame=tame)
        feat_dim = kw.get("feat_dim", kw.get("acoustic_dim"))
        x = synth_feats(iseed, B, T, feat_dim)
        inter = {}
        hooks = []
        if name == "ecapa_c512_b2_t200":
            for lname in ("layer1", "layer2", "layer3", "layer4", "conv", "pool"):
                def hook(_m, _i, o, lname=lname):
                    inter[lname] = o.detach().numpy().copy()
                hooks.append(getattr(model, lname).register_forward_hook(hook))
        with torch.no_grad():
            outs = model(torch.from_numpy(x))
        emb = outs[-1] if isinstance(outs, tuple) else outs
        for h in hooks:
            h.remove()
        rec = dict(arch=np.array(ctor), weight_seed=np.int64(wseed), input_seed=np.int64(iseed),
                   B=np.int64(B), T=np.int64(T), feat_dim=np.int64(feat_dim),
                   in_planes=np.int64(kw.get("in_planes", 64 if ctor.startswith("SimAM") else 32)),
                   embed_dim=np.int64(kw["embed_dim"]), emb_bn=np.int64(int(kw.get("emb_bn", False))),
                   two_emb_layer=np.int64(int(kw.get("two_emb_layer", False))),
                   residual_tame=np.int64(int(tame)),
                   input_sum=np.float64(x.astype(np.float64).sum()), input_head=x.reshape(-1)[:16].copy(),
                   param_names=np.array([k for k in model.state_dict()]),
                   param_shapes=np.array([",".join(map(str, v.shape)) for v in model.state_dict().values()]),
                   embed=emb.numpy().astype(np.float32))
        if inter:
            # channels-first (B,C,T) as the reference produces; keep only batch 0
            for k, v in inter.items():
                rec["inter_" + k] = v[:1].astype(np.float32)
        np.savez_compressed(os.path.join(out, name + ".npz"), **rec)
        print(name, emb.shape, float(emb.abs().max()), float(emb.std()))


def make_pooling(out):
    _, _, pooling_layers, _, _ = _import_reference()
    rng = np.random.default_rng(301)
    x = rng.standard_normal((2, 48, 37)).astype(np.float32) * 1.5 + 0.3
    res = {"x": x}
    torch.manual_seed(0)
    for tag, glob in (("astp", False), ("astp_glob", True)):
        p = pooling_layers.ASTP(in_dim=48, bottleneck_dim=16, global_context_att=glob)
        shapes = [(k, tuple(v.shape)) for k, v in p.state_dict().items()]
        sd = synth_state_dict(302 if glob else 303, shapes)
        p.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        with torch.no_grad():
            res[tag] = p(torch.from_numpy(x)).numpy()
        res[tag + "_seed"] = np.int64(302 if glob else 303)
    x4 = rng.standard_normal((2, 8, 5, 29)).astype(np.float32)
    res["x4"] = x4
    with torch.no_grad():
        res["tstp4"] = pooling_layers.TSTP(in_dim=40)(torch.from_numpy(x4)).numpy()
        res["tstp3"] = pooling_layers.TSTP(in_dim=48)(torch.from_numpy(x)).numpy()
    np.savez_compressed(os.path.join(out, "pooling.npz"), **res)
    print("pooling", {k: v.shape for k, v in res.items() if hasattr(v, "shape")})


# (segment id, frames, window_fs, period_fs): shorter than a window, exact
# multiples, ragged tails, the reference's "+2 frames" id/fbank mismatch
DIAR_CASES = [
    ("spk1-utt1-00000000-00001000", 98, 150, 75),
    ("spk1-utt1-00001000-00002500", 148, 150, 75),
    ("spk2-utt7-00000120-00004730", 459, 150, 75),
    ("spk2-utt7-00010000-00013330", 331, 150, 75),
    ("spk3-utt2-00000000-00006000", 598, 150, 50),
    ("spk3-utt2-00000000-00001510", 149, 150, 75),
]


def make_diar(out):
    """diar/extract_emb.py:55-83 subsegment() on synthetic fbanks."""
    import importlib
    _import_reference()
    extract_emb = importlib.import_module("wespeaker.diar.extract_emb")
    rng = np.random.default_rng(77)
    arrays = {}
    for n, (seg_id, frames, win, per) in enumerate(DIAR_CASES):
        fb = rng.standard_normal((frames, 8)).astype(np.float32)  # any feature dim
        ids, wins = extract_emb.subsegment(fb, seg_id, win, per, 10)
        arrays[f"fbank_{n}"] = fb
        arrays[f"ids_{n}"] = np.array(ids)
        arrays[f"wins_{n}"] = np.stack(wins).astype(np.float32)
        arrays[f"case_{n}"] = np.array([seg_id, str(win), str(per)])
    np.savez_compressed(os.path.join(out, "diar_subsegment.npz"), **arrays)
    print("diar cases", len(DIAR_CASES))


def make_scoring(out):
    _, _, _, score_norm, score_metrics = _import_reference()
    rng = np.random.default_rng(401)
    D = 64
    emb = rng.standard_normal((7, D)).astype(np.float32)
    cohort = rng.standard_normal((500, D)).astype(np.float32)
    mean_vec = (0.1 * rng.standard_normal(D)).astype(np.float32)
    mu, sd = score_norm.get_mean_std(emb - mean_vec, cohort - mean_vec, 100)
    mu_all, sd_all = score_norm.get_mean_std(emb - mean_vec, cohort - mean_vec, 500)
    # EER / minDCF on synthetic trials
    n = 3000
    labels = rng.random(n) < 0.3
    scores = np.where(labels, rng.normal(0.6, 0.15, n), rng.normal(0.1, 0.15, n))
    scores = np.round(scores, 5)
    fnr, fpr = score_metrics.compute_pmiss_pfa_rbst(scores, labels)
    eer, thres = score_metrics.compute_eer(fnr, fpr, scores)
    mindcf = score_metrics.compute_c_norm(fnr, fpr, p_target=0.01, c_miss=1, c_fa=1)
    mindcf5 = score_metrics.compute_c_norm(fnr, fpr, p_target=0.05, c_miss=1, c_fa=1)
    np.savez_compressed(os.path.join(out, "scoring.npz"), emb=emb, cohort=cohort, mean_vec=mean_vec,
                        top_n=np.int64(100), mu=mu, sd=sd, mu_all=mu_all, sd_all=sd_all,
                        scores=scores, labels=labels, eer=np.float64(eer), thres=np.float64(thres),
                        mindcf=np.float64(mindcf), mindcf5=np.float64(mindcf5))
    print("scoring eer", eer, "mindcf", mindcf)


def make_calibration(out):
    """bin/score_calibration.py:30-164 (gather -> train -> infer) on a synthetic
    AS-Norm side-output file; stores the inputs, the factor lines, the fitted
    weights and the calibrated scores."""
    import importlib
    import tempfile
    _import_reference()
    cal = importlib.import_module("wespeaker.bin.score_calibration")
    for stub in ("fire", "kaldiio", "onnxruntime"):  # torch.optim probes module specs: drop the stubs
        if getattr(sys.modules.get(stub), "__spec__", 0) is None:
            del sys.modules[stub]
    rng = np.random.default_rng(501)
    n_utt, n_trial = 40, 600
    utts = [f"id{i // 4:03d}/u{i:03d}.wav" for i in range(n_utt)]
    dur = rng.uniform(2.0, 20.0, n_utt)
    mag = rng.uniform(8.0, 14.0, n_utt)
    cmean = rng.uniform(0.05, 0.3, n_utt)
    a = rng.integers(0, n_utt, n_trial)
    b = (a + 1 + rng.integers(0, n_utt - 1, n_trial)) % n_utt
    tgt = (a // 4) == (b // 4)
    score = np.where(tgt, rng.normal(3.0, 1.2, n_trial), rng.normal(-0.5, 1.0, n_trial))
    with tempfile.TemporaryDirectory() as d:
        dur_scp, sn, fac = os.path.join(d, "dur"), os.path.join(d, "sn"), os.path.join(d, "fac")
        mdl, cs = os.path.join(d, "m.pt"), os.path.join(d, "cal")
        with open(dur_scp, "w") as f:
            for u, t in zip(utts, dur):
                f.write(f"{u} {t:.3f}\n")
        with open(sn, "w") as f:
            for i in range(n_trial):
                f.write("{} {} {:.5f} {} {:.4f} {:.4f} {:.4f} {:.4f}\n".format(
                    utts[a[i]], utts[b[i]], score[i], "target" if tgt[i] else "nontarget",
                    mag[a[i]], mag[b[i]], cmean[a[i]], cmean[b[i]]))
        cal.gather_calibration_factors(dur_scp, 15.0, sn, fac)
        cal.train_calibration_model(fac, mdl)
        cal.infer_calibration(fac, mdl, cs)
        sd = torch.load(mdl, weights_only=True)
        res = dict(dur_lines=np.array(open(dur_scp).read().splitlines()),
                   score_norm_lines=np.array(open(sn).read().splitlines()),
                   factor_lines=np.array(open(fac).read().splitlines()),
                   weight=sd["linear.weight"].numpy(), bias=sd["linear.bias"].numpy(),
                   calibrated_lines=np.array(open(cs).read().splitlines()), max_dur=np.float64(15.0))
    np.savez_compressed(os.path.join(out, "calibration.npz"), **res)
    print("calibration weight", res["weight"], "bias", res["bias"])


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 1)
    what = sys.argv[1:] or ["models", "pooling", "scoring", "diar", "calibration"]
    if "calibration" in what:
        make_calibration(HERE)
    if "pooling" in what:
        make_pooling(HERE)
    if "scoring" in what:
        make_scoring(HERE)
    if "diar" in what:
        make_diar(HERE)
    if "models" in what:  # `models simam` regenerates only the fixtures whose name contains "simam"
        make_models(HERE, [w for w in what if w not in ("models", "pooling", "scoring", "diar", "calibration")])
