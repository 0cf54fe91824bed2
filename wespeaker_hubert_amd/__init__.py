"""wespeaker_hubert_amd — MI355X-native speaker-embedding extraction + scoring.

Drop-in for the reference package surface `wespeaker.load_model()` /
`wespeaker.load_model_pt()` (wespeaker/__init__.py:1-2) on the extraction hot
path: Kaldi fbank -> ECAPA-TDNN -> attentive statistics pooling -> embedding,
and cosine / AS-Norm scoring.  All compute runs in the hand-written gfx950
HIP library `libwsp_hip.so` (csrc/), reached through a C-ABI
(include/wespeaker_amd.h).
"""
__version__ = "0.1.0"


def load_model(model_name_or_path: str):
    from .cli.speaker import load_model as _lm
    return _lm(model_name_or_path)


def load_model_pt(model_name_or_path: str):
    from .cli.speaker import load_model_pt as _lmp
    return _lmp(model_name_or_path)
