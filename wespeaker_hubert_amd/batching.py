"""Whole-utterance extraction in ragged batches.

The reference extracts evaluation sets one whole utterance at a time
(bin/extract.py with batch_size 1 -> Dataset(whole_utt=True), and
Speaker.extract_embedding_list, cli/speaker.py:170-179).  On the GPU a batch
of one 5 s utterance fills a few of the 256 CUs, so consecutive utterances are
packed into segmented batches (wsp_fbank_segments_ex + wsp_model_forward_segments):
every embedding equals the batch-of-one result (same per-row arithmetic; convs
pad at utterance edges, pooling / SE / CMVN per utterance).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .frontend import DEFAULT, FbankArgs, apply_cmvn, compute_fbank, compute_fbank_segments

DEFAULT_MAX_FRAMES = 256 * 500  # ~ the bench batch (256 x 5 s) per launch


@dataclass(frozen=True)
class Cmvn:
    """bin/extract.py:104-106: `if test_conf.get('cmvn', True): apply_cmvn(feats,
    **test_conf.get('cmvn_args', {}))` (dataset_utils.py:19-26 defaults)."""
    enabled: bool = True
    norm_mean: bool = True
    norm_var: bool = False

    @classmethod
    def from_config(cls, test_conf: dict) -> "Cmvn":
        args = dict(test_conf.get("cmvn_args", {}) or {})
        unknown = set(args) - {"norm_mean", "norm_var"}
        if unknown:
            raise TypeError(f"apply_cmvn() got unexpected keyword arguments {sorted(unknown)}")
        return cls(bool(test_conf.get("cmvn", True)), bool(args.get("norm_mean", True)),
                   bool(args.get("norm_var", False)))

    @property
    def mean(self) -> bool:  # fused into the fbank / HuBERT launch
        return self.enabled and self.norm_mean

    @property
    def var(self) -> bool:  # a wsp_cmvn pass after it
        return self.enabled and self.norm_var


CMN = Cmvn()


def _frames(n: int, fbank_args: FbankArgs = DEFAULT) -> int:
    return fbank_args.num_frames(n)


def pack(lengths: Sequence[int], max_frames: int = DEFAULT_MAX_FRAMES,
         fbank_args: FbankArgs = DEFAULT) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) groups of utterances, each holding <= max_frames fbank frames
    (a single longer utterance forms its own group)."""
    return _pack_counts([_frames(n, fbank_args) for n in lengths], max_frames)


def _pack_counts(counts: Sequence[int], budget: int) -> List[Tuple[int, int]]:
    groups, lo, acc = [], 0, 0
    for i, n in enumerate(counts):
        if i > lo and acc + n > budget:
            groups.append((lo, i))
            lo, acc = i, 0
        acc += n
    if lo < len(counts):
        groups.append((lo, len(counts)))
    return groups


def _embed_ragged(model, feats: torch.Tensor, off: torch.Tensor, cmvn: Cmvn, mean_done: bool) -> np.ndarray:
    if cmvn.enabled and (cmvn.var or (cmvn.norm_mean and not mean_done)):
        apply_cmvn(feats, norm_mean=cmvn.norm_mean and not mean_done, norm_var=cmvn.norm_var, frame_offsets=off)
    return model.embed_segments(feats, off).cpu().numpy()


def _embed_one(model, feats: torch.Tensor, cmvn: Cmvn, mean_done: bool) -> np.ndarray:
    if cmvn.enabled and (cmvn.var or (cmvn.norm_mean and not mean_done)):
        apply_cmvn(feats, norm_mean=cmvn.norm_mean and not mean_done, norm_var=cmvn.norm_var)
    outputs = model(feats)
    outputs = outputs[-1] if isinstance(outputs, tuple) else outputs
    return outputs.cpu().numpy()


def embed_utterances(model, pcms: Sequence, device, max_frames: int = DEFAULT_MAX_FRAMES,
                     scale: float = 1.0, frontend=None, fbank_args: FbankArgs = DEFAULT,
                     cmvn: Cmvn = CMN) -> List[np.ndarray]:
    """Embeddings of whole utterances (int16-valued PCM), in input order.  With an SSL
    `frontend` (S3prlFrontend) the audio is fed as [-1, 1] floats (x / 32768, as
    torchaudio.load(normalize=True)), then CMVN, then the backbone — all ragged."""
    out: List[np.ndarray] = []
    if frontend is not None:
        budget = max(1, max_frames) * 160  # samples per group, ~ the fbank-frame budget in audio time
        for lo, hi in _pack_counts([len(x) for x in pcms], budget):
            wav = [torch.from_numpy(np.asarray(x, np.float32) * (1.0 / 32768.0)) for x in pcms[lo:hi]]
            feats, offs = frontend.extract_segments(wav, cmn=cmvn.mean)
            off = torch.tensor(offs, dtype=torch.int32, device=feats.device)
            emb = _embed_ragged(model, feats, off, cmvn, mean_done=True)
            out.extend(emb[i] for i in range(hi - lo))
        return out
    if not getattr(model, "supports_segments", False):
        for x in pcms:  # ResNet: per-utterance forward
            feats = compute_fbank(torch.as_tensor(np.asarray(x, np.float32)).to(device)[None], scale=scale,
                                  cmn=cmvn.mean, args=fbank_args)
            out.append(_embed_one(model, feats, cmvn, mean_done=True)[0])
        return out
    for lo, hi in pack([len(x) for x in pcms], max_frames, fbank_args):
        wav = [torch.from_numpy(np.asarray(x, np.float32)) for x in pcms[lo:hi]]
        feats, off, _ = compute_fbank_segments(wav, scale=scale, cmn=cmvn.mean, device=device, args=fbank_args)
        emb = _embed_ragged(model, feats, off, cmvn, mean_done=True)
        out.extend(emb[i] for i in range(hi - lo))
    return out


def embed_features(model, mats: Sequence[np.ndarray], device, max_frames: int = DEFAULT_MAX_FRAMES,
                   cmvn: Cmvn = CMN) -> List[np.ndarray]:
    """Embeddings of whole precomputed feature matrices ((T_b, feat_dim) float32, the
    `feat` data type: kaldiio.load_mat rows, dataset.py:173-199 with whole_utt), in input
    order; CMVN on the device, ragged batches where the backbone supports them."""
    out: List[np.ndarray] = []
    if not getattr(model, "supports_segments", False):
        for m in mats:
            feats = torch.from_numpy(np.ascontiguousarray(m, dtype=np.float32))[None].to(device)
            out.append(_embed_one(model, feats, cmvn, mean_done=False)[0])
        return out
    for lo, hi in _pack_counts([len(m) for m in mats], max_frames):
        rows = [np.ascontiguousarray(m, dtype=np.float32) for m in mats[lo:hi]]
        feats = torch.from_numpy(np.concatenate(rows, axis=0)).to(device)
        off_host = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int32)
        off = torch.from_numpy(off_host).to(device)
        emb = _embed_ragged(model, feats, off, cmvn, mean_done=False)
        out.extend(emb[i] for i in range(hi - lo))
    return out


def embed_feature_batch(model, mats: Sequence[np.ndarray], device, cmvn: Cmvn = CMN) -> np.ndarray:
    """One (B, T, F) batch of equal-length feature chunks (batch_size > 1 with `feat`)."""
    feats = torch.from_numpy(np.ascontiguousarray(np.stack(mats), dtype=np.float32)).to(device)
    return _embed_one(model, feats, cmvn, mean_done=False)


def stream_groups(items: Iterable[Tuple[str, np.ndarray]], max_frames: int = DEFAULT_MAX_FRAMES,
                  count: Optional[callable] = None) -> Iterator[Tuple[List[str], List[np.ndarray]]]:
    """Group a (key, item) stream into consecutive ragged batches of <= max_frames frames
    (`count(item)` frames per item; default: fbank frames of a 16 kHz waveform)."""
    count = count or (lambda x: _frames(len(x)))
    keys, items_, acc = [], [], 0
    for k, x in items:
        f = count(x)
        if keys and acc + f > max_frames:
            yield keys, items_
            keys, items_, acc = [], [], 0
        keys.append(k)
        items_.append(x)
        acc += f
    if keys:
        yield keys, items_
