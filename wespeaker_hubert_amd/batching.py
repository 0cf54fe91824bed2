"""Whole-utterance extraction in ragged batches.

The reference extracts evaluation sets one whole utterance at a time
(bin/extract.py with batch_size 1 -> Dataset(whole_utt=True), and
Speaker.extract_embedding_list, cli/speaker.py:170-179).  On the GPU a batch
of one 5 s utterance fills a few of the 256 CUs, so consecutive utterances are
packed into segmented batches (wsp_fbank_segments + wsp_model_forward_segments):
every embedding equals the batch-of-one result (same per-row arithmetic; convs
pad at utterance edges, pooling / SE / CMN per utterance).
"""
from __future__ import annotations

from typing import Iterable, Iterator, List, Sequence, Tuple

import numpy as np
import torch

from .frontend import FRAME_LEN, FRAME_SHIFT, compute_fbank, compute_fbank_segments

DEFAULT_MAX_FRAMES = 256 * 500  # ~ the bench batch (256 x 5 s) per launch


def _frames(n: int) -> int:
    return 1 + (n - FRAME_LEN) // FRAME_SHIFT if n >= FRAME_LEN else 0


def pack(lengths: Sequence[int], max_frames: int = DEFAULT_MAX_FRAMES) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) groups of utterances, each holding <= max_frames fbank frames
    (a single longer utterance forms its own group)."""
    groups, lo, acc = [], 0, 0
    for i, n in enumerate(lengths):
        f = _frames(n)
        if i > lo and acc + f > max_frames:
            groups.append((lo, i))
            lo, acc = i, 0
        acc += f
    if lo < len(lengths):
        groups.append((lo, len(lengths)))
    return groups


def _pack_samples(lengths: Sequence[int], budget: int) -> List[Tuple[int, int]]:
    groups, lo, acc = [], 0, 0
    for i, n in enumerate(lengths):
        if i > lo and acc + n > budget:
            groups.append((lo, i))
            lo, acc = i, 0
        acc += n
    if lo < len(lengths):
        groups.append((lo, len(lengths)))
    return groups


def embed_utterances(model, pcms: Sequence, device, max_frames: int = DEFAULT_MAX_FRAMES,
                     scale: float = 1.0, frontend=None) -> List[np.ndarray]:
    """Embeddings of whole utterances (int16-valued PCM), in input order.  With an SSL
    `frontend` (S3prlFrontend) the audio is fed as [-1, 1] floats (x / 32768, as
    torchaudio.load(normalize=True)), then CMN, then the backbone — all ragged."""
    out: List[np.ndarray] = []
    if frontend is not None:
        budget = max(1, max_frames) * 160  # samples per group, ~ the fbank-frame budget in audio time
        for lo, hi in _pack_samples([len(x) for x in pcms], budget):
            wav = [torch.from_numpy(np.asarray(x, np.float32) * (1.0 / 32768.0)) for x in pcms[lo:hi]]
            feats, offs = frontend.extract_segments(wav, cmn=True)
            off = torch.tensor(offs, dtype=torch.int32, device=feats.device)
            emb = model.embed_segments(feats, off).cpu().numpy()
            out.extend(emb[i] for i in range(hi - lo))
        return out
    if not getattr(model, "supports_segments", False):
        for x in pcms:  # ResNet: per-utterance forward
            feats = compute_fbank(torch.as_tensor(np.asarray(x, np.float32)).to(device)[None], scale=scale, cmn=True)
            outputs = model(feats)
            outputs = outputs[-1] if isinstance(outputs, tuple) else outputs
            out.append(outputs[0].cpu().numpy())
        return out
    for lo, hi in pack([len(x) for x in pcms], max_frames):
        wav = [torch.from_numpy(np.asarray(x, np.float32)) for x in pcms[lo:hi]]
        feats, off, _ = compute_fbank_segments(wav, scale=scale, cmn=True, device=device)
        emb = model.embed_segments(feats, off).cpu().numpy()
        out.extend(emb[i] for i in range(hi - lo))
    return out


def stream_groups(items: Iterable[Tuple[str, np.ndarray]], max_frames: int = DEFAULT_MAX_FRAMES
                  ) -> Iterator[Tuple[List[str], List[np.ndarray]]]:
    """Group a (key, pcm) stream into consecutive ragged batches of <= max_frames frames."""
    keys, pcms, acc = [], [], 0
    for k, x in items:
        f = _frames(len(x))
        if keys and acc + f > max_frames:
            yield keys, pcms
            keys, pcms, acc = [], [], 0
        keys.append(k)
        pcms.append(x)
        acc += f
    if keys:
        yield keys, pcms
