"""Diarization embedding front end: sub-segmentation of a speech segment's fbank
into fixed windows (mirror of wespeaker/diar/extract_emb.py:55-83 `subsegment`)
whose embeddings `Speaker.extract_embedding_feats` computes in GPU batches
(wespeaker/cli/speaker.py:106-121) — SURVEY.md §8(f) item 2.

Only the embedding batcher is on the MI355X path; VAD, clustering and RTTM
writing of the reference's diarize() stay out of scope.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def subsegment(fbank: np.ndarray, seg_id: str, window_fs: int, period_fs: int,
               frame_shift: int) -> Tuple[List[str], List[np.ndarray]]:
    """Split one segment's (frames, F) fbank into windows of `window_fs` frames every
    `period_fs` frames.

    seg_id ends in "-<begin>-<end>" (ms); the segment length in frames is
    (end - begin) // frame_shift (the reference notes it is 2 more than the fbank's
    frame count and uses it on purpose).  A window shorter than window_fs — the
    whole segment, or the tail window — is filled to window_fs frames by repeating
    its rows cyclically (np.resize).  Sub-segment ids append
    "-<first frame:08d>-<last frame:08d>".
    """
    begin, end = seg_id.split('-')[-2:]
    seg_len = (int(end) - int(begin)) // frame_shift
    dim = fbank.shape[1]
    ids: List[str] = []
    wins: List[np.ndarray] = []
    if seg_len <= window_fs:
        ids.append(f"{seg_id}-{0:08d}-{seg_len:08d}")
        wins.append(np.resize(fbank, (window_fs, dim)))
        return ids, wins
    for start in range(0, seg_len - window_fs + period_fs, period_fs):
        stop = min(start + window_fs, seg_len)
        ids.append(f"{seg_id}-{start:08d}-{stop:08d}")
        wins.append(np.resize(fbank[start:stop], (window_fs, dim)))
    return ids, wins
