"""Batch embedding extraction driver — drop-in for wespeaker/bin/extract.py.

Same flags as the reference (fire-style; `tools/extract_embedding.sh:51-62`):
  --config --model_path --data_type {raw,shard,feat} --data_list --embed_ark
  --batch-size --num-workers [--reverb_data --noise_data --aug-prob]
Writes `<embed_ark>` and `<embed_ark[:-3]>scp` (extract.py:86-88).

Semantics (bin/extract.py:33-120, dataset/dataset.py:136-247):
  * batch_size == 1: whole utterances, packed into ragged (segmented) batches of
    <= max_frames_per_batch frames (default 128000; each embedding equals the
    utterance's batch-of-one result); batch_size > 1: one random chunk of
    ((num_frms-1)*frame_shift + frame_length)*sr/1000 samples per utterance
    (processor.get_random_chunk, repeat-padded when shorter) — seeded here
    (`--chunk_seed`, default 0) so extraction is reproducible;
  * fbank on the GPU with the recipe's `fbank_args` (num_mel_bins,
    frame_length, frame_shift; dither forced to 0, extract.py:66-67) at
    `resample_rate`, then apply_cmvn as `dataset_args.cmvn` / `cmvn_args`
    say (extract.py:104-106; norm_mean fused into the fbank launch, norm_var
    a wsp_cmvn pass); or, with `dataset_args.frontend: s3prl` (hubert_base),
    the HuBERT front end on [-1, 1] audio (extract.py:100-102) + CMVN, then
    the backbone on its 768-dim frames;
  * `--data_type feat`: JSON lines {key, feat, spk} whose `feat` is a
    kaldiio.load_mat specifier (processor.parse_feat, processor.py:171-196;
    Kaldi FM / DM / CM / CM2 / CM3 matrices, kaldi_io.load_mat); whole
    matrices at batch_size 1, one `num_frms` random chunk per utterance
    (repeat-padded, processor.random_chunk(..., 'feat')) above it
    (dataset.py:193-199), then CMVN and the backbone;
  * under torchrun (WORLD_SIZE > 1) the data list is split into contiguous
    parts exactly like tools/extract_embedding.sh:40-42 and rank r writes
    `<embed_ark stem>_<r:03d>.ark/.scp` (cat the scps in rank order).
Audio decode runs on a host thread pool (`--num-workers`); augmentation
(aug_prob > 0) is not available on this path.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import random
import sys
import tarfile
import io
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, List, Tuple

import numpy as np
import torch
import yaml

from .. import audio
from ..batching import (DEFAULT_MAX_FRAMES, Cmvn, embed_feature_batch, embed_features, embed_utterances,
                        stream_groups)
from ..dist import shard_lines
from ..frontend import FbankArgs, apply_cmvn, compute_fbank
from ..kaldi_io import WriteHelper, load_mat, validate_path
from ..resample import resample
from ..s3prl_frontend import S3prlFrontend
from ..speaker_model import get_speaker_model
from . import _fire

AUDIO_FORMAT_SETS = {"flac", "mp3", "m4a", "ogg", "opus", "wav", "wma"}  # processor.py:34


def parse_config_or_kwargs(config_file, **kwargs):
    """utils/utils.py:37-51."""
    with open(config_file) as f:
        cfg = yaml.safe_load(f)
    return dict(cfg, **kwargs)


def read_lists(path: str) -> List[str]:
    with open(path, "r", encoding="utf8") as f:
        return [ln.strip() for ln in f if ln.strip()]


def iter_raw(lines: List[str]) -> Iterator[Tuple[str, str, list]]:
    for ln in lines:
        obj = json.loads(ln)
        yield obj["key"], obj["wav"], obj.get("vad")


def decode_raw(item) -> Tuple[str, np.ndarray, int]:
    key, wav, vad = item
    # processor.py:162-168 torchaudio.load(normalize=True); the stream carries the
    # int16-scale values compute_fbank sees (processor.py:492 `wav * (1 << 15)`)
    pcm, sr = audio.load_wav(wav, normalize=True)
    x = pcm[0] * np.float32(1 << 15)
    if vad:  # processor.parse_raw apply_vad: concatenate voiced segments
        x = np.concatenate([x[int(float(s) * sr):int(float(e) * sr)] for s, e in vad])
    return key, x, sr


def iter_shard(lines: List[str]) -> Iterator[Tuple[str, np.ndarray, int]]:
    """processor.tar_file_and_group (processor.py:70-110): files grouped by
    prefix, audio decoded by extension with torchaudio.load's normalize=True
    scaling (audio.load_audio).  Audio extensions this build cannot decode
    raise instead of being dropped from the ark."""
    for path in lines:
        with tarfile.open(path, mode="r:*") as tar:
            for ti in tar:
                prefix, _, ext = ti.name.rpartition(".")
                if ext in AUDIO_FORMAT_SETS:
                    data = tar.extractfile(ti).read()
                    x, sr = audio.load_audio(data, fmt=ext, normalize=True, name=f"{path}:{ti.name}")
                    yield prefix, x[0] * np.float32(1 << 15), sr  # int16 scale, as decode_raw


def decode_feat(line: str) -> Tuple[str, np.ndarray]:
    """processor.parse_feat (processor.py:171-196): a {key, feat, spk} JSON line,
    feat = kaldiio.load_mat(obj['feat'])."""
    obj = json.loads(line)
    assert "key" in obj and "feat" in obj and "spk" in obj
    return obj["key"], load_mat(obj["feat"])


def get_random_chunk(data: np.ndarray, chunk_len: int, rng: random.Random) -> np.ndarray:
    """processor.py:291-323 (1-D waveforms and (T, F) feature matrices: rows)."""
    n = len(data)
    if n >= chunk_len:
        s = rng.randint(0, n - chunk_len)
        return data[s:s + chunk_len].copy()
    reps = chunk_len // n + 1
    return np.tile(data, (reps,) + (1,) * (data.ndim - 1))[:chunk_len]


def extract(config="conf/config.yaml", **kwargs):
    configs = parse_config_or_kwargs(config, **kwargs)
    model_path = configs["model_path"]
    embed_ark = configs["embed_ark"]
    batch_size = int(configs.get("batch_size", 1))
    num_workers = max(1, int(configs.get("num_workers", 1)))
    test_conf = copy.deepcopy(configs["dataset_args"])
    frontend_type = test_conf.get("frontend", "fbank")
    if frontend_type not in ("fbank", "s3prl"):
        raise NotImplementedError(f"frontend {frontend_type!r} is not available on the MI355X path")
    if float(configs.get("aug_prob", 0.0) or 0.0) > 0:
        logging.warning("aug_prob > 0 ignored: augmentation is out of scope at extraction")
    cmvn = Cmvn.from_config(test_conf)  # extract.py:104-106
    data_type = configs["data_type"]
    if data_type not in ("raw", "shard", "feat"):
        raise ValueError(f"data_type {data_type!r}")  # dataset.py:160
    sr_target = int(test_conf.get("resample_rate", 16000))
    fbank_args = None
    if frontend_type == "fbank":
        # processor.compute_fbank(**fbank_args) at the resampled rate (dataset.py:227-229)
        fbank_args = FbankArgs.from_config(test_conf.get("fbank_args", {}), sample_rate=sr_target)
        if data_type != "feat":
            fbank_args.geometry()  # raises here for configurations the kernel does not implement
        frame_shift, frame_length = fbank_args.frame_shift, fbank_args.frame_length
    else:
        if data_type == "feat":
            raise NotImplementedError("data_type 'feat' carries fbank features; frontend s3prl reads audio")
        fa = test_conf["s3prl_args"]
        frame_shift, frame_length = int(fa.get("frame_shift", 10)), int(fa.get("frame_length", 25))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.device_count() > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
    device = torch.device("cuda", torch.cuda.current_device())

    model_args = dict(configs["model_args"])
    frontend = None
    if frontend_type == "s3prl":
        # extract.py:49-55: model.add_module("frontend", frontend_class(**s3prl_args, sample_rate=...))
        frontend = S3prlFrontend(**test_conf["s3prl_args"], sample_rate=sr_target)
        if int(model_args.get("feat_dim", -1)) == -1:  # bin/train.py:117-119
            model_args["feat_dim"] = frontend.output_size()
    model = get_speaker_model(configs["model"])(**model_args)
    state = torch.load(model_path, map_location="cpu", weights_only=True)
    if frontend is not None:
        frontend.load_state_dict({k: v for k, v in state.items() if k.startswith("frontend.")})
        state = {k: v for k, v in state.items() if not k.startswith("frontend.")}
        frontend.to(device)
    model.load_state_dict(state, strict=False)
    model.to(device)

    lines = read_lists(configs["data_list"])
    if world > 1:  # tools/extract_embedding.sh:40-42 contiguous split
        lines = shard_lines(lines, rank, world)
        stem = embed_ark[:-4] if embed_ark.endswith(".ark") else embed_ark
        embed_ark = f"{stem}_{rank:03d}.ark"
    validate_path(embed_ark)
    embed_ark = os.path.abspath(embed_ark)
    embed_scp = embed_ark[:-3] + "scp"

    if data_type == "raw":
        pool = ThreadPoolExecutor(num_workers)
        stream = pool.map(decode_raw, iter_raw(lines))
    elif data_type == "shard":
        stream = iter_shard(lines)
    else:
        pool = ThreadPoolExecutor(num_workers)
        stream = pool.map(decode_feat, lines)

    rng = random.Random(int(configs.get("chunk_seed", 0)))
    num_frms = int(test_conf.get("num_frms", 200))
    if data_type == "feat":
        chunk_len = num_frms  # dataset.py:193-199: random_chunk(num_frms, 'feat') over rows
    else:
        chunk_len = int(((num_frms - 1) * frame_shift + frame_length) * sr_target // 1000)  # dataset.py:212-215

    def run(keys, wavs, writer):
        if data_type == "feat":
            emb = embed_feature_batch(model, wavs, device, cmvn)
        else:
            x = torch.from_numpy(np.stack(wavs).astype(np.float32)).to(device)
            if frontend is None:
                feats = compute_fbank(x, scale=1.0, cmn=cmvn.mean, args=fbank_args)
            else:  # torchaudio.load(normalize=True) audio in [-1, 1]; norm_mean fused
                feats = frontend.extract(x * (1.0 / 32768.0), cmn=cmvn.mean)
            if cmvn.var:
                apply_cmvn(feats, norm_mean=False, norm_var=True)
            outputs = model(feats)  # extract.py:114-116: embed or (aux, embed)
            emb = (outputs[-1] if isinstance(outputs, tuple) else outputs).cpu().numpy()
        for k, e in zip(keys, emb):
            writer(k, e)

    def checked(items):
        # processor.py:242-260 `resample`: torchaudio.transforms.Resample(sr, resample_rate)
        # before chunking / fbank, here on the device (resample.Resample)
        if data_type == "feat":  # no resampling: features as stored
            yield from items
            return
        for key, x, sr in items:
            if sr != sr_target:
                x = resample(torch.from_numpy(np.asarray(x, np.float32)).to(device), sr, sr_target).cpu().numpy()
            yield key, x

    n = 0
    with torch.no_grad(), WriteHelper("ark,scp:" + embed_ark + "," + embed_scp) as writer:
        if batch_size == 1:
            # whole utterances, packed into ragged batches (each embedding = its batch-of-one result)
            max_frames = int(configs.get("max_frames_per_batch", DEFAULT_MAX_FRAMES))
            if data_type == "feat":
                groups = stream_groups(checked(stream), max_frames, count=len)
            elif frontend is None:
                groups = stream_groups(checked(stream), max_frames, count=lambda x: fbank_args.num_frames(len(x)))
            else:
                groups = stream_groups(checked(stream), max_frames)
            for keys, items in groups:
                if data_type == "feat":
                    embs = embed_features(model, items, device, max_frames, cmvn=cmvn)
                else:
                    embs = embed_utterances(model, items, device, max_frames, frontend=frontend,
                                            fbank_args=fbank_args or FbankArgs(), cmvn=cmvn)
                for k, e in zip(keys, embs):
                    writer(k, e)
                n += len(keys)
            print(f"extracted {n} embeddings -> {embed_scp}")
            return embed_scp
        keys, wavs = [], []
        for key, x in checked(stream):
            keys.append(key)
            wavs.append(get_random_chunk(x, chunk_len, rng))
            if len(keys) == batch_size:
                run(keys, wavs, writer)
                keys, wavs = [], []
            n += 1
        if keys:
            run(keys, wavs, writer)
    print(f"extracted {n} embeddings -> {embed_scp}")
    return embed_scp


def main(argv=None):
    pos, kw = _fire.parse(sys.argv[1:] if argv is None else argv)
    if pos:
        kw.setdefault("config", pos[0])
    extract(**kw)


if __name__ == "__main__":
    main()
