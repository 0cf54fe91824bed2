"""world-8 CPU rehearsal of the multi-GPU extraction path (gloo, no GPU).

Each rank runs the product's `bin/extract.py` driver (tools/extract_embedding.sh:40-73: the data
list split contiguously with `split -l $((N/nj + 1))`, rank r writing `xvector_<r:03d>.ark/scp`,
the scps concatenated in rank order) and then one cohort-statistics pass through
`dist.allreduce_sums` (tools/vector_mean.py:24-53 over ranks).  Only the model's arithmetic is
stubbed — a deterministic function of each utterance's PCM in place of the HIP embedding, which
`tests/test_gpu_api.py::test_recipe_extract_embedding_sh_two_shards` covers on the GPU — so the
test checks the sharding, file naming, ark bytes and the collective at world sizes no GPU box
here offers: world 8 with 20 utterances (the last shard empty) and with 5 (three empty shards).
"""
import json
import os
import socket
import wave

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
import yaml

D = 8


def _write_wavs(root, n):
    rng = np.random.default_rng(5)
    lines = []
    for i in range(n):
        x = (rng.standard_normal(800 + 160 * (i % 7)) * 3000).astype(np.int16)
        path = os.path.join(root, f"u{i:03d}.wav")
        with wave.open(path, "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(16000)
            w.writeframes(x.tobytes())
        lines.append(json.dumps({"key": f"spk{i % 3}-u{i:03d}", "wav": path}))
    data_list = os.path.join(root, "wav.list")
    with open(data_list, "w") as f:
        f.write("\n".join(lines) + "\n")
    model_path = os.path.join(root, "avg_model.pt")
    torch.save({"w": torch.zeros(1)}, model_path)
    config = os.path.join(root, "config.yaml")
    with open(config, "w") as f:
        yaml.safe_dump({"model": "ECAPA_TDNN_c512", "model_args": {"feat_dim": 80, "embed_dim": D},
                        "dataset_args": {"fbank_args": {"num_mel_bins": 80, "frame_shift": 10, "frame_length": 25},
                                         "cmvn": True}}, f)
    return data_list, model_path, config


def _stub_embedding(pcm):
    """Deterministic stand-in for the HIP embedding: a fixed function of the utterance's PCM."""
    x = np.asarray(pcm, np.float64)
    v = [x.mean(), x.std(), np.abs(x).max(), len(x), x[::2].sum(), x[1::2].sum(), (x[1:] * x[:-1]).mean(), x[0]]
    return np.asarray(v, np.float32)


class _StubModel:
    def __init__(self, **kw):
        pass

    def load_state_dict(self, state, strict=True):
        pass

    def to(self, device):
        return self


def _rank_main(rank, world, port, data_list, model_path, config, out_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from wespeaker_hubert_amd import dist as wdist
    from wespeaker_hubert_amd.bin import extract as ex
    from wespeaker_hubert_amd.kaldi_io import load_scp_sequential

    # the GPU arithmetic is stubbed; the driver's file and shard logic runs as shipped
    torch.cuda.current_device = lambda: 0
    torch.cuda.device_count = lambda: 1
    ex.get_speaker_model = lambda name: _StubModel
    ex.embed_utterances = lambda model, pcms, device, max_frames, frontend=None, **kw: [_stub_embedding(p) for p in pcms]
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    scp = ex.extract(config=config, model_path=model_path, data_type="raw", data_list=data_list,
                     embed_ark=os.path.join(out_dir, "xvector.ark"), batch_size=1, num_workers=1)
    # one cohort pass: this rank's contiguous shard of the concatenated utterance list, per-speaker
    # f64 sums, ONE all-reduce (bin/vector_mean.py's collective)
    if world > 1:
        dist.barrier()  # every rank's scp is on disk
    keys, embs = [], []
    for r in range(world):
        path = os.path.join(out_dir, f"xvector_{r:03d}.scp") if world > 1 else scp
        for k, e in load_scp_sequential(path):
            keys.append(k)
            embs.append(e)
    lo, hi = wdist.shard_bounds(len(embs), rank, world)
    spk = np.array([int(k[3]) for k in keys], np.int64)
    acc = torch.zeros(3, D, dtype=torch.float64)
    cnt = torch.zeros(3, dtype=torch.float64)
    if hi > lo:
        acc.index_add_(0, torch.from_numpy(spk[lo:hi]), torch.from_numpy(np.stack(embs[lo:hi])).double())
        cnt.index_add_(0, torch.from_numpy(spk[lo:hi]), torch.ones(hi - lo, dtype=torch.float64))
    wdist.allreduce_sums(acc, cnt)
    q.put((rank, scp, (acc / cnt.clamp(min=1).unsqueeze(1)).numpy()))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, data_list, model_path, config, out_dir):
    os.makedirs(out_dir, exist_ok=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, data_list, model_path, config, out_dir, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, scp, means = q.get(timeout=240)
        res[r] = (scp, means)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _read_ark_records(scp_paths):
    from wespeaker_hubert_amd.kaldi_io import load_scp_sequential
    return [(k, e.tobytes()) for path in scp_paths for k, e in load_scp_sequential(path)]


@pytest.mark.parametrize("n_utts", [20, 5])
def test_world8_extract_shards_match_world1(tmp_path, n_utts):
    from wespeaker_hubert_amd.dist import shard_lines
    root = str(tmp_path)
    data_list, model_path, config = _write_wavs(root, n_utts)
    one = _run(1, data_list, model_path, config, os.path.join(root, "w1"))
    eight = _run(8, data_list, model_path, config, os.path.join(root, "w8"))
    lines = open(data_list).read().split("\n")[:-1]
    per = n_utts // 8 + 1  # split -l $((N / nj + 1))
    for r in range(8):
        scp = os.path.join(root, "w8", f"xvector_{r:03d}.scp")
        assert eight[r][0] == scp and os.path.exists(scp) and os.path.exists(scp[:-3] + "ark")
        want = [json.loads(ln)["key"] for ln in lines[r * per:(r + 1) * per]]
        assert want == [json.loads(ln)["key"] for ln in shard_lines(lines, r, 8)]
        with open(scp) as f:
            assert [ln.split()[0] for ln in f] == want
    if n_utts == 20:
        assert os.path.getsize(os.path.join(root, "w8", "xvector_007.scp")) == 0  # 3 x 7 + 0: tail empty
    else:
        assert all(os.path.getsize(os.path.join(root, "w8", f"xvector_{r:03d}.scp")) == 0 for r in (5, 6, 7))
    # cat in rank order == the world-1 run: same keys, same embedding bytes
    cat = _read_ark_records([os.path.join(root, "w8", f"xvector_{r:03d}.scp") for r in range(8)])
    ref = _read_ark_records([one[0][0]])
    assert [k for k, _ in cat] == [k for k, _ in ref]
    assert [b for _, b in cat] == [b for _, b in ref]
    # the one cohort all-reduce over 8 ranks (some with empty shards) equals the world-1 means
    for r in range(8):
        np.testing.assert_allclose(eight[r][1], one[0][1], rtol=0, atol=1e-9)
