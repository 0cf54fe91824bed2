"""kaldi ark/scp byte format (kaldiio WriteHelper layout; parity with kaldiio
itself is unpinned — kaldiio is absent) and fire-style flag parsing."""
import struct

import numpy as np

from wespeaker_hubert_amd.bin import _fire
from wespeaker_hubert_amd.kaldi_io import WriteHelper, load_ark, load_scp_sequential


def test_ark_scp_roundtrip_and_bytes(tmp_path):
    ark = str(tmp_path / "x.ark")
    scp = str(tmp_path / "x.scp")
    rng = np.random.default_rng(0)
    vecs = {f"utt{i}": rng.standard_normal(192).astype(np.float32) for i in range(5)}
    with WriteHelper(f"ark,scp:{ark},{scp}") as w:
        for k, v in vecs.items():
            w(k, v)
    raw = open(ark, "rb").read()
    head = b"utt0 \x00BFV \x04" + struct.pack("<i", 192)
    assert raw.startswith(head)
    assert raw[len(head):len(head) + 192 * 4] == vecs["utt0"].tobytes()
    assert len(raw) == 5 * (len(head) + 192 * 4)
    lines = open(scp).read().splitlines()
    assert lines[0] == f"utt0 {ark}:5"
    assert lines[1] == f"utt1 {ark}:{5 + len(head) - 5 + 192 * 4 + 5}"
    got = dict(load_scp_sequential(scp))
    for k, v in vecs.items():
        np.testing.assert_array_equal(got[k], v)
    assert [k for k, _ in load_ark(ark)] == list(vecs)


def test_fire_parse():
    pos, kw = _fire.parse(["--exp_dir", "e", "--cal_mean", "True", "--batch-size", "16", "--top_n=300", "t1", "t2"])
    assert pos == ["t1", "t2"]
    assert kw == {"exp_dir": "e", "cal_mean": True, "batch_size": 16, "top_n": 300}
