"""The standalone kernel checks in the driver's GPU suite:
tools/gemm_check's operand forms no shipped model sends to tile family 7 (ragged row
bias, ragged k3 dilated conv, a 1x1 with input rows != output rows: the AM 1 identity
row-map rule of ADVICE r4) must equal family 6 bit for bit, and tools/tail_check's
partial frequency / time tiles of the fused ResNet bottleneck tail (tail2_kernel with
the next conv1 fused) must equal the tail alone bit for bit, with the fused conv1 within
1e-4 of a host float64 conv1.  Both binaries are built by __graft_entry__.build()
(`make -C wespeaker_hubert_amd/csrc tools`)."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEMM_CHECK = os.path.join(ROOT, "tools", "gemm_check")
TAIL_CHECK = os.path.join(ROOT, "tools", "tail_check")


def _run(args, timeout=120):
    if not os.path.exists(args[0]):
        pytest.fail(f"{args[0]} not built (run __graft_entry__.build())")
    p = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


@pytest.mark.parametrize("case", ["rb_ragged", "k3_ragged", "tiT_1x1"])
def test_gemm_family7_bit_identical_on_ragged_operands(case):
    rc, out = _run([GEMM_CHECK, case, "1", "67"])
    assert rc == 0, out
    m = re.search(r"family 7 vs 6: (\d+) of (\d+) outputs differ, (\d+) column-sum words differ", out)
    assert m and m.group(1) == "0" and m.group(3) == "0" and int(m.group(2)) > 0, out
    assert "all families bit-identical" in out


@pytest.mark.parametrize("C,B,F,T", [(128, 2, 5, 70), (64, 2, 7, 45), (32, 1, 11, 33), (128, 1, 2, 32)])
def test_res_tail_partial_tiles(C, B, F, T):
    rc, out = _run([TAIL_CHECK, str(C), str(B), str(F), str(T), "1"])
    assert rc == 0, out
    m = re.search(r"out: max \|diff\| (\S+) \(max \|ref\| (\S+)\)", out)
    assert m, out
    assert float(m.group(1)) == 0.0 and float(m.group(2)) > 0, out  # tail2 block outputs = the unfused tail
    assert "first mismatch" not in out
    m = re.search(r"y1n vs host f64 conv1 \((\d+) positions\): max \|diff\| (\S+)", out)
    assert m and int(m.group(1)) > 0 and float(m.group(2)) <= 1e-4, out
