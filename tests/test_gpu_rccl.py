"""RCCL on the one GPU the pool gives: a fresh process joins a
world-1 "nccl" (= RCCL on ROCm) process group over a TCP store -- set up before any GPU
call in that process -- and runs the extraction path's one collective,
dist.allreduce_sums (AS-Norm cohort statistics, bin/score.py:25-35,
tools/vector_mean.py:24-53), on float64 device buffers with the world-1 shortcut
bypassed, ordered behind a kernel on a side stream; then bench.py's rccl_check
against its closed form."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["WSP_ROOT"])
import torch
import torch.distributed as dist
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + os.environ["WSP_PORT"], rank=0, world_size=1)
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
from wespeaker_hubert_amd.dist import allreduce_sums
import bench
G, D = 777, 192
side = torch.cuda.Stream(dev)
with torch.cuda.stream(side):  # producer on a side stream, the collective on the current one
    x = torch.randn(G * 3, D, dtype=torch.float64, device=dev)
    acc = x.view(G, 3, D).sum(1)
    cnt = torch.full((G,), 3.0, dtype=torch.float64, device=dev)
torch.cuda.current_stream(dev).wait_stream(side)
want_acc, want_cnt = acc.clone(), cnt.clone()
acc2, cnt2 = allreduce_sums(acc, cnt, force=True)
torch.cuda.synchronize(dev)
ok_sum = bool(torch.equal(acc2, want_acc)) and bool(torch.equal(cnt2, want_cnt)) and acc2.data_ptr() == acc.data_ptr()
chk = bench.rccl_check(dev, 1, 0)
print("RESULT " + json.dumps({"backend": dist.get_backend(), "ok_sum": ok_sum, "check": chk}), flush=True)
dist.destroy_process_group()
'''


def test_rccl_world1_allreduce_on_device():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, WSP_ROOT=ROOT, WSP_PORT=str(port), MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    r = json.loads(line[7:])
    assert r["backend"] == "nccl"
    assert r["ok_sum"], r
    assert r["check"]["ok"] and r["check"]["backend"] == "nccl" and r["check"]["world"] == 1, r
