"""Headline benchmark: embeddings/sec on synthetic 5 s 16 kHz utterances.

Workload (BASELINE.json configs[1], C2): ECAPA_TDNN_c1024, Kaldi fbank80 front
end, batch 256 x 80 000-sample utterances per GPU, resident in HBM before the
timed region.  One step = fbank + CMN + ECAPA forward + embedding for the whole
batch, all in libwsp_hip.so.  Multi-GPU: one rank per GPU (torchrun), each
rank extracts its own shard (weak scaling, no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W]

`--gpus N` without a torchrun environment starts N ranks itself (torchrun as a
child process, before anything touches the GPU) and relays rank 0's line;
under torchrun WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from wespeaker_hubert_amd.arch import (RESNET_ARCHS, ecapa_gflop_per_utt, hubert_gflop_per_utt,  # noqa: E402
                                       make_spec, resnet_gflop_per_utt, simam_gflop_per_utt)
from wespeaker_hubert_amd.frontend import compute_fbank  # noqa: E402
from wespeaker_hubert_amd.s3prl_frontend import S3prlFrontend  # noqa: E402
from wespeaker_hubert_amd.speaker_model import HipSpeakerModel  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)
HBM_PEAK_GBPS = 8000.0
def x3_tile(variant, N: int, K: int, gelu: bool = False):
    """(template prefix, BM, BN, threads) of the bf16x3 block launch_conv_gemm_x3 picks."""
    v = 5 if variant is None else variant
    if v in (5, 6, 7) and N % 256 == 0:
        return "ILi4ELi2ELi2ELi4E", 256, 256, 512
    if v in (1, 4, 5, 6, 7):
        return "ILi4ELi2ELi2ELi2E", 256, 128, 512
    return "ILi2ELi2ELi2ELi2E", 128, 128, 256


def dominant_symbol(precision: int, variant, N: int, K: int, role: int, se_fused: bool = True):
    """Kernel-symbol prefix and block geometry of the SE-Res2Block 1x1 CxC conv
    (role 1) or a plain role-0 1-D GEMM (the HuBERT FFN fc1)."""
    if precision == 0:
        return "_ZN3wsp12_GLOBAL__N_113conv_gemm_f32ILi2ELi2ELi2ELi2ELi0ELb1E", 128, 128, 256
    t, bm, bn, nt = x3_tile(variant, N, K, gelu=(role == 0))  # role 0 here = HuBERT fc1 (GELU)
    if variant == 7 and bn == 256:
        # family 7 (conv_gemm_x3_t6.hip, conv_gemm_g<AM, CSK>, AM 1 = dense 1x1): the SE-Res2Block
        # conv3 (role 1) runs the column-sum instance when the SE squeeze is fused (uniform batches
        # with T >= 256 rows), the plain one otherwise
        return G_SYMBOL + ("ILi1ELb1E" if role == 1 and se_fused else "ILi1ELb0E"), bm, bn, nt
    sym = f"_ZN3wsp12_GLOBAL__N_112conv_gemm_x3{t}Li0ELb1ELi{role}E" + ("" if role else "Lb0E")
    if bn == 256:  # the 256 x 256 tile (one staging set): 32x32x16 (variant 5) or 16x16x32 (6) MFMAs
        sym += ("" if role == 0 else "Lb0E") + "Lb1ELi1E" + ("Li16E" if variant in (6, 7) else "Li32E")
    return sym, bm, bn, nt

# family 7's LDS-DMA tile kernel conv_gemm_g<AM, CSK> (conv_gemm_x3_t6.hip; AM 1 = dense, 0 = conv)
G_SYMBOL = "_ZN3wsp12_GLOBAL__N_111conv_gemm_g"
HUBERT_ARCH = "HuBERT_ECAPA_GLOB_c512"  # C4: HuBERT-base front end + ECAPA_TDNN_GLOB_c512(feat_dim 768)
HEAD_TAGS = ("layer1", "conv1x1_CxC", "res2_k3", "se", "conv_cat", "glob_ctx", "pool_linear1", "pool_linear2",
             "astp", "head", "stem", "shortcut", "res_conv1x1", "res_conv3x3", "res_tail", "tstp_head",
             "simam", "asp_rows", "asp_linear1", "asp_linear2", "asp_pool_head")
HUBERT_TAGS = ("h_conv0", "h_cnn", "h_ln", "h_proj", "h_pos_conv", "h_qkv", "h_attn", "h_out_proj", "h_fc1",
               "h_fc2", "h_cmn")


# workload tag of the profile summaries that may describe this run's kernels
# (profiles/r<N>_<tag>_traffic.json): the same template symbol and grid can occur in
# two workloads (C4's fc1 at B = 256 has conv_cat's C2 grid), so only the run's own
# workload's summaries are searched
PROFILE_TAG = "c2"


def profiled_record(symbol: str, grid: int):
    """PMC record of a kernel launch geometry from the newest committed rocprofv3
    summary of this workload (profiles/r*_<PROFILE_TAG>_traffic.json, made by
    scripts/make_profile_summary.py): HBM bytes per launch, MFMA utilisation
    (SQ_VALU_MFMA_BUSY_CYCLES over the SIMD cycles of GRBM_GUI_ACTIVE) and the
    clock the launch ran at."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{PROFILE_TAG}_traffic.json")),
                   key=lambda f: os.path.basename(f))
    for f in reversed(files):
        d = json.load(open(f))
        for key, v in d.items():
            sym, _, g = key.rpartition("|")
            if sym.startswith(symbol) and g == str(grid) and v.get("hbm_bytes"):
                return v, os.path.basename(f) + ":" + sym
    return None, None


def profiled_traffic(symbol: str, grid: int):
    rec, src = profiled_record(symbol, grid)
    return (rec["hbm_bytes"], src) if rec else (None, None)


def pmc_fields(symbol: str, grid: int) -> dict:
    rec, _ = profiled_record(symbol, grid)
    if not rec or rec.get("mfma_util") is None:
        return {"mfma_util_pmc": None, "clock_ghz_pmc": None}
    return {"mfma_util_pmc": round(rec["mfma_util"], 4),
            "clock_ghz_pmc": round(rec["clock_ghz"], 3) if rec.get("clock_ghz") else None}


def resnet_1x1_bytes_by_stage(arch: str, F: int, T: int, m: int = 32) -> dict:
    """resnet_1x1_bytes_per_utt split by profiling sub-class (res_conv1x1.{c1,c3}.L<n>)."""
    kind, nblocks = RESNET_ARCHS[arch]
    out, cin, fi, ti = {}, m, F, T
    for li, n in enumerate(nblocks):
        p = m << li
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            fo, to = (fi - 1) // s + 1, (ti - 1) // s + 1
            k1, k3 = f"res_conv1x1.c1.L{li + 1}", f"res_conv1x1.c3.L{li + 1}"
            out[k1] = out.get(k1, 0.0) + 4.0 * fi * ti * (cin + p)
            out[k3] = out.get(k3, 0.0) + 4.0 * fo * to * (p + 4 * p + 4 * p)
            cin, fi, ti = 4 * p, fo, to
    return out


def resnet_1x1_launch_geometry(arch: str, F: int, T: int, bc: int, m: int = 32) -> dict:
    """Per 1x1 sub-class: (kernel symbol, grid threads) of its launches at `bc`
    utterances per launch — the tile launch_conv_gemm_x3 picks for N at the ResNet
    default variant 3 (N % 64: 128x32, N % 128: 128x64, else 128x128 swizzled)."""
    kind, nblocks = RESNET_ARCHS[arch]
    out, fi, ti = {}, F, T

    def launch(rows, N):
        if N % 64:
            tmpl, swz, bn = "4ELi1ELi1ELi1", 0, 32
        elif N % 128:
            tmpl, swz, bn = "4ELi1ELi1ELi2", 0, 64
        else:
            tmpl, swz, bn = "2ELi2ELi2ELi2", 1, 128
        sym = f"_ZN3wsp12_GLOBAL__N_112conv_gemm_x3ILi{tmpl}ELi0ELb1ELi0ELb0ELb{swz}E"
        return sym, ((bc * rows + 127) // 128) * (N // bn) * 256

    for li, n in enumerate(nblocks):
        p = m << li
        s = 2 if li > 0 else 1
        fo, to = (fi - 1) // s + 1, (ti - 1) // s + 1
        # (symbol, grid, launches per chunk); a stride-2 first block's conv1 runs at the input resolution
        c1 = [(*launch(fi * ti, p), 1), (*launch(fo * to, p), n - 1)] if s == 2 else [(*launch(fo * to, p), n)]
        out[f"res_conv1x1.c1.L{li + 1}"] = [x for x in c1 if x[2] > 0]
        out[f"res_conv1x1.c3.L{li + 1}"] = [(*launch(fo * to, 4 * p), n)]
        fi, ti = fo, to
    return out


def resnet_1x1_bytes_per_utt(arch: str, F: int, T: int, m: int = 32) -> float:
    """Algorithmic HBM bytes of every 1x1 conv of one ResNet forward (resnet.py:72-107):
    fp32 activations read once (+ the residual read by conv3's epilogue), output written
    once; weights (bf16 hi+lo, L2-resident) excluded."""
    kind, nblocks = RESNET_ARCHS[arch]
    if kind != "bottleneck":
        return 0.0
    total, cin, fi, ti = 0.0, m, F, T
    for li, n in enumerate(nblocks):
        p = m << li
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            fo, to = (fi - 1) // s + 1, (ti - 1) // s + 1
            total += 4.0 * fi * ti * (cin + p)             # conv1: read x, write y1
            total += 4.0 * fo * to * (p + 4 * p + 4 * p)   # conv3: read y2 + residual, write out
            cin, fi, ti = 4 * p, fo, to
    return total


def resnet_tail_launches(arch: str, F: int, T: int, m: int = 32) -> dict:
    """Per stage L<n>: the bottleneck-tail launches of one utterance-chunk forward
    (model_impl.h forward_resnet, option res_tail 1): every stride-1 block with 32 / 64 /
    128 planes runs conv2 + conv3 + residual (+ the next block's conv1 when the next block
    of the stage is a stride-1 block too: tail2_kernel) in one launch.  Returns
    {stage: (positions per utterance, planes, fused launches, unfused launches)}."""
    kind, nblocks = RESNET_ARCHS[arch]
    out, fi, ti = {}, F, T
    for li, n in enumerate(nblocks):
        p = m << li
        s = 2 if li > 0 else 1
        fo, to = (fi - 1) // s + 1, (ti - 1) // s + 1
        if kind == "bottleneck" and p <= 128:
            tails = [bi for bi in range(n) if not (li > 0 and bi == 0)]
            fused = sum(1 for bi in tails if bi + 1 < n)
            out[f"L{li + 1}"] = (fo * to, p, fused, len(tails) - fused)
        fi, ti = fo, to
    return out


def resnet_model_bytes_per_utt(arch: str, F: int, T: int, m: int = 32) -> float:
    """Algorithmic HBM bytes of one whole bottleneck-ResNet forward (resnet.py:110-260):
    every conv's fp32 input read once and output written once (the stem, the 1x1
    convs with conv3's residual read, the 3x3 convs, the projection shortcuts), plus
    the pooling read of the last activations; weights excluded."""
    kind, nblocks = RESNET_ARCHS[arch]
    if kind != "bottleneck":
        return 0.0
    total = 4.0 * F * T * (1 + m)  # stem 3x3: 1 -> m channels
    cin, fi, ti = m, F, T
    for li, n in enumerate(nblocks):
        p = m << li
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            fo, to = (fi - 1) // s + 1, (ti - 1) // s + 1
            total += 4.0 * fi * ti * (cin + p)             # conv1
            total += 4.0 * (fi * ti * p + fo * to * p)     # conv2 (3x3, stride s)
            total += 4.0 * fo * to * (p + 4 * p + 4 * p)   # conv3 + residual
            if s != 1 or cin != 4 * p:
                total += 4.0 * fo * to * (cin + 4 * p)     # projection shortcut
            cin, fi, ti = 4 * p, fo, to
    return total + 4.0 * fi * ti * cin                     # statistics pooling read


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="per GPU (default 256 ECAPA and HuBERT + ECAPA, 128 ResNet)")
    ap.add_argument("--arch", default="ECAPA_TDNN_c1024",
                    help=f"ECAPA_TDNN_*, ResNet*, or {HUBERT_ARCH} (wav -> HuBERT -> CMN -> ECAPA)")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--precision", type=int, default=1, help="1 = bf16x3 split MFMA, 0 = f32 MFMA")
    ap.add_argument("--x3-variant", type=int, default=None)
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="extra model option (wsp_model_set_option), e.g. res2_variant=1; repeatable")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-kernel event timing pass")
    ap.add_argument("--no-f32", action="store_true", help="skip the exact-f32 (precision 0) side measurement")
    ap.add_argument("--no-kernel-roofline", action="store_true",
                    help="skip the streams=1 side pass behind the C3 / C4 dominant-kernel roofline")
    ap.add_argument("--no-hubert-b64", dest="hubert_small_batch", action="store_false",
                    help="skip the C4 side measurement at the survey's per-rank batch 64")
    ap.add_argument("--sustain-seconds", type=float, default=2.0,
                    help="extra untimed-for-value window reported as value_sustained (>= this many seconds)")
    ap.add_argument("--configs", default="C3,C4,C5",
                    help="sub-configurations timed after the C2 headline (C3 = ResNet293 B=128, C4 = HuBERT-base + "
                         "ECAPA_TDNN_GLOB_c512 B=256, C5 = the vox1-O-shaped extract + score + AS-Norm pipeline "
                         "through the product's file path), comma-separated, or 'none'")
    ap.add_argument("--sub-steps", type=int, default=10)
    ap.add_argument("--sub-warmup", type=int, default=2)
    ap.add_argument("--sub-cpu-seconds", type=float, default=10.0)
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU/gloo rehearsal of the rank launch, barriers and JSON (no GPU work; tests only)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(gpus: int) -> int:
    """One process per GPU, as the driver's own torchrun line does (and as
    tools/extract_embedding.sh:40-63 starts one extractor per GPU): a child
    torchrun, started before any GPU call in this process; rank 0 prints the
    JSON line, which reaches our stdout directly."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ))


def plumbing_main(args):
    """--plumbing: the multi-rank skeleton of main() on CPU (gloo) with a
    sleep as the step, so tests can check the launch / max-over-ranks / JSON
    contract without a GPU."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if world > 1:
        dist.init_process_group("gloo")
    B = args.batch or 256
    for _ in range(args.warmup):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.002 * (1 + rank))
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    check = rccl_check(torch.device("cpu"), world, rank) if world > 1 else None
    if rank == 0:
        print(json.dumps({"metric": "embeddings/sec on 5s 16kHz utts (plumbing rehearsal, no GPU work)",
                          "rccl_allreduce_check": check,
                          "value": round(world * B * args.steps / el, 2), "unit": "emb/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "scaling": "weak",
                          "config": {"batch_per_gpu": B, "global_batch": B * world,
                                     "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rccl_check(dev, world: int, rank: int) -> dict:
    """Runs wespeaker_hubert_amd.dist.allreduce_sums on device buffers (rank r adds
    r + 1 to a [G, D] sum and its counts) and compares with the closed form (at world 1
    too: the collective is forced, tests/test_gpu_rccl.py)."""
    import torch.distributed as tdist
    from wespeaker_hubert_amd.dist import allreduce_sums
    G, D = 1000, 192
    acc = torch.full((G, D), float(rank + 1), dtype=torch.float64, device=dev)
    cnt = torch.full((G,), float(rank + 1), dtype=torch.float64, device=dev)
    t = time.perf_counter()
    allreduce_sums(acc, cnt, force=True)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t) * 1e3
    want = world * (world + 1) / 2
    ok = torch.tensor([float(bool((acc == want).all()) and bool((cnt == want).all()))], device=dev)
    tdist.all_reduce(ok, op=tdist.ReduceOp.MIN)
    return {"backend": tdist.get_backend(), "world": world, "elements": G * D + G,
            "ok": bool(ok.item() == 1.0), "ms_rank0": round(ms, 3)}


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the CPUs this process may actually use
    (BASELINE.md §3 asks for os.cpu_count(); on the GPU box os.cpu_count() and the
    affinity mask report the whole host (256) while the cgroup quota
    (/sys/fs/cgroup/cpu.max) grants 16 CPUs -- 256 threads on 16 CPUs ran the
    oracle 200x slower, so the quota caps the count)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(arch: str, sd, num_samples: int, budget_s: float, batch: int = 8):
    """Oracle ('port') pipeline timed on the host cores: numpy float64 fbank +
    CMN, then the fp32 PyTorch-CPU restatement of the reference forward (ECAPA /
    ResNet).  Bounded sample: batches of `batch` utterances until >= budget_s of work."""
    from oracle import fbank_ref, models_ref
    threads = cpu_threads()
    torch.set_num_threads(threads)
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}

    def run(n, seed):
        wav = synth_audio(seed, n, num_samples)
        feats = np.stack([fbank_ref.fbank(w, cmn=True) for w in wav])
        with torch.no_grad():
            models_ref.forward(arch, torch.from_numpy(feats), sdt)

    run(min(2, batch), 1000)  # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        run(batch, 1001 + done)
        done += batch
        el = time.perf_counter() - t0
        if el >= budget_s or done >= 256:
            break
    return {"value": done / el, "unit": "emb/s", "cores": threads, "kind": "port", "os_cpu_count": os.cpu_count(),
            "sample": f"{done} synthetic {num_samples / 16000:.0f}s utts, batches of {batch}, "
                      f"numpy-f64 fbank + torch-CPU fp32 {arch} (oracle restatement), {el:.1f}s"}


def cpu_baseline_hubert(sd_fe, sd, num_samples: int, budget_s: float):
    """Oracle ('port') C4 chain on the host cores: fp32 torch-CPU HuBERT-base +
    s3prl glue + CMN + ECAPA_TDNN_GLOB_c512.  Bounded sample: batches of 2."""
    from oracle import hubert_ref, models_ref
    threads = cpu_threads()
    torch.set_num_threads(threads)
    sdf = {k: torch.from_numpy(v) for k, v in sd_fe.items()}
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}

    def run(n, seed):
        wav = torch.from_numpy(synth_audio(seed, n, num_samples, int16_scale=False))
        with torch.no_grad():
            f = hubert_ref.s3prl_frontend(wav, sdf)
            models_ref.forward("ECAPA_TDNN_GLOB_c512", f - f.mean(dim=1, keepdim=True), sdt)

    run(1, 1000)  # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        run(2, 1001 + done)
        done += 2
        el = time.perf_counter() - t0
        if el >= budget_s or done >= 64:
            break
    return {"value": done / el, "unit": "emb/s", "cores": threads, "kind": "port", "os_cpu_count": os.cpu_count(),
            "sample": f"{done} synthetic {num_samples / 16000:.0f}s utts, batches of 2, torch-CPU fp32 "
                      f"HuBERT-base + s3prl glue + CMN + ECAPA_TDNN_GLOB_c512 (oracle restatement), {el:.1f}s"}


# Sub-configurations reported beside the headline (BASELINE.json configs[2] and [3]):
# name -> (arch, per-GPU batch).  C4's per-GPU batch is 256 like C2 (SURVEY §8(d) quotes
# 64: with 64 utterances fc2 / out_proj fill 189 of the 256 CUs, with 256 they fill 2.9
# rounds, +12.5 % -- DESIGN.md §5)
SUB_CONFIGS = {"C3": ("ResNet293", 128), "C4": (HUBERT_ARCH, 256)}


def build_workload(args, arch: str, B: int, rank: int, dev):
    """Model(s), synthetic HBM-resident inputs and the step closure of one workload."""
    hubert = arch == HUBERT_ARCH
    simam = arch.startswith("SimAM")
    resnet_like = arch.startswith("ResNet") or simam
    N = int(round(args.seconds * 16000))
    emb_dim = 256 if resnet_like else 192
    head_arch = "ECAPA_TDNN_GLOB_c512" if hubert else arch
    feat_dim = 768 if hubert else 80
    margs = dict(acoustic_dim=feat_dim, embed_dim=emb_dim) if simam else dict(feat_dim=feat_dim, embed_dim=emb_dim)
    spec = make_spec(head_arch, **margs)
    model = HipSpeakerModel(head_arch, **margs)
    sd = synth_state_dict(1234, model.state_dict_layout(), residual_tame=resnet_like)
    model.load_state_dict(sd)
    fe, sd_fe = None, None
    if hubert:
        fe = S3prlFrontend({"name": "hubert_base"})
        sd_fe = synth_state_dict(1235, fe.state_dict_layout())
        fe.load_state_dict(sd_fe)
    for mm in (model, fe):
        if mm is None:
            continue
        mm.set_option("precision", args.precision)
        if args.x3_variant is not None:
            mm.set_option("x3_variant", args.x3_variant)
        for kv in args.opt:
            k, _, v = kv.partition("=")
            mm.set_option(k, int(v))
        mm.to(dev)
    # inputs resident in HBM before the timed region (per-rank shard)
    wav = torch.from_numpy(synth_audio(7 + rank, B, N, int16_scale=not hubert)).to(dev)
    T = (N + 319) // 320 if hubert else 1 + (N - 400) // 160
    feats = torch.empty(B, T, feat_dim, device=dev)
    emb = torch.empty(B, emb_dim, device=dev)

    def step():
        if hubert:
            fe.extract(wav, cmn=True, out=feats)
        else:
            compute_fbank(wav, scale=1.0, cmn=True, out=feats)
        model.embed(feats, out=emb)

    return dict(arch=arch, head_arch=head_arch, hubert=hubert, simam=simam, resnet_like=resnet_like, B=B, N=N, T=T,
                spec=spec, model=model, fe=fe, sd=sd, sd_fe=sd_fe, step=step, wav=wav, feats=feats, emb=emb)


def kernel_table(w, steps: int) -> dict:
    """Per kernel class: launches, average launch time (HIP events on the launch
    stream, wsp_model_profile), time per step and the class's algorithmic rate."""
    kernels = {}
    queries = [(w["model"], t) for t in HEAD_TAGS] + ([(w["fe"], t) for t in HUBERT_TAGS] if w["fe"] else [])
    if w["fe"]:
        queries += [(w["fe"], f"h_cnn.c{i}") for i in range(1, 7)]  # per-layer sub-classes of h_cnn
    for mm, tag in queries:
        n, ms, fl = mm.profile_query(tag)
        if n:
            avg = ms / n
            kernels[tag] = {"launches_per_step": n // steps, "avg_ms": round(avg, 4),
                            "ms_per_step": round(ms / steps, 4),
                            "tflops": round(fl / (avg * 1e-3) / 1e12, 2) if fl else None,
                            "flops_per_launch": fl or None}
    return kernels


def dominant_class(kernels: dict, streams: int) -> dict:
    """The kernel class with the most launch time per step (a top-level class, not a
    per-stage sub-class); with concurrent streams the summed launch times of both
    utterance ranges are compared (they overlap in wall time)."""
    top = {k: v for k, v in kernels.items() if "." not in k}
    if not top:
        return None
    name = max(top, key=lambda k: top[k]["ms_per_step"])
    d = {"class": name, **top[name]}
    if d.get("tflops"):
        d["frac_of_bf16_peak"] = round(d["tflops"] / BF16_MFMA_PEAK_TFLOPS, 4)
        d["frac_of_issue_peak"] = round(3 * d["tflops"] / BF16_MFMA_PEAK_TFLOPS, 4)
    if streams > 1:
        d["note"] = (f"launch times summed over {streams} concurrent utterance-range streams; "
                     "per-launch rates are measured while the other range's kernels share the GPU")
    return d


def roofline_ecapa(args, w, k, streams):
    """Per-kernel MFMA roofline of the SE-Res2Block 1x1 CxC conv (the headline's dominant kernel)."""
    C = 1024 if "c1024" in w["arch"] else 512
    M = w["B"] * w["T"] // streams   # rows per launch (one utterance range)
    flops = 2.0 * M * C * C          # algorithmic: 2*M*N*K, M = B*T frames
    ach = flops / (k["avg_ms"] * 1e-3) / 1e12
    x3 = args.precision == 1
    peak = BF16_MFMA_PEAK_TFLOPS if x3 else FP32_MFMA_PEAK_TFLOPS
    sym, bm, bn, nt = dominant_symbol(args.precision, w["model"].get_option("x3_variant"), C, C, 1,
                                      se_fused=w["T"] >= 256)
    grid = ((M + bm - 1) // bm) * (C // bn) * nt
    traffic, src = profiled_traffic(sym, grid)
    algo_bytes = 4.0 * M * C * 2 + (2 if x3 else 4) * C * C * (2 if x3 else 1)
    return {"kernel": sym, "bound": "mfma", "achieved": round(ach, 2), "peak": peak,
            "unit": "TFLOP/s", "frac": round(ach / peak, 4),
            "traffic": traffic, "traffic_source": src, "algorithmic_bytes": algo_bytes,
            "flops_per_launch": flops, "avg_launch_ms": k["avg_ms"],
            "mfma_dtype": "bf16 (3-term split, fp32 accumulate)" if x3 else "f32",
            "mfma_work_factor": 3 if x3 else 1,
            "frac_of_issue_peak": round(ach * (3 if x3 else 1) / peak, 4), **pmc_fields(sym, grid),
            "concurrent_streams": streams}


def roofline_resnet_model(args, w, kernels, el, steps, streams):
    """C3: whole-model HBM roofline -- every conv's algorithmic fp32 bytes of a step
    (resnet_model_bytes_per_utt x B) over the measured step time, independent of how
    launches overlap; the 1x1-conv class figure (summed launch time) beside it."""
    arch, B, T, model = w["arch"], w["B"], w["T"], w["model"]
    mb = resnet_model_bytes_per_utt(arch, 80, T) * B
    ms_step = el / steps * 1e3
    ach = mb / (ms_step * 1e-3) / 1e9
    roof = {"kernel": "whole ResNet forward (fbank + stem + every conv + TSTP), algorithmic bytes / step time",
            "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4), "algorithmic_bytes_per_step": mb, "ms_per_step": round(ms_step, 3),
            "traffic": None,
            "bytes_note": "fp32 activations: each conv's input read once, output written once, the bottleneck "
                          "conv3's residual read once, the pooling read; weights excluded (L2-resident)"}
    kr = kernels.get("res_conv1x1")
    if not kr:
        return roof
    bc = B // -(-B // 64) if B > 64 else B  # the model's 2-GiB chunking at T = 498
    geo = resnet_1x1_launch_geometry(arch, 80, T, bc)
    traffic_step, srcs, byts = 0.0, set(), 0.0
    chunks = -(-B // bc)
    for tag, bpu in resnet_1x1_bytes_by_stage(arch, 80, T).items():
        n, ms, _ = model.profile_query(tag)
        if not n:
            continue
        # with res_tail the stride-1 blocks' conv3 runs inside bottleneck_tail: only the
        # stride-2 first blocks' conv3 launches remain (same output shape as the others)
        expected = chunks * sum(c for _, _, c in geo[tag])
        bts = bpu * B * (n // steps) / expected
        byts += bts
        kernels[tag] = {"launches_per_step": n // steps, "avg_ms": round(ms / n, 4),
                        "ms_per_step": round(ms / steps, 4),
                        "gbps": round(bts / (ms / steps * 1e-3) / 1e9, 1)}
        if traffic_step is not None:
            if n // steps != expected:
                traffic_step = None  # PMC summaries are per launch geometry of the unfused schedule
                continue
            for sym, grid, cnt in geo[tag]:
                tb, src = profiled_traffic(sym, grid)
                if tb is None:
                    traffic_step = None
                    break
                traffic_step += tb * cnt * chunks
                srcs.add(src.split(":")[0])
    for cls in ("res_conv3x3", "res_tail"):
        for li in range(1, 5):
            n, ms, fl = model.profile_query(f"{cls}.L{li}")
            if n:
                kernels[f"{cls}.L{li}"] = {"launches_per_step": n // steps, "avg_ms": round(ms / n, 4),
                                           "ms_per_step": round(ms / steps, 4),
                                           "tflops": round(fl / (ms / n * 1e-3) / 1e12, 2)}
    a1 = byts / (kr["ms_per_step"] * 1e-3) / 1e9
    roof["class_1x1"] = {"kernel": "conv_gemm_x3 ResNet 1x1 convs (res_conv1x1, all launches of a step)",
                         "achieved": round(a1, 1), "frac": round(a1 / HBM_PEAK_GBPS, 4),
                         "algorithmic_bytes": byts, "launches_per_step": kr["launches_per_step"],
                         "ms_per_step": kr["ms_per_step"], "traffic": traffic_step or None,
                         "traffic_source": ",".join(sorted(srcs)) or None,
                         "traffic_note": "PMC HBM bytes of all 1x1 launches of a step (FETCH_SIZE x2 + WRITE_SIZE)"}
    if streams > 1:
        roof["class_1x1"]["note"] = ("launch durations measured beside the other utterance range's kernels "
                                     "(option streams); --opt streams=1 gives the standalone rate")
    return roof


def standalone_pass(w, handle, tags, steps: int = 2) -> dict:
    """Per-launch durations of `tags` with the workload on ONE stream (option streams = 1):
    with the default two utterance-range streams a launch shares the GPU with the other
    range's kernels, so its event-timed duration is not the kernel's own.  Untimed for
    `value`; the handle's streams option is restored afterwards."""
    old = handle.get_option("streams")
    handle.set_option("streams", 1)
    try:
        w["step"]()
        torch.cuda.synchronize()
        handle.profile(True)
        for _ in range(steps):
            w["step"]()
        torch.cuda.synchronize()
        handle.profile(False)
        out = {}
        for t in tags:
            n, ms, fl = handle.profile_query(t)
            if n:
                out[t] = {"launches_per_step": n // steps, "avg_ms": ms / n, "flops_per_launch": fl}
        return out
    finally:
        handle.set_option("streams", old)


def kernel_roofline_record(name: str, cls: str, launches: int, avg_ms: float, algo_bytes: float, flops: float,
                           pmc: dict | None, pmc_src: str | None, pmc_algo_bytes: float | None, bound: str) -> dict:
    """Roofline of ONE kernel from its standalone launch duration: algorithmic bytes and
    FLOP per launch, fraction of the HBM peak and of the bf16 MFMA peak counted as issued
    bf16x3 work (3 bf16 MFMAs per fp32 product); PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE,
    scripts/make_profile_summary.py) of the same kernel's launch in the newest committed
    profile, with its own algorithmic bytes for the ratio."""
    gbps = algo_bytes / (avg_ms * 1e-3) / 1e9
    tf = flops / (avg_ms * 1e-3) / 1e12
    rec = {"kernel": name, "class": cls, "bound": bound, "launches_per_step": launches,
           "standalone_avg_ms": round(avg_ms, 4),
           "algorithmic_bytes_per_launch": algo_bytes, "flops_per_launch": flops,
           "achieved_gbps": round(gbps, 1), "frac_hbm": round(gbps / HBM_PEAK_GBPS, 4),
           "achieved_tflops": round(tf, 2), "frac_bf16_peak": round(tf / BF16_MFMA_PEAK_TFLOPS, 4),
           "frac_issue_peak": round(3 * tf / BF16_MFMA_PEAK_TFLOPS, 4),
           "traffic": None, "traffic_ratio": None, "traffic_source": pmc_src,
           "pmc_dur_ms": None, "mfma_util_pmc": None, "clock_ghz_pmc": None}
    rec["frac"] = rec["frac_hbm"] if bound == "hbm" else rec["frac_issue_peak"]
    if pmc:
        ratio = pmc["hbm_bytes"] / pmc_algo_bytes if pmc_algo_bytes else None
        rec.update({"traffic": round(ratio * algo_bytes) if ratio else pmc["hbm_bytes"],
                    "traffic_ratio": round(ratio, 4) if ratio else None,
                    "pmc_dur_ms": round(pmc["pmc_dur_ns"] * 1e-6, 4) if pmc.get("pmc_dur_ns") else None,
                    "mfma_util_pmc": round(pmc["mfma_util"], 4) if pmc.get("mfma_util") is not None else None,
                    "clock_ghz_pmc": round(pmc["clock_ghz"], 3) if pmc.get("clock_ghz") else None})
    return rec


def pmc_lookup(pred):
    """Newest committed PMC record (profiles/r*_<PROFILE_TAG>_traffic.json) whose
    (symbol, grid) satisfies pred; returns (record, source, grid)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{PROFILE_TAG}_traffic.json")),
                   key=lambda f: os.path.basename(f))
    for f in reversed(files):
        d = json.load(open(f))
        for key, v in d.items():
            sym, _, g = key.rpartition("|")
            if v.get("hbm_bytes") and pred(sym, int(g)):
                return v, os.path.basename(f) + ":" + sym, int(g)
    return None, None, None


def kernel_roofline_resnet(w) -> dict:
    """C3: the dominant kernel, the stage-3 bottleneck tail + next conv1 (tail2_kernel<128>,
    resnet.py:72-107; 126 launches per B = 128 step), from a streams = 1 side pass.  Bytes per
    position: y1 (p) + residual (4p) + out (4p) + the next block's y1 (p) fp32 values; FLOP per
    position 2 (9p.p + 4p.p + 4p.p)."""
    arch, B, T, model = w["arch"], w["B"], w["T"], w["model"]
    tails = resnet_tail_launches(arch, 80, T)
    if "L3" not in tails:
        return None
    sa = standalone_pass(w, model, ["res_tail.L3"])
    if "res_tail.L3" not in sa:
        return None
    pos, p, nf, nu = tails["L3"]
    bc = B // -(-B // 64) if B > 64 else B  # the model's 2-GiB utterance chunking at T = 498
    # class time = fused + unfused launches; bytes / flops summed the same way
    cls_bytes = 4.0 * pos * bc * (nf * 10 * p + nu * 9 * p)
    cls_launch = nf + nu
    k = sa["res_tail.L3"]
    launches = k["launches_per_step"]
    avg_bytes = cls_bytes / cls_launch
    fused_bytes = 4.0 * pos * bc * 10 * p
    fused_flops = 2.0 * pos * bc * (9 * p * p + 4 * p * p + 4 * p * p)
    f3, t3 = 80, T
    for _ in range(2):  # the stride-2 first blocks of stages 2 and 3
        f3, t3 = (f3 - 1) // 2 + 1, (t3 - 1) // 2 + 1
    grid = bc * (-(-f3 // 2)) * (-(-t3 // 32)) * 256  # tail2<128>: 2 x 32 positions, 256 threads per block
    pmc, src, _ = pmc_lookup(lambda s, g: "tail2_kernel<128," in s and g == grid)
    rec = kernel_roofline_record("tail2_kernel<128, 8, 4, 4> (conv3x3_img.hip: conv2 + conv3 + residual + next conv1)",
                                 "res_tail.L3", launches, k["avg_ms"], avg_bytes, k["flops_per_launch"], pmc, src,
                                 fused_bytes, "hbm")
    rec["note"] = (f"class res_tail.L3 = {nf} fused tail2 + {nu} unfused bottleneck_tail launch(es) per "
                   f"{bc}-utterance chunk; standalone = option streams 1 side pass; traffic_ratio from the PMC-"
                   f"serialised tail2<128> launch (grid {grid}) against its {fused_bytes / 1e6:.0f} MB algorithmic")
    return rec


def kernel_roofline_hubert(w) -> dict:
    """C4: the dominant kernel, HuBERT's first strided CNN GEMM (h_cnn.c1: conv k3 s2,
    512 -> 512, GELU; fairseq ConvFeatureExtractionModel layer 1 under s3prl.py:80-93), from a
    streams = 1 side pass.  FLOP per output frame 2 . 512 . 1536; bytes: the conv0 output read
    once + the output written once (fp32)."""
    fe = w["fe"]
    sa = standalone_pass(w, fe, ["h_cnn.c1"])
    if "h_cnn.c1" not in sa:
        return None
    k = sa["h_cnn.c1"]
    N = w["N"]
    t0 = (N - 10) // 5 + 1
    t1 = (t0 - 3) // 2 + 1
    flops = k["flops_per_launch"]
    utts = flops / (2.0 * t1 * 512 * 1536)  # utterances per launch (the feature extractor's chunk)
    algo = 4.0 * 512 * (t0 + t1) * utts

    def is_c1(s, g):  # the 16x16x32 256 x 256 GELU tile at a grid of whole 7 999-row utterances
        if ("conv_gemm_x3ILi4ELi2ELi2ELi4ELi0ELb1ELi0ELb0ELb1ELi1ELi16E" not in s
                and not s.startswith(G_SYMBOL + "ILi0ELb0E")):  # conv_gemm_g<0, false>
            return False
        blocks = g // 512 // 2
        nb = round(blocks * 256 / t1)
        return nb > 0 and -(-nb * t1 // 256) == blocks
    pmc, src, grid = pmc_lookup(is_c1)
    pmc_algo = None
    if pmc:
        nb = round(grid // 1024 * 256 / t1)
        pmc_algo = 4.0 * 512 * (t0 + t1) * nb
    fam7 = fe.get_option("x3_variant") == 7
    name = ("conv_gemm_g<0, false> (family 7: 256 x 256 tile, operands by LDS-DMA, bf16x3 on 16x16x32 MFMAs), "
            "h_cnn.c1" if fam7 else "conv_gemm_x3<4,2,2,4,...,MF=16> (256 x 256 tile, bf16x3 on 16x16x32 MFMAs), h_cnn.c1")
    rec = kernel_roofline_record(name,
                                 "h_cnn.c1", k["launches_per_step"], k["avg_ms"], algo, flops, pmc, src, pmc_algo, "mfma")
    rec["note"] = (f"{utts:.0f} utterances per launch (feature-extractor chunk); standalone = option streams 1 "
                   "side pass; frac = issued bf16x3 MFMA work over the dense bf16 peak")
    return rec


def roofline_model_mfma(args, w, gf_utt, el, steps):
    """C4: model-level MFMA roofline -- the whole chain's algorithmic FLOP per step
    (HuBERT-base + ECAPA head, 2 x MACs) over the measured step time, against the dense
    bf16 peak; the issued fraction (3 bf16 MFMAs per fp32 product) beside it."""
    B = w["B"]
    flops = gf_utt * 1e9 * B
    ms_step = el / steps * 1e3
    ach = flops / (ms_step * 1e-3) / 1e12
    x3 = args.precision == 1
    peak = BF16_MFMA_PEAK_TFLOPS if x3 else FP32_MFMA_PEAK_TFLOPS
    return {"kernel": "whole HuBERT-base + CMN + ECAPA_TDNN_GLOB_c512 chain, algorithmic FLOP / step time",
            "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "algorithmic_flops_per_step": flops, "ms_per_step": round(ms_step, 3),
            "mfma_dtype": "bf16 (3-term split, fp32 accumulate)" if x3 else "f32",
            "mfma_work_factor": 3 if x3 else 1, "frac_of_issue_peak": round(ach * (3 if x3 else 1) / peak, 4),
            "traffic": None}


def roofline_simam(args, k3):
    ach = k3["tflops"] or 0.0
    x3 = args.precision == 1
    return {"kernel": "conv_gemm_x3 SimAM-ResNet 3x3 convs (res_conv3x3, all launches of a step)",
            "bound": "mfma", "achieved": ach, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4), "traffic": None, "traffic_source": None,
            "launches_per_step": k3["launches_per_step"], "ms_per_step": k3["ms_per_step"],
            "mfma_dtype": "bf16 (3-term split, fp32 accumulate)", "mfma_work_factor": 3 if x3 else 1,
            "frac_of_issue_peak": round(ach * 3 / BF16_MFMA_PEAK_TFLOPS, 4)}


def gflop_per_utt(w) -> float:
    arch, spec, T, N = w["arch"], w["spec"], w["T"], w["N"]
    if w["hubert"]:
        return hubert_gflop_per_utt(N) + ecapa_gflop_per_utt(spec, T)
    if arch.startswith("ECAPA"):
        return ecapa_gflop_per_utt(spec, T)
    if w["simam"]:
        return simam_gflop_per_utt(spec, T)
    return resnet_gflop_per_utt(spec, T)


def run_workload(args, arch: str, B: int, steps: int, warmup: int, world: int, rank: int, dev, dist,
                 headline: bool, cpu_seconds: float) -> dict:
    """One workload: W untimed warm-up steps, then K steps timed between barrier +
    synchronize, max over ranks; per-kernel-class HIP events inside the timed region."""
    w = build_workload(args, arch, B, rank, dev)
    model, fe, step = w["model"], w["fe"], w["step"]

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(e):
        if dist is not None:
            t = torch.tensor([e], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e = float(t.item())
        return e

    for _ in range(warmup):
        step()
    barrier()
    # Per-kernel-class HIP events are recorded on the launch stream around
    # every launch inside the timed region (wsp_model_profile); they feed the
    # roofline figure below.
    if not args.no_profile:
        for mm in (model, fe):
            if mm is not None:
                mm.profile(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    el = time.perf_counter() - t0
    if not args.no_profile:
        for mm in (model, fe):
            if mm is not None:
                mm.profile(False)
    el = max_over_ranks(el)
    value = world * B * steps / el

    def timed(n):
        barrier()
        t = time.perf_counter()
        for _ in range(n):
            step()
        barrier()
        return max_over_ranks(time.perf_counter() - t)

    sustained = exact = None
    if headline and args.sustain_seconds > 0:
        # >= --sustain-seconds of back-to-back steps, profiling off: the same step
        # count on every rank, derived from the max-over-ranks time
        n_s = max(steps, int(np.ceil(args.sustain_seconds / (el / steps))))
        e_s = timed(n_s)
        sustained = {"value": round(world * B * n_s / e_s, 2), "steps": n_s, "seconds": round(e_s, 3),
                     "ms_per_step": round(e_s / n_s * 1e3, 3)}
    if headline and args.precision == 1 and not args.no_f32 and not arch.startswith(("ResNet", "SimAM")):
        # exact-f32 MFMA (precision 0) beside the bf16x3 headline (ECAPA-TDNN / HuBERT: the ResNet
        # families run on the bf16x3 kernels only)
        for mm in (model, fe):
            if mm is not None:
                mm.set_option("precision", 0)
                mm.to(dev)
        step()
        n_f = max(2, steps // 4)
        e_f = timed(n_f)
        exact = {"value": round(world * B * n_f / e_f, 2), "steps": n_f,
                 "ms_per_step": round(e_f / n_f * 1e3, 3), "dtype": "f32 (v_mfma_f32_32x32x2_f32)"}

    # concurrent sub-batch streams in effect (model option "streams"; front end for C4):
    # with more than one, per-launch durations are measured while another range's
    # kernels share the GPU, so per-kernel roofline fractions read low
    streams = max(m.get_option("streams") for m in (model, fe) if m is not None)
    gf = gflop_per_utt(w)
    kernels, roof = {}, None
    if not args.no_profile:
        kernels = kernel_table(w, steps)
        if w["hubert"]:
            roof = roofline_model_mfma(args, w, gf, el, steps)
        elif arch.startswith("ResNet"):
            roof = roofline_resnet_model(args, w, kernels, el, steps, streams)
        elif w["simam"] and kernels.get("res_conv3x3"):
            roof = roofline_simam(args, kernels["res_conv3x3"])
        elif kernels.get("conv1x1_CxC"):
            roof = roofline_ecapa(args, w, kernels["conv1x1_CxC"], streams)
        if roof is not None and streams > 1 and "note" not in roof and not w["resnet_like"] and not w["hubert"]:
            roof["note"] = ("launch durations measured beside the other utterance range's kernels "
                            "(option streams); --opt streams=1 gives the standalone rate")
    # the dominant kernel's own roofline (standalone launch duration, one stream), untimed
    kroof = None
    if not args.no_profile and not args.no_kernel_roofline:
        if arch.startswith("ResNet"):
            kroof = kernel_roofline_resnet(w)
        elif w["hubert"]:
            kroof = kernel_roofline_hubert(w)
    # C4 at the per-rank batch SURVEY §8(d) / BASELINE.md §3 quote (64), beside the default 256:
    # the same model, the first 64 utterances of the batch, timed the same way
    small = None
    if w["hubert"] and B > 64 and args.hubert_small_batch:
        bs = 64
        fe_, model_ = w["fe"], w["model"]
        wav_s, feats_s, emb_s = w["wav"][:bs], w["feats"][:bs], w["emb"][:bs]

        def step_s():
            fe_.extract(wav_s, cmn=True, out=feats_s)
            model_.embed(feats_s, out=emb_s)
        for _ in range(warmup):
            step_s()
        barrier()
        t = time.perf_counter()
        for _ in range(steps):
            step_s()
        barrier()
        e_s = max_over_ranks(time.perf_counter() - t)
        small = {"batch_per_gpu": bs, "value": round(world * bs * steps / e_s, 2),
                 "ms_per_step": round(e_s / steps * 1e3, 3), "steps": steps}
    res = {
        "value": round(value, 2),
        "ms_per_step": round(el / steps * 1e3, 3),
        "steps": steps,
        "warmup": warmup,
        "workload": (f"HuBERT-base (s3prl featurizer) + CMN + ECAPA_TDNN_GLOB_c512 extract, "
                     f"{args.seconds:g}s 16kHz utts" if w["hubert"] else
                     f"{arch} fbank80 extract, {args.seconds:g}s 16kHz utts"),
        "arch": arch, "batch_per_gpu": B, "global_batch": B * world,
        "samples_per_utt": w["N"], "frames": w["T"], "streams": streams,
        "model_tflops": round(value * gf / 1e3, 2),
        "gflop_per_utt": round(gf, 3),
        "roofline": roof,
        "kernel_roofline": kroof,
        "value_batch64": small,
        "dominant_class": dominant_class(kernels, streams) if kernels else None,
        "kernels": kernels,
        "value_sustained": sustained,
        "value_exact_f32": exact,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = (cpu_baseline_hubert(w["sd_fe"], w["sd"], w["N"], cpu_seconds) if w["hubert"] else
                               cpu_baseline(arch, w["sd"], w["N"], cpu_seconds,
                                            batch=2 if w["resnet_like"] else 8))
    # free the workload's device buffers before the next one
    for key in ("model", "fe"):
        if w[key] is not None:
            w[key]._release()
    del w
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.plumbing:
        return plumbing_main(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    arch = args.arch
    hubert = arch == HUBERT_ARCH
    resnet_like = arch.startswith("ResNet") or arch.startswith("SimAM")
    global PROFILE_TAG
    PROFILE_TAG = {"ECAPA_TDNN_c1024": "c2", "ResNet293": "c3", HUBERT_ARCH: "c4"}.get(arch, "none")
    B = args.batch or (128 if resnet_like else 256)
    r = run_workload(args, arch, B, args.steps, args.warmup, world, rank, dev, dist, headline=True,
                     cpu_seconds=args.cpu_seconds)
    res = {
        "metric": "embeddings/sec on 5s 16kHz utts",
        "value": r["value"],
        "unit": "emb/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (bf16x3 split MFMA, fp32 accumulate)" if args.precision == 1 else "f32",
        "value_sustained": r["value_sustained"],
        "value_exact_f32": r["value_exact_f32"],
        "data": ("synthetic (clip(N(0,0.1)) [-1,1] audio, seeded random-init weights)" if hubert else
                 "synthetic (clip(N(0,0.1)) x32768 PCM16-valued audio, seeded random-init weights)"),
        "config": {"workload": r["workload"], "arch": arch, "batch_per_gpu": B, "global_batch": B * world,
                   "samples_per_utt": r["samples_per_utt"], "frames": r["frames"], "parallelism": f"dp{world}",
                   "streams": r["streams"]},
        "model_tflops": r["model_tflops"],
        "gflop_per_utt": r["gflop_per_utt"],
        "roofline": r["roofline"],
        "kernel_roofline": r["kernel_roofline"],
        "value_batch64": r["value_batch64"],
        "dominant_class": r["dominant_class"],
        "options": args.opt or None,
        "kernels": r["kernels"],
        "cpu_baseline": r["cpu_baseline"],
    }
    # the other single-GPU-per-rank configurations of BASELINE.json (C3 ResNet293,
    # C4 HuBERT + ECAPA), each timed the same way (own warm-up, barrier-bracketed
    # steps, max over ranks), with its own roofline and CPU baseline
    subs = [s for s in args.configs.split(",") if s and s != "none"] if arch == "ECAPA_TDNN_c1024" else []
    if subs:
        res["configs"] = {}
        for name in subs:
            if name == "C5":
                # BASELINE.json configs[4]: end-to-end seconds by stage (scripts/bench_c5.py)
                sys.path.insert(0, os.path.join(REPO, "scripts"))
                import bench_c5
                res["configs"][name] = bench_c5.run_c5("ECAPA_TDNN_c1024", dev, world, rank, dist)
                continue
            if name not in SUB_CONFIGS:
                raise SystemExit(f"bench.py: unknown --configs entry {name} (known: {sorted(SUB_CONFIGS)})")
            sarch, sb = SUB_CONFIGS[name]
            PROFILE_TAG = name.lower()
            res["configs"][name] = run_workload(args, sarch, sb, args.sub_steps, args.sub_warmup, world, rank, dev,
                                                dist, headline=False, cpu_seconds=args.sub_cpu_seconds)
    # compact per-config summary, LAST key of the line (the driver keeps only the tail of
    # stdout): value, step time, whole-model roofline fraction, dominant-kernel fraction, CPU
    res["summary"] = summarize(res)
    if dist is not None:
        # untimed: the AS-Norm cohort-statistics all-reduce (dist.allreduce_sums, one fused
        # f64 buffer over RCCL/xGMI, score_norm.py's cohort means) on this run's ranks,
        # checked against its closed form -- the one collective of the extraction path
        try:
            res["rccl_allreduce_check"] = rccl_check(dev, world, rank)
        except Exception as e:  # reported, never fatal to the measurement above
            res["rccl_allreduce_check"] = {"ok": False, "error": repr(e)[:300]}
    if rank == 0:
        summ = res.pop("summary")
        if "rccl_allreduce_check" in res:
            summ["rccl_allreduce_ok"] = (res["rccl_allreduce_check"] or {}).get("ok")
        res["summary"] = summ  # keep it last
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def summarize(res: dict) -> dict:
    def one(r, roof, kroof, cpu):
        # ECAPA headlines carry the dominant kernel's roofline as `roofline` itself (a per-kernel
        # figure: kernel_roofline repeats it); C3 / C4 carry a whole-model figure plus the
        # dominant kernel's from the standalone side pass
        per_kernel = (roof or {}).get("kernel", "").startswith("_Z")
        if kroof is None and per_kernel:
            kroof = roof
        k = kroof or {}
        mfma = k.get("bound") == "mfma"
        # the dominant kernel on one basis for every config: issued bf16x3 MFMA work (3 bf16
        # products per fp32 product) over the dense bf16 peak, or HBM bytes over 8 TB/s
        kfrac = (k.get("frac_issue_peak", k.get("frac_of_issue_peak")) if mfma else k.get("frac"))
        d = {"value": r.get("value"), "ms_per_step": r.get("ms_per_step"),
             "roofline_frac": (roof or {}).get("frac"),
             "roofline_kind": "kernel" if per_kernel else "model",
             "kernel_roofline_frac": kfrac,
             "kernel_roofline_basis": ("issued bf16x3 / bf16 peak" if mfma else "HBM") if k else None,
             "cpu_baseline": (cpu or {}).get("value")}
        if (kroof or {}).get("standalone_avg_ms") is not None:
            d["kernel_ms"] = kroof["standalone_avg_ms"]
        return d
    out = {res["config"]["arch"]: one(res, res.get("roofline"), res.get("kernel_roofline"), res.get("cpu_baseline"))}
    if res.get("value_batch64"):
        out[res["config"]["arch"]]["value_batch64"] = res["value_batch64"]["value"]
    for name, r in (res.get("configs") or {}).items():
        if name == "C5":
            if r:
                out[name] = {"seconds": r.get("value"), "stages_s": r.get("stages_s"),
                             "eval_emb_per_s": r.get("eval_emb_per_s")}
            continue
        out[name] = one(r, r.get("roofline"), r.get("kernel_roofline"), r.get("cpu_baseline"))
        if r.get("value_batch64"):
            out[name]["value_batch64"] = r["value_batch64"]["value"]
    out["n_gpus"] = res["n_gpus"]
    return out


if __name__ == "__main__":
    main()
