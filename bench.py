#!/usr/bin/env python3
"""Throughput benchmark: multimodal samples/s (train fwd+bwd+AdamW) on MI355X.

Workload (BASELINE.json metric "multimodal samples/sec (train fwd+bwd) at 1/2/4/8 MI355X;
MFMA util %"): the C3/C4 model — ResNet-50 image tower + 2-layer BiLSTM report encoder +
concat-fusion MLP + BCE — at C4's per-GPU batch (128 samples/GPU = 1024 global on 8 GPUs),
weak scaling, bf16 compute / fp32 master weights, synthetic 224x224 images + 128-token
reports.  `--config c2|c3|c5` selects the other BASELINE configs.

One step = H2D-free synthetic batch already in HBM -> image tower || text tower (two HIP
streams) -> fusion -> BCE -> backward -> (N>1: RCCL all-reduce of gradient buckets over
xGMI) -> clip_grad_norm_(1.0) -> fused AdamW.  Run:  python bench.py [--gpus N --steps K
--warmup W]; N>1 under torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    "c2": dict(image="resnet18", text="embed-mean", batch=64, seq=128,
               name="C2: ResNet-18 + embedding-mean text tower"),
    "c3": dict(image="resnet50", text="bilstm", batch=256, seq=128,
               name="C3: ResNet-50 + 2-layer BiLSTM, bs 256 on 1 GPU"),
    "c4": dict(image="resnet50", text="bilstm", batch=128, seq=128,
               name="C4: ResNet-50 + 2-layer BiLSTM, 128 samples/GPU (1024 global at 8 GPUs)"),
    "c5": dict(image="vit_b_16", text="bert-base-uncased", batch=64, seq=128,
               name="C5: ViT-B/16 + BERT-base, concat-fusion MLP, 64 samples/GPU "
                    "(512 global at 8 GPUs)"),
}

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def conv_flops_per_sample(trunk, hw=224):
    """Algorithmic conv FLOPs of one sample: fwd 2*MACs, dgrad 2*MACs (not for the stem,
    whose input needs no gradient), wgrad 2*MACs."""
    fwd = dgrad = 0
    H = W = hw
    convs = []

    def conv(c, H, W):
        k, s, p = c.kernel_size, c.stride, c.padding
        P = (H + 2 * p - k) // s + 1
        Q = (W + 2 * p - k) // s + 1
        return P * Q * c.out_channels * c.in_channels * k * k, P, Q

    macs, H, W = conv(trunk[0], H, W)
    convs.append(("stem", macs))
    fwd += macs
    H, W = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    for layer in list(trunk)[4:8]:
        for blk in layer:
            Hb, Wb = H, W
            for c, _, _ in blk.units():
                m, H, W = conv(c, H, W)
                fwd += m
                dgrad += m
            if blk.downsample is not None:
                m, _, _ = conv(blk.downsample[0], Hb, Wb)
                fwd += m
                dgrad += m
    return 2 * fwd, 2 * dgrad, 2 * fwd


def load_traffic(cfg_name, batch):
    """HBM bytes per launch of the dominant family (conv, or C5's dense GEMMs) from the newest
    committed PMC pass of this config (tools/pmc_traffic.py), or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            with open(f) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        if t.get("config") == cfg_name and t.get("per_gpu_batch") == batch:
            best = (t["traffic_bytes_per_launch"], os.path.relpath(f, ROOT),
                    t.get("git_rev", "unstamped"))
    return best


def load_mfma_util(cfg_name):
    """Per-family MFMA utilisation from the newest committed PMC pass of this config
    (tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8),
    dispatches serialised by the profiler; files without a config key are C4's), with the
    git revision it was measured on, or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_mfma_util.json"))):
        try:
            with open(f) as fh:
                t = json.load(fh)
        except (OSError, ValueError):
            continue
        if t.get("config", "c4") == cfg_name:
            best = (f, t)
    if best is None:
        return None
    f, t = best
    pct = {k: round(100 * v["mfma_util"], 1) for k, v in t.items()
           if isinstance(v, dict) and v.get("mfma_util") is not None
           and k in ("conv_fwd", "conv_dgrad", "conv_wgrad", "conv_all", "gemm")}
    return {"pct": pct, "source": os.path.relpath(f, ROOT),
            "git_rev": t.get("git_rev", "unstamped")}


def vit_flops_per_sample(layers=12, S=197, D=768, I=3072, patches=196, kpatch=768):
    """ViT-B/16 forward FLOPs of one 224x224 image (2 per MAC): patch embedding GEMM, per
    layer the QKV/out/MLP GEMMs and the two attention contractions (QK^T, PV)."""
    per_layer = S * (4 * D * D + 2 * D * I) + 2 * S * S * D
    return 2 * (patches * kpatch * D + layers * per_layer)


def model_flops_per_sample(cfg, img, txt):
    """(dominant-kernel-family train FLOPs, whole-model train FLOPs) per sample."""
    L = cfg["seq"]
    if cfg["image"] == "vit_b_16":
        D, I, layers = 768, 3072, 12
        bert = layers * L * 2 * (4 * D * D + 2 * D * I) + layers * 2 * 2 * L * L * D
        heads = 2 * (768 * 1024 + 768 * 512 + 1536 * 1024 + 1024 * 13)
        vit = vit_flops_per_sample()
        total = 3 * (vit + bert + heads)
        return None, total
    f, d, w = conv_flops_per_sample(img.backbone)
    conv_train = f + d + w
    text = 0
    if cfg["text"] == "bilstm":
        H = 256
        for l, inp in ((0, 256), (1, 512)):
            per_tok = 2 * (4 * H * inp + 4 * H * H)  # both directions: x2 below
            text += 2 * per_tok * L
    elif cfg["text"].startswith("bert"):
        D, I, layers = 768, 3072, 12
        text += layers * L * 2 * (4 * D * D + 2 * D * I) + layers * 2 * 2 * L * L * D
    heads = 2 * (img.backbone.feat_dim * 1024 + 512 * txt.hidden_size + 1536 * 1024 + 1024 * 13)
    return conv_train, conv_train + 3 * (text + heads)


def build(cfg, dev, dtype):
    import mmdx
    torch.manual_seed(0)
    img = mmdx.ImageEncoderCNN(cfg["image"], 1024, 13, compute_dtype=dtype).to(dev)
    txt = mmdx.TextEncoderTransformer(cfg["text"], 512, 13, compute_dtype=dtype).to(dev)
    fus = mmdx.FusionTransformerModel(1024, 512, 1024, 13, dropout=0.1).to(dev)
    img.unfreeze_backbone()
    txt.unfreeze_encoder()
    fus.train()
    # reference learning rates: image backbone 1e-4 / heads 5e-4 (TP:866-868), text encoder
    # 2e-5 / heads 5e-4 (TP:927), fusion 5e-4 (TP:1018-1023); weight decay 1e-2.
    groups = [
        {"params": list(img.backbone.parameters()), "lr": 1e-4},
        {"params": list(img.proj.parameters()) + list(img.classifier.parameters()), "lr": 5e-4},
        {"params": list(txt.encoder.parameters()), "lr": 2e-5},
        {"params": list(txt.proj.parameters()) + list(txt.classifier.parameters()), "lr": 5e-4},
        {"params": list(fus.parameters()), "lr": 5e-4},
    ]
    opt = mmdx.AdamW(groups, weight_decay=1e-2)
    return img, txt, fus, opt


def synth(cfg, B, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.rand(B, 3, 224, 224, generator=g, device=dev)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1)
    x = ((x - mean) / std).contiguous()
    L = cfg["seq"]
    ids = torch.randint(1000, 30522, (B, L), generator=g, device=dev)
    ids[:, 0] = 101
    ids[:, -1] = 102
    mask = torch.ones(B, L, dtype=torch.long, device=dev)
    y = (torch.rand(B, 13, generator=g, device=dev) < 0.15).float()
    return x, ids, mask, y


class StepTimer:
    """HIP events around every implicit-GEMM conv launch (or, for C5, every dense GEMM
    launch; the tag is then its FLOP count), recorded on the launching stream.  Events come
    from a pool created before the timed region (creating them inside it costs host time)."""

    def __init__(self):
        self.pairs = []
        self.enabled = False
        self.pool = []

    @property
    def active(self):
        return self.enabled

    def reserve(self, n):
        st = torch.cuda.current_stream()
        while len(self.pool) < 2 * n:
            e = torch.cuda.Event(enable_timing=True)
            e.record(st)  # creates the HIP event, so native code can record it by handle
            self.pool.append(e)
        torch.cuda.synchronize()

    def _event(self):
        if not self.pool:
            self.reserve(64)
        return self.pool.pop()

    def take(self, names):
        """(start, end) events for each named launch of a native plan run, in order."""
        evs = []
        for name in names:
            s, e = self._event(), self._event()
            self.pairs.append((name, s, e))
            evs += [s, e]
        return evs

    def __call__(self, name):
        timer = self

        class _Ctx:
            def __enter__(self_):
                if timer.enabled:
                    self_.s = timer._event()
                    self_.e = timer._event()
                    self_.s.record(torch.cuda.current_stream())
                return self_

            def __exit__(self_, *a):
                if timer.enabled:
                    self_.e.record(torch.cuda.current_stream())
                    timer.pairs.append((name, self_.s, self_.e))
        return _Ctx()


def graph_text_tower(txt, ids, mask):
    """The text tower's forward and backward as two hipGraphs (torch.cuda.make_graphed_callables
    over the mmdx launch sequence; tests/test_graph_capture_gpu.py checks replay == eager bit
    for bit): one replay call each per step instead of the tower's Python-issued launches.
    Returns text_fn() -> z_txt for make_step."""
    class _Tower(torch.nn.Module):
        def __init__(self, t):
            super().__init__()
            self.t = t

        def forward(self, i, m):
            return self.t(input_ids=i, attention_mask=m)["embeddings"]

    g = torch.cuda.make_graphed_callables(_Tower(txt), (ids, mask), allow_unused_input=True)
    return lambda: g(ids, mask)


def make_step(img, txt, fus, opt, params, reducer, x, ids, mask, y, side, side_bwd=None,
              scaler=None, text_fn=None):
    """One train step.  `scaler` (mmdx.GradScaler, the fp16 C5 path): the loss
    is scaled before the backward (TP:1056), clip_grad_norm_(1.0) is taken on the SCALED
    gradients as the reference's loop does (TP:1058, before scaler.step unscales them,
    TP:1060), the clip coefficient is folded with 1/scale into AdamW's gradient scale, and an
    overflow skips the update and backs the scale off (TP:1060-1061)."""
    import mmdx
    from mmdx import optim as MO
    from mmdx.schedule import TwoTowerForward, two_tower_backward
    from mmdx.trace import rng
    towers = TwoTowerForward(text_stream=side)
    text_early = os.environ.get("MMDX_DP_TEXT_EARLY", "1") != "0"

    def step():
        mk = step.marks
        opt.zero_grad(set_to_none=True)
        main = torch.cuda.current_stream()
        if mk:
            mk("start", main)
        side.wait_stream(main)
        # both towers issued at once: the image trunk (one native plan call) from this
        # thread onto the main stream, the text tower (Python-issued) from a worker thread
        # onto the side stream
        z_img, z_txt = towers(lambda: img(x)["embeddings"],
                              text_fn or (lambda: txt(input_ids=ids, attention_mask=mask)
                                                     ["embeddings"]))
        if mk:
            mk("image_fwd", main)
            mk("text_fwd", side)
        main.wait_stream(side)
        with rng("mmdx/fusion_fwd"):
            logits = fus(z_img, z_txt)["disease_logits"]
            loss = mmdx.BCEWithLogitsLoss()(logits, y)
        if mk:
            mk("head_fwd", main)
        # = loss.backward(), with the text tower's backward queued before the image trunk's;
        # N > 1: the text tower's and fusion head's gradients start their RCCL all-reduce
        # (from the text stream) while the image trunk is still in its backward
        early = None
        if reducer is not None and text_early:
            early = lambda: reducer.launch(list(txt.parameters()) + list(fus.parameters()))
        two_tower_backward(scaler.scale(loss) if scaler is not None else loss, z_img, z_txt,
                           fus.parameters(), text_stream=side if side_bwd is None else side_bwd,
                           on_text_done=early, mark=mk)
        if reducer is not None:
            reducer.reduce()
        with rng("mmdx/optimizer"):
            if scaler is not None:
                # the reference's order (TP:1056-1061): clip on the scaled gradients
                step.norm = scaler.clip_and_step(opt, 1.0, unscale_first=False, params=params)
                scaler.update()
            else:
                step.norm, scale = MO.grad_norm(params, 1.0)
                opt.step(grad_scale=scale)
        if mk:
            mk("optimizer", torch.cuda.current_stream())
        return loss
    step.norm = None
    step.marks = None   # diagnostics: mark(name, stream) once each part is issued
    step.towers = towers   # (tools/host_profile.py profiles the text thread through it)
    return step


def capture_step(step):
    """`step` recorded once into a hipGraph (torch.cuda.graph, relaxed capture: the text
    tower is issued from its worker thread onto the joined side stream); the returned
    callable replays it.  Inputs, parameters, gradients and optimizer state keep their
    addresses between replays; the dropout counters and the AdamW step count live on the
    device, so every replay is a fresh step."""
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, capture_error_mode="relaxed"):
        out = step()
    torch.cuda.synchronize()

    def replay():
        g.replay()
        return out
    replay.graph = g
    replay.norm = step.norm
    replay.towers = step.towers
    return replay


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Host threads for the CPU baseline: BASELINE.md's plan says os.cpu_count(), but on a
    GPU box that counts the whole machine while this process gets a share of it
    (OMP_NUM_THREADS / the affinity mask); oversubscribing that share only slows torch's
    CPU kernels, so the share is used and both numbers are reported."""
    share = os.environ.get("OMP_NUM_THREADS")
    n = int(share) if share and share.isdigit() else len(os.sched_getaffinity(0))
    return max(1, min(n, os.cpu_count() or n))


def cpu_baseline(cfg, bs=8, warmup=10, steps=50):
    """Time the CPU oracle (the reference's PyTorch-CPU path restated, oracle/ref_cpu.py) per
    BASELINE.md's plan: the reference's AdamW groups (TP:238-269 image phase 2, TP:408-432
    text phase 2, TP:1018-1023 fusion), clip_grad_norm_(1.0), `warmup` untimed steps, then
    the MEDIAN of `steps` timed fwd+bwd+AdamW steps of `bs` samples."""
    from oracle import ref_cpu as R
    threads = cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    text = cfg["text"]
    model = R.RefMultimodal(cfg["image"], text, dropout=0.0)
    model.train()
    groups = [
        {"params": list(model.image.backbone.parameters()), "lr": 1e-4},
        {"params": list(model.image.proj.parameters()) +
         list(model.image.classifier.parameters()), "lr": 5e-4},
        {"params": list(model.text.encoder.parameters()), "lr": 2e-5},
        {"params": list(model.text.proj.parameters()) +
         list(model.text.classifier.parameters()), "lr": 5e-4},
        {"params": list(model.fusion.parameters()), "lr": 5e-4},
    ]
    opt = torch.optim.AdamW(groups, weight_decay=1e-2)
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(bs, 3, 224, 224, generator=g)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    x = (x - mean) / std
    ids = torch.randint(1000, 30522, (bs, cfg["seq"]), generator=g)
    ids[:, 0], ids[:, -1] = 101, 102
    mask = torch.ones(bs, cfg["seq"], dtype=torch.long)
    y = (torch.rand(bs, 13, generator=torch.Generator().manual_seed(1235)) < 0.15).float()
    for _ in range(warmup):
        R.ref_train_step(model, opt, x, ids, mask, y)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        R.ref_train_step(model, opt, x, ids, mask, y)
        ts.append(time.perf_counter() - t0)
    med = sorted(ts)[len(ts) // 2]
    return {"value": round(bs / med, 3), "unit": "samples/s", "cores": threads,
            "kind": "port", "cpu_model": _cpu_model(), "machine_cpus": os.cpu_count(),
            "sample": f"median of {steps} oracle train steps (after {warmup} warm-up) x {bs} "
                      f"samples ({cfg['image']} + {text}, 224x224, L={cfg['seq']}; "
                      f"reference AdamW groups, clip 1.0), torch CPU fp32, {threads} threads"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(n, argv, port):
    """The command that starts `n` bench ranks (one process per GPU) on this node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """`python bench.py --gpus N` with no launcher around it: start the N ranks as child
    processes of torch.distributed.run (this process has made no GPU call, and it waits for
    the children instead of replacing itself) and return their exit status.  Rank 0 prints
    the JSON line."""
    import subprocess
    backend = os.environ.get("MMDX_DIST_BACKEND", "nccl")
    if backend == "nccl":
        have = torch.cuda.device_count()   # counts devices without initialising HIP
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} GPUs for RCCL, {have} visible "
                  f"(MMDX_DIST_BACKEND=gloo rehearses several ranks on one GPU)",
                  file=sys.stderr, flush=True)
            return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_cmd(n, argv, _free_port()), env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch override")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=50)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks",
              file=sys.stderr, flush=True)
        sys.exit(2)

    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg["batch"] = args.batch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MMDX_DIST_BACKEND=gloo rehearses the DP path with several ranks on one GPU (RCCL
    # refuses two ranks per device); the real multi-GPU run uses "nccl" (= RCCL over xGMI).
    backend = os.environ.get("MMDX_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    # MMDX_DP_REHEARSE=1 under torch.distributed.run with one rank: the full data-parallel
    # path (RCCL process group, comm stream, mid-backward trunk all-reduces) on one GPU
    dp = world > 1 or os.environ.get("MMDX_DP_REHEARSE", "0") == "1"
    if dp:
        from mmdx.dist import init_distributed
        torch.cuda.set_device(local)
        init_distributed(backend, local)   # RCCL async errors / timeouts fail the job fast
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the process group has "
                  f"{dist.get_world_size()} ranks", file=sys.stderr, flush=True)
            sys.exit(2)
        world = dist.get_world_size()
    dev = torch.device("cuda", local)
    # C5 is specified as "fp16 MFMA" (BASELINE.json); C2-C4 compute in bf16 (fp32 masters)
    dtype = torch.float16 if cfg["image"] == "vit_b_16" else torch.bfloat16

    import mmdx
    from mmdx import resnet as RN
    from mmdx import functional as MF
    img, txt, fus, opt = build(cfg, dev, dtype)
    vit = cfg["image"] == "vit_b_16"
    params = [p for grp in opt.param_groups for p in grp["params"]]
    if dp:  # identical initial weights on every rank (broadcast from rank 0)
        with torch.no_grad():
            for p in list(img.parameters()) + list(txt.parameters()) + list(fus.parameters()):
                dist.broadcast(p, 0)
    B = cfg["batch"]
    # Stream priorities: the step is issued on a high-priority stream (the dgrad chain, BN
    # and the heads) and the text tower's stream is high priority too, so the trunk's
    # weight-gradient stream (default priority) fills the CUs they leave.  Measured at C4
    # (2 x 40 steps each): main+text 7866, text only 7822, main only 7781, none 7805.
    torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    x, ids, mask, y = synth(cfg, B, dev, 1234 + rank)
    side = torch.cuda.Stream(device=dev, priority=-1)
    if os.environ.get("MMDX_TEXT_STREAM", "side") == "main":  # A/B: towers in series
        side = torch.cuda.current_stream()
    from mmdx.dist import GradAllReducer
    # Every gradient reduces in fp32 (the mean of 8 bf16 sums would drop ~3 bits against
    # the fp32 DDP mean).  MMDX_DP_BUCKET_DTYPE=bf16 sends C5's packed buckets (the ViT-B/16 and
    # BERT-base gradients outside the two encoder stacks: embeddings, patch projection,
    # heads) in bf16, half their xGMI bytes, the mean taken in fp32 after the cast back.
    bdt = None
    if vit and os.environ.get("MMDX_DP_BUCKET_DTYPE", "fp32") == "bf16":
        bdt = torch.bfloat16
    reducer = GradAllReducer(params, world, rehearse=dp, bucket_dtype=bdt) if dp else None
    # The trunk's layer 4, 3, 2 gradients start their all-reduce mid-backward.  The first
    # version waited on a plan event from a comm stream: in the one-rank RCCL rehearsal it
    # cost 0.43 ms/step (15.83 vs 15.40 ms) — the comm and RCCL streams' event waits share
    # the process's 4 hardware queues with the text and weight-gradient streams.  The text
    # tower's and fusion head's buckets start as soon as their gradients are final
    # (MMDX_DP_TEXT_EARLY, on: 0.08 ms here, ~66 MB of the collective hidden at N > 1).
    # gloo's CUDA path would stall the issuing host thread (1.3 s/step in the one-GPU
    # rehearsal), so gloo keeps the after-backward reduce.
    # Default (RCCL): the trunk backward plan is replayed in per-layer segments and the
    # all-reduce of layers 4, 3, 2's gradient slices is issued between them from the
    # weight-gradient stream itself (resnet.TRUNK_SEGMENT_HOOK): no comm stream, no event
    # waits beyond RCCL's own, so the process stays within its 4 hardware queues (main, text,
    # weight-gradient, RCCL).  MMDX_DP_EARLY_TAIL=event: the comm-stream variant above;
    # 0: the whole arena after the backward.
    early_tail = os.environ.get("MMDX_DP_EARLY_TAIL", "seg" if backend == "nccl" else "0")
    if reducer is not None and early_tail == "event":
        RN.TRUNK_GRAD_HOOK = reducer.trunk_hook
    elif reducer is not None and early_tail not in ("0", ""):
        RN.TRUNK_SEGMENT_HOOK = reducer.trunk_segment
        # C5: the ViT-B/16 and BERT-base encoder stacks' backward plans are cut every
        # xplan.SEG_LAYERS layers and each finished group's gradient slice is all-reduced in
        # place from there, beside the remaining layers' backward (the same hook: issued
        # with the backward's stream current; every rank issues the collectives in the same
        # order — image stack, then text stack — from the thread running the backward)
        from mmdx import xplan as XP
        XP.STACK_SEGMENT_HOOK = reducer.trunk_segment
    # fp16 (C5): loss scaling with GradScaler semantics (TP:1025-1026, 1056-1061)
    scaler = mmdx.GradScaler() if dtype == torch.float16 else None
    # MMDX_GRAPH_TEXT=1: the text tower replayed from hipGraphs (capture after build, before
    # the warm-up; the capture itself runs eagerly on torch's capture stream)
    text_fn = None
    graph_text = os.environ.get("MMDX_GRAPH_TEXT", "0") == "1"
    if graph_text:
        with torch.cuda.stream(side):
            text_fn = graph_text_tower(txt, ids, mask)
        torch.cuda.synchronize()
    step = make_step(img, txt, fus, opt, params, reducer, x, ids, mask, y, side, scaler=scaler,
                     text_fn=text_fn)
    timer = StepTimer()
    if vit:   # dominant kernel family: the dense GEMMs of the ViT and BERT encoders
        MF.GEMM_TIMER = timer
    else:     # dominant kernel family: the implicit-GEMM conv launches
        RN.CONV_TIMER = timer

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # MMDX_GRAPH_STEP=1: the whole train step (both towers, backward, clip, AdamW) captured
    # into one hipGraph after the warm-up and replayed per step (no per-kernel host issue)
    graph_step = os.environ.get("MMDX_GRAPH_STEP", "0") == "1"
    if graph_step:
        step = capture_step(step)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    if dp:
        dist.barrier()
    # Conv (dominant-family) launch durations: HIP events around every conv launch of the
    # LAST `ev_steps` timed steps (default K/10).  Bracketing every step costs ~0.75 ms/step
    # of event markers at C4 (316 records), which would bias `value`; the sampled steps are
    # ordinary steps of the timed loop, so the per-launch average is the timed region's.
    timing = os.environ.get("MMDX_BENCH_EVENTS", "1") != "0"
    ev_steps = min(args.steps, max(1, int(os.environ.get("MMDX_BENCH_EVENT_STEPS",
                                                         max(1, args.steps // 10)))))
    timer.reserve(400 * ev_steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        timer.enabled = timing and i >= args.steps - ev_steps
        loss = step()
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (no device sync)
    torch.cuda.synchronize()
    if cfg["text"] == "bilstm":
        # a cooperative recurrence that lost a peer invalidates the run: fail loudly
        from mmdx.bilstm import check_recurrence
        check_recurrence()
    if dp:
        dist.barrier()
    el = time.perf_counter() - t0
    # host cost of one step issued onto an idle device (no queue back-pressure)
    was = timer.enabled
    timer.enabled = False
    t1 = time.perf_counter()
    step()
    host_one = time.perf_counter() - t1
    torch.cuda.synchronize()
    timer.enabled = was
    # MMDX_BENCH_TIMELINE=N (diagnostics): N more steps after the timed region with a HIP event
    # recorded when each part of the step has been issued, on the stream it runs on — when
    # each part ENDS on the device, in ms after the step's start (mean over the N steps): which
    # stream the step's tail waits for
    timeline = None
    tl_steps = int(os.environ.get("MMDX_BENCH_TIMELINE", "0") or 0)
    if tl_steps > 0 and not graph_step:
        recs = []
        only = os.environ.get("MMDX_BENCH_TIMELINE_MARKS")  # e.g. "start,optimizer"
        only = set(only.split(",")) | {"start"} if only else None

        def mark(name, stream):
            if only is None or name in only:
                e = torch.cuda.Event(enable_timing=True)
                e.record(stream)
                recs[-1].append((name, e))
        step.marks = mark
        for _ in range(tl_steps):
            recs.append([])
            step()
        step.marks = None
        torch.cuda.synchronize()
        # device time per marked step over the second half (steady state): the start mark of
        # its first step to the last step's final mark
        half = len(recs) // 2
        tl_wall = recs[half][0][1].elapsed_time(recs[-1][-1][1]) / (len(recs) - half)
        acc = {}
        for rec in recs[len(recs) // 2:]:   # the second half: steady state
            for name, e in rec[1:]:
                acc.setdefault(name, []).append(rec[0][1].elapsed_time(e))
        timeline = {k: round(sum(v) / len(v), 3) for k, v in acc.items()}
        timeline["ms_per_step"] = round(tl_wall, 3)
    conv_steps = ev_steps
    timer.enabled = False
    if dp:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    conv_ms = sum(s.elapsed_time(e) for _, s, e in timer.pairs)
    n_conv = len(timer.pairs)
    # wall time during which at least one timed launch was running (union of the launch
    # intervals, all events on one device): the family's launches overlap each other (the
    # weight-gradient stream beside the dgrad chain), so the per-launch sum above counts
    # shared time twice; this is the extra `busy_*` figure, the contract's `frac` stays
    busy_ms = 0.0
    if timer.pairs:
        ref = timer.pairs[0][1]
        iv = sorted((ref.elapsed_time(s), ref.elapsed_time(e)) for _, s, e in timer.pairs)
        lo, hi = iv[0]
        for a, b in iv[1:]:
            if a > hi:
                busy_ms += hi - lo
                lo, hi = a, b
            else:
                hi = max(hi, b)
        busy_ms += hi - lo
    conv_flops, total_flops = model_flops_per_sample(cfg, img, txt)
    table = os.environ.get("MMDX_BENCH_LAUNCH_TABLE")
    if table and rank == 0 and timer.pairs:
        # per-launch in-step durations (launch order of one step, averaged over the timed
        # steps with events) against each launch's own roof max(FLOPs/peak, bytes/BW)
        per = len(timer.pairs) // conv_steps
        with open(table, "w") as fh:
            fh.write("idx kind gflop mb us roof_us frac bound shape\n")
            for i in range(per):
                tag = timer.pairs[i][0]
                us = sum(timer.pairs[i + k * per][1].elapsed_time(timer.pairs[i + k * per][2])
                         for k in range(conv_steps)) / conv_steps * 1e3
                fr = tag[1] / (PEAK_BF16_TFLOPS * 1e6)
                br = tag[2] / (PEAK_HBM_GBS * 1e3)
                roof = max(fr, br)
                fh.write(f"{i} {tag[0]} {tag[1] / 1e9:.3f} {tag[2] / 1e6:.2f} {us:.1f} "
                         f"{roof:.1f} {roof / us if us > 0 else 0:.3f} "
                         f"{'mfma' if fr > br else 'hbm'} {tag[3].replace(' ', '_')}\n")

    samples = B * world * args.steps
    value = samples / el
    ms_step = el / args.steps * 1e3
    # every timed launch carries its algorithmic cost (resnet.LaunchCost: kind, FLOPs, bytes)
    fam_flops = sum(tag[1] for tag, _, _ in timer.pairs)
    fam_bytes = sum(tag[2] for tag, _, _ in timer.pairs)
    # combined per-launch roofline: each launch's own roof max(FLOPs / MFMA peak, bytes / HBM
    # peak), summed over the family, against the family's summed launch durations
    roof_ms = sum(max(tag[1] / (PEAK_BF16_TFLOPS * 1e9), tag[2] / (PEAK_HBM_GBS * 1e6))
                  for tag, _, _ in timer.pairs)
    flop_ms = fam_flops / (PEAK_BF16_TFLOPS * 1e9)
    byte_ms = fam_bytes / (PEAK_HBM_GBS * 1e6)
    # The family's time is the union of its launch intervals (wall time with at least one of
    # its kernels running; never more than the step).  The per-launch event SUM over-counts:
    # each pair also spans the launch's dispatch gap behind the previous packet of its stream
    # (≈ 7 µs per launch at C4, the sum exceeded the step), and launches on the weight-gradient
    # stream overlap the dgrad chain.  The sum stays in the line as `family_event_sum_ms`.
    fam_ms = busy_ms if busy_ms > 0 else conv_ms
    conv_tf = fam_flops / (fam_ms * 1e-3) / 1e12 if fam_ms > 0 else 0.0
    conv_gbs = fam_bytes / (fam_ms * 1e-3) / 1e9 if fam_ms > 0 else 0.0
    if vit:
        conv_flops = fam_flops / max(1, conv_steps) / B
    alg_bytes = fam_bytes / max(1, conv_steps)
    alg_launches = max(1, n_conv // max(1, conv_steps))
    hbm_bound = byte_ms > flop_ms
    traffic = load_traffic(args.config, B)
    result = {
        "metric": "multimodal samples/sec (train fwd+bwd) at 1/2/4/8 MI355X; MFMA util %",
        "value": round(value, 2),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16" if dtype == torch.float16 else "bf16",
        "data": "synthetic (U[0,1) ImageNet-normalised 224x224 images, 128-token [CLS]..[SEP] "
                "reports, Bernoulli(0.15) labels); random-init weights",
        "launch": ("hipGraph (whole step)" if graph_step else
                   "eager" + (" (text tower: hipGraph replay)" if graph_text else "")),
        "stream_priority": "main+text",
        "dist_backend": backend if dp else None,
        "config": {"workload": cfg["name"], "image_tower": cfg["image"],
                   "text_tower": cfg["text"], "global_batch": B * world,
                   "per_gpu_batch": B, "seq_len": cfg["seq"], "image_hw": 224,
                   "parallelism": f"dp{world}" + ("-rccl-rehearsal" if dp and world == 1
                                                  else "")},
        "loss": round(float(loss.item()), 5),
        "loss_scale": scaler.get_scale() if scaler is not None else None,
        "dp_bucket_dtype": ("bf16" if bdt is not None else "fp32") if dp else None,
        "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 3),
        "host_ms_one_step_idle_device": round(host_one * 1e3, 3),
        **({"timeline_ms": timeline} if timeline else {}),
        "model_tflops": round(total_flops * samples / el / 1e12, 2),
        "mfma_util_pct_end_to_end": round(100 * total_flops * samples / el / 1e12 /
                                          (PEAK_BF16_TFLOPS * world), 2),
        "mfma_util_pmc": load_mfma_util(args.config),
        "amp": ({"loss_scaling": "mmdx.GradScaler (init 2^16, growth 2 per 2000 clean steps, "
                                 "backoff 0.5, device-side inf check, overflow skips AdamW)",
                 "clip_order": "reference (scaled): clip_grad_norm_(1.0) on the SCALED "
                               "gradients, then scaler.step unscales (TP:1056-1061)"}
                if scaler is not None else None),
        "roofline": {
            "kernel": ("igemm_dma_kernel (dense GEMMs of the ViT-B/16 and BERT-base encoders, "
                       "fwd + both backward GEMMs)") if vit else
                      "igemm_dma_kernel (implicit-GEMM conv fwd/dgrad/wgrad, all ResNet convs)",
            # the family's bound: the larger of its summed FLOP time and byte time at peak
            "bound": "hbm" if hbm_bound else "mfma",
            "achieved": round(conv_gbs if hbm_bound else conv_tf, 2),
            "peak": PEAK_HBM_GBS if hbm_bound else PEAK_BF16_TFLOPS,
            "unit": "GB/s" if hbm_bound else "TFLOP/s",
            "frac": round((conv_gbs / PEAK_HBM_GBS) if hbm_bound
                          else (conv_tf / PEAK_BF16_TFLOPS), 4),
            "traffic": traffic[0] if traffic else None,
            "traffic_unit": ("HBM bytes per %s launch (PMC, (2*FETCH_SIZE+WRITE_SIZE)*1KiB)"
                             % ("GEMM" if vit else "conv")),
            "traffic_source": traffic[1] if traffic else None,
            "traffic_git_rev": traffic[2] if traffic else None,
            "algorithmic_bytes_per_launch": round(alg_bytes / alg_launches),
            "mfma_achieved_tflops": round(conv_tf, 2),
            "mfma_frac": round(conv_tf / PEAK_BF16_TFLOPS, 4),
            "hbm_achieved_gbs": round(conv_gbs, 1),
            "hbm_frac": round(conv_gbs / PEAK_HBM_GBS, 4),
            "combined_roof_ms_per_step": round(roof_ms / conv_steps, 3),
            "combined_frac": round(roof_ms / fam_ms, 4) if fam_ms > 0 else None,
            "combined_frac_note": "sum over launches of max(FLOPs/2.5 PF, bytes/8 TB/s) "
                                  "divided by the family's busy time",
            "family_ms_per_step": round(fam_ms / conv_steps, 3),
            "family_time": "union of the family's HIP-event launch intervals (busy time)",
            "family_event_sum_ms_per_step": round(conv_ms / conv_steps, 3),
            "event_sum_frac": (round((fam_bytes / (conv_ms * 1e6)) / PEAK_HBM_GBS if hbm_bound
                                     else fam_flops / (conv_ms * 1e9) / PEAK_BF16_TFLOPS, 4)
                               if conv_ms > 0 else None),
            "family_launches_per_step": n_conv // max(1, conv_steps),
            "family_gflop_per_sample": round(conv_flops / 1e9, 3),
            "family_alg_gb_per_step": round(alg_bytes / 1e9, 3),
            "timed_steps_with_events": conv_steps,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # C5's oracle (ViT-B/16 + BERT-base) takes seconds per CPU step: a shorter sample
        heavy = cfg["image"] == "vit_b_16"
        result["cpu_baseline"] = cpu_baseline(cfg, warmup=2 if heavy else 10,
                                              steps=min(args.cpu_steps, 5) if heavy
                                              else args.cpu_steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
