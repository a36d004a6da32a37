"""Benchmark: SwinV2-T 224 (window 7) + HXE over a 7-tier, 10 000-leaf iNat21-shaped
taxonomy, one data-parallel training step per "step", 256 images per GPU
(BASELINE.json configs[2]; the metric BASELINE.json names).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself
(torch.distributed.run on 127.0.0.1 as a child process, before anything touches the GPU) and
exits with its status; under an external launcher WORLD_SIZE must equal --gpus.

A step = forward + HXE loss + backward (bucketed RCCL all-reduce overlapped) + grad-norm
clip + DecoupledSGDW update, bf16 autocast, f32 master weights; synthetic images/labels
resident in HBM.  Rank 0 prints one JSON line.  The W-MSA roofline is measured live with
HIP events around every W-MSA launch inside the timed steps; the CPU baseline (rank 0,
N = 1 only) times the oracle's f32 CPU restatement of the same model + loss on a bounded
sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec/GPU SwinV2-T 224² HXE bs256; W-MSA HBM GB/s vs peak; 1→8 scaling"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--model", default="swinv2_tiny_window7_224")
    ap.add_argument("--loss", default="hxe", choices=["hxe", "multitask", "ce"])
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: time HIP-graph replays of the step (trainer.capture/replay); 0: eager "
                         "(default: keeps the RCCL all-reduce overlapped with the backward)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the measured path); gloo only to rehearse the "
                         "multi-rank flow with several ranks sharing one GPU")
    ap.add_argument("--roofline-steps", type=int, default=4,
                    help="graph mode: eager warm-up steps whose W-MSA launches are timed")
    return ap.parse_args()


def build(args, device):
    from hvamd import configs, hierarchy, models, optim
    from hvamd.algorithmic import GradientClipping
    from hvamd.trainer import Trainer

    cfg = configs.Config()
    cfg.model.name = args.model
    tax = hierarchy.Taxonomy.synthetic()
    if args.loss == "hxe":
        cfg.hierarchy.variant = "hxe"
        cfg.hierarchy.hxe_tree_weights = "exponential"
        info = models.DatasetInfo(num_classes=tax.num_leaves, taxonomy=tax)
    elif args.loss == "multitask":
        cfg.hierarchy.variant = "multitask"
        cfg.hierarchy.multitask_coeffs = [8, 5.65, 4, 2.82, 2, 1.41, 1]
        info = models.DatasetInfo(num_classes=tax.num_classes, taxonomy=tax)
    else:
        info = models.DatasetInfo(num_classes=1000)
    # reference optimizer (DecoupledSGDW, momentum 0.875, wd 5e-4; configs.py:421-425) at an
    # lr that does not diverge from random init (2.048 is tuned for ResNet-50 at batch 2048);
    # the work per step does not depend on it
    cfg.optim.lr = 0.02
    model = models.build_composer_model(cfg, info).to(device)
    opt = optim.build_optimizer(cfg, model)
    trainer = Trainer(model, opt, [GradientClipping("norm", 2.0)])
    return cfg, tax, model, trainer


def synthetic_batch(args, tax, rank, device, img=224):
    g = torch.Generator(device=device)
    g.manual_seed(42 + rank)
    x = torch.randn((args.batch, 3, img, img), generator=g, device=device)
    leaves = np.random.default_rng(42 + rank).integers(0, tax.num_leaves, args.batch)
    if args.loss == "ce":
        y = torch.from_numpy(leaves % 1000).to(device)
    else:
        y = torch.from_numpy(tax.leaf_paths[leaves]).to(device)
        if args.loss == "hxe":
            y = y.contiguous()
    return x, y


TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_traffic.json")
TRAFFIC_SOURCE = ("bench_traffic.json: HBM bytes per launch (mean over the step's launches) from "
                  "rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE passes over this bench "
                  "(tools/gpu_traffic.sh); null when that file is absent")


def measured_traffic(kernel):
    """Mean HBM bytes per launch of `kernel` from the committed PMC measurement, or None."""
    try:
        with open(TRAFFIC_FILE) as f:
            return json.load(f)["kernels"][kernel]["traffic_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def wmsa_algorithmic_bytes(model, batch):
    """Per-step algorithmic HBM bytes of the W-MSA kernels:
    forward 8*T*C (bf16 qkv read 3C + out write C), backward 16*T*C."""
    from hvamd.swinv2 import SwinTransformerBlock
    tc = 0
    for m in model.modules():
        if isinstance(m, SwinTransformerBlock):
            H, W = m.input_resolution
            tc += batch * H * W * m.dim
    return 8 * tc, 16 * tc


def cpu_baseline(args, seconds):
    """The oracle's f32 CPU restatement: SwinV2-T forward + HXE + backward."""
    from hvamd.hierarchy import Taxonomy
    from oracle import hierarchy_ref, swinv2_ref

    threads = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    cfg = dict(img_size=224, embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24),
               window_size=7)
    tax = Taxonomy.synthetic()
    p = swinv2_ref.init_params_from_rng(swinv2_ref.state_shapes(num_classes=tax.num_leaves, **cfg), 0)
    for v in p.values():
        v.requires_grad_(True)
    geom = swinv2_ref.model_geometry(**cfg)
    lam = hierarchy_ref.hxe_level_weights("exponential", 0.1)
    bs = 8
    x = torch.randn(bs, 3, 224, 224)
    paths = tax.leaf_paths[np.random.default_rng(0).integers(0, tax.num_leaves, bs)]

    def step():
        logits = swinv2_ref.forward(p, x, geom)
        loss = hierarchy_ref.hxe_loss_torch(logits, paths, tax.perm, tax.node_start, tax.node_end,
                                            tax.tier_base, lam)
        loss.backward()
        for v in p.values():
            v.grad = None

    step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return {"value": round(n * bs / el, 3), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"{n} train steps x {bs} images (SwinV2-T 224 + HXE, f32, oracle/swinv2_ref.py)"}


def launch_ranks(args):
    """--gpus N > 1 without a launcher: run this script under torch.distributed.run as a child
    (one process per GPU, RCCL rendezvous on 127.0.0.1) and return its exit status.  Nothing
    here touches the GPU, so the parent holds no device context while the ranks run."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":  # rehearsal: ranks may share a GPU
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != world:
            raise RuntimeError(f"RCCL sees {dist.get_world_size()} ranks, expected {world}")
    import hvamd.ops as ops

    cfg, tax, model, trainer = build(args, device)
    img = model.module.patch_embed.img_size[0]
    batch = synthetic_batch(args, tax, rank, device, img)

    fwd_bytes, bwd_bytes = wmsa_algorithmic_bytes(model.module, args.batch)
    timing = not args.no_roofline
    timer, timed_steps = None, args.steps
    if args.graph:
        # eager warm-up; the last roofline_steps of it carry the W-MSA kernel timer (graph
        # replays cannot: per-kernel dispatch events are not captured), then capture
        rsteps = min(args.roofline_steps, max(args.warmup, 1)) if timing else 0
        for i in range(max(args.warmup, 1)):
            if timing and i == max(args.warmup, 1) - rsteps:
                torch.cuda.synchronize()
                ops.kernel_timer_start()
            trainer.train_step(batch)
        if timing:
            torch.cuda.synchronize()
            timer, timed_steps = ops.kernel_timer_stop(), rsteps
        trainer.capture(batch)
        step = trainer.replay
    else:
        for _ in range(args.warmup):
            trainer.train_step(batch)

        def step():
            return trainer.train_step(batch)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if timing and not args.graph:  # W-MSA launches timed by their own dispatch packets
        ops.kernel_timer_start()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if timing and not args.graph:
        timer = ops.kernel_timer_stop()
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_val = float(loss)
    if not np.isfinite(loss_val):
        raise RuntimeError(f"non-finite loss {loss_val}")
    images = world * args.batch * args.steps
    value = images / elapsed
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (randn images resident in HBM, leaves uniform over a synthetic 10k-leaf "
                "7-tier tree); random-init weights",
        "config": {"workload": "SwinV2-T 224 w7 + HXE (10000 leaves, 7 tiers) train step",
                   "model": args.model, "loss": args.loss, "global_batch": world * args.batch,
                   "per_gpu_batch": args.batch, "image_size": img,
                   "parallelism": f"dp{world}",
                   "execution": "hip-graph replay" if args.graph else "eager"},
        "value_per_gpu": round(value / world, 2),
        "comm": ({"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                  "grad_buckets": len(trainer.buckets.buckets),
                  "grad_bytes_per_step": 4 * sum(b[0].numel() for b in trainer.buckets.buckets)}
                 if world > 1 else None),
        "final_loss": round(loss_val, 4),
    }
    if timer:
        fw_ms, fw_n = timer["wmsa_fwd"]
        bw_ms, bw_n = timer["wmsa_bwd"]
        n_launch = fw_n // timed_steps
        fwd_gbs = fwd_bytes * timed_steps / (fw_ms / 1000) / 1e9
        bwd_gbs = bwd_bytes * timed_steps / (bw_ms / 1000) / 1e9
        result["roofline"] = {
            "kernel": "wmsa_fwd_ring_kernel<7,3|4> (all %d launches per step)" % n_launch,
            "bound": "hbm", "achieved": round(fwd_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(fwd_gbs / HBM_PEAK_GBS, 4), "traffic": measured_traffic("wmsa_fwd"),
            "algorithmic_bytes_per_step": fwd_bytes,
            "avg_launch_us": round(1000 * fw_ms / fw_n, 2),
            "ms_per_step": round(fw_ms / timed_steps, 3),
            "timing": ("dispatch-packet events (hipExtLaunchKernelGGL) over %d eager steps just "
                       "before the graph capture (replays carry no per-kernel events)" % timed_steps
                       if args.graph else
                       "dispatch-packet events (hipExtLaunchKernelGGL) over the timed steps")}
        if result["roofline"]["traffic"] is not None:
            result["roofline"]["algorithmic_bytes_per_launch"] = fwd_bytes // n_launch
            result["roofline"]["traffic_source"] = TRAFFIC_SOURCE
        result["roofline_bwd"] = {
            "kernel": "wmsa_bwd_kernel<7>", "bound": "hbm", "achieved": round(bwd_gbs, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bwd_gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_step": bwd_bytes, "traffic": measured_traffic("wmsa_bwd"),
            "avg_launch_us": round(1000 * bw_ms / bw_n, 2),
            "ms_per_step": round(bw_ms / timed_steps, 3)}
    if rank == 0 and world == 1 and args.cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
