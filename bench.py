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
dispatch-packet events around every W-MSA launch of extra steps right after the timed ones (the
timed region carries no timer; those steps keep the parameter-gradient side stream off, so a
launch is not priced with a concurrent weight gradient on its CUs); the CPU baseline (rank 0,
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
MFMA_PEAK_TFS = 2500.0  # MI355X dense bf16 MFMA (no sparsity)
# transcendental roof: v_exp_f32 issues at 8 cycles per wave64 instruction on a SIMD (quarter
# of the 2-cycle VALU rate; MI355X_MICROARCH.md, vector-instruction issue cost): 8 exp per
# cycle per SIMD x 1024 SIMDs x 2.4 GHz
EXP_PEAK_TS = 8 * 1024 * 2.4e9 / 1e12


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
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="set a libhvk option (include/hvk.h hvk_set_option) before the run; A/B runs")
    ap.add_argument("--stream-priority", type=int, default=0,
                    help="run on a stream of this priority (negative = higher than the side stream's)")
    ap.add_argument("--host-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="set a host routing option (hvamd.options) before the run; A/B runs")
    ap.add_argument("--steps-in-flight", type=int, default=-1,
                    help="eager steps the host may enqueue ahead of the GPU (Trainer.max_steps_in_flight; "
                         "0: unbounded; default: the Trainer's)")
    ap.add_argument("--comm-steps", type=int, default=5,
                    help="world > 1: extra eager steps after the timed region that record the "
                         "exchange's exposed time and bucket enqueue points (the `comm` block)")
    return ap.parse_args()


def build(args, device):
    from hvamd import configs, hierarchy, models, optim
    from hvamd.algorithmic import EMA, GradientClipping
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
    # the recipe's EMA (configs/pretrain/inat21.yaml:32-35: half-life 100 batches, updated every
    # 20), folded into the fused optimizer step on its update batches
    trainer = Trainer(model, opt, [GradientClipping("norm", 2.0), EMA(half_life="100ba", update_interval="20ba")])
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


def measured_traffic(kernel, fetch_scale=2.0):
    """Mean HBM bytes per launch of `kernel` from the committed PMC measurement, or None.
    fetch_scale: the gfx950 FETCH_SIZE correction (x2 for coalesced 16-B-per-lane reads and
    LDS-DMA, the committed figure; x1.5 for isolated 64-B segment reads, reported beside it)."""
    try:
        with open(TRAFFIC_FILE) as f:
            k = json.load(f)["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None
    if fetch_scale == 2.0:
        return k["traffic_bytes_per_launch"]
    return int(k["fetch_bytes_per_launch"] * fetch_scale / 2.0) + k["write_bytes_per_launch"]


def wmsa_work(model, batch):
    """Per-step algorithmic work of the W-MSA kernels, summed over blocks with
    each block's effective window: bytes forward 8*T*C (bf16 qkv read 3C + out write C per
    token), backward 16*T*C; flops forward 4*T*N*C (Q K^T and P V), backward 10*T*N*C, with
    T = batch*H*W tokens and N = w*w tokens per window; exponentials forward T*N*nH (one per
    query-key pair and head), backward 2*T*N*nH (P recomputed in the query phase and again in
    the key phase of the large-window kernels), nH = C/32."""
    from hvamd.swinv2 import SwinTransformerBlock
    w = dict(fwd_bytes=0, bwd_bytes=0, fwd_flops=0, bwd_flops=0, fwd_exp=0, bwd_exp=0, windows=set())
    for m in model.modules():
        if isinstance(m, SwinTransformerBlock):
            H, W = m.input_resolution
            tc = batch * H * W * m.dim
            n = m.window_size * m.window_size
            w["fwd_bytes"] += 8 * tc
            w["bwd_bytes"] += 16 * tc
            w["fwd_flops"] += 4 * tc * n
            w["bwd_flops"] += 10 * tc * n
            w["fwd_exp"] += tc * n // 32
            w["bwd_exp"] += 2 * tc * n // 32
            w["windows"].add(m.window_size)
    return w


def stage_breakdown(model, batch, durations_ms, per_elem, backward):
    """Per-stage view of the timed W-MSA launches (libhvk's per-launch dispatch-packet times,
    in launch order): a step launches one per SwinTransformerBlock, forward in block order and
    backward in reverse, so launch i belongs to block i mod (blocks); grouped by the block's
    resolution: mean duration, algorithmic bytes (per_elem * T * C) and rate against 8 TB/s."""
    from hvamd.swinv2 import SwinTransformerBlock
    blocks = [m for m in model.modules() if isinstance(m, SwinTransformerBlock)]
    if not blocks or not durations_ms or len(durations_ms) % len(blocks):
        return None
    order = blocks[::-1] if backward else blocks
    groups = {}
    for i, ms in enumerate(durations_ms):
        m = order[i % len(blocks)]
        key = (tuple(m.input_resolution), m.dim, m.window_size)
        g = groups.setdefault(key, [0.0, 0, per_elem * batch * m.input_resolution[0] * m.input_resolution[1] * m.dim])
        g[0] += ms
        g[1] += 1
    out = []
    for (res, dim, win), (ms, n, nbytes) in sorted(groups.items(), key=lambda kv: -kv[0][0][0]):
        avg = ms / n
        gbs = nbytes / (avg / 1000) / 1e9
        out.append({"resolution": list(res), "dim": dim, "window": win,
                    "launches_per_step": n * len(blocks) // len(durations_ms),
                    "avg_launch_us": round(1000 * avg, 2), "bytes_per_launch": nbytes,
                    "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)})
    return out


def kernel_names(windows):
    # w <= 8: one workgroup per (window, head group) (wmsa_win.hip)
    fwd = sorted({f"wmsa_fwd_win_kernel<{w},HG>" if w <= 8 else f"wmsa_fwd_large_kernel<{w}>" for w in windows})
    bwd = sorted({f"wmsa_bwd_pair_kernel<{w}>" if w <= 8 else f"wmsa_bwd_large_kernel<{w}>" for w in windows})
    return "+".join(fwd), "+".join(bwd)


def roofline_block(kernel, nbytes, flops, ms_total, launches, steps, traffic, n_exp=None):
    """The kernel's achieved HBM rate and MFMA rate against the MI355X peaks; bound = the
    roof its arithmetic intensity sits under (ridge = 2.5 PF / 8 TB/s = 312 flop/B)."""
    sec = ms_total / 1000.0
    gbs = nbytes * steps / sec / 1e9
    tfs = flops * steps / sec / 1e12
    ai = flops / nbytes
    bound = "mfma" if ai > MFMA_PEAK_TFS * 1e3 / HBM_PEAK_GBS else "hbm"
    # achieved / peak / frac against the roof the kernel sits under (w24: MFMA), both kept
    if bound == "mfma":
        head = {"achieved": round(tfs, 1), "peak": MFMA_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(tfs / MFMA_PEAK_TFS, 4)}
    else:
        head = {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4)}
    return {"kernel": kernel, "bound": bound, **head, "traffic": traffic,
            "algorithmic_bytes_per_step": nbytes, "algorithmic_flops_per_step": flops,
            "arith_intensity": round(ai, 1), "achieved_gbs": round(gbs, 1),
            "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), "achieved_tflops": round(tfs, 1),
            "mfma_frac": round(tfs / MFMA_PEAK_TFS, 4),
            "avg_launch_us": round(1000 * ms_total / launches, 2),
            "ms_per_step": round(ms_total / steps, 3),
            # third roof for the large-window kernels, whose softmax is exp-issue heavy
            **({"trans": {"exp_per_step": n_exp, "achieved": round(n_exp * steps / sec / 1e12, 3),
                          "peak": round(EXP_PEAK_TS, 3), "unit": "Texp/s",
                          "frac": round(n_exp * steps / sec / 1e12 / EXP_PEAK_TS, 4)}}
               if n_exp else {})}


def shape_table(launches, steps):
    """Per-shape binding-roof table of the timed GEMM launches: grouped by (kernel, M, N, K);
    roof = max(flops / MFMA peak, algorithmic bytes / HBM peak) per launch, binding_frac =
    roof / measured average.  Also the whole family's binding fraction (sum of roofs / sum of
    times), split into forward / input-gradient (kind 2) and weight-gradient (kind 3)."""
    groups = {}
    for r in launches:
        key = (r["kernel"], r["M"], r["N"], r["K"], r["kind"])
        g = groups.setdefault(key, {"ms": 0.0, "n": 0, "bytes": r["bytes"], "flops": r["flops"]})
        g["ms"] += r["ms"]
        g["n"] += 1
    rows, tot = [], {2: [0.0, 0.0], 3: [0.0, 0.0]}
    for (name, M, N, K, kind), g in groups.items():
        avg_us = 1000.0 * g["ms"] / g["n"]
        t_mfma = g["flops"] / (MFMA_PEAK_TFS * 1e12) * 1e6
        t_hbm = g["bytes"] / (HBM_PEAK_GBS * 1e9) * 1e6
        roof = max(t_mfma, t_hbm)
        tot[kind][0] += roof * g["n"]
        tot[kind][1] += avg_us * g["n"]
        rows.append({"kernel": name, "M": M, "N": N, "K": K, "wgrad": kind == 3,
                     "launches_per_step": round(g["n"] / steps, 2), "avg_us": round(avg_us, 2),
                     "gflop": round(g["flops"] / 1e9, 2), "mbytes": round(g["bytes"] / 1e6, 1),
                     "bound": "mfma" if t_mfma >= t_hbm else "hbm", "roof_us": round(roof, 2),
                     "binding_frac": round(roof / avg_us, 4),
                     "ms_per_step": round(g["ms"] / steps, 4)})
    rows.sort(key=lambda r: -r["ms_per_step"])
    binding = {k: {"roof_ms_per_step": round(v[0] / 1000 / steps, 3), "ms_per_step": round(v[1] / 1000 / steps, 3),
                   "binding_frac": round(v[0] / v[1], 4) if v[1] else None}
               for k, v in (("gemm", tot[2]), ("wgrad", tot[3]))}
    a = tot[2][0] + tot[3][0]
    b = tot[2][1] + tot[3][1]
    binding["all"] = {"binding_frac": round(a / b, 4) if b else None}
    return rows, binding


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args, seconds):
    """The oracle's f32 CPU restatement of the bench's model + loss (SwinV2-T 224 + HXE): train
    steps (forward + loss + backward) at batch 32 for ~`seconds`, then ONE step at the GPU's
    batch 256 (BASELINE.md plan).  Threads: every CPU in this process's affinity set, capped by
    OMP_NUM_THREADS when the host sets it (the GPU box grants each GPU a 16-CPU share)."""
    from hvamd.hierarchy import Taxonomy
    from oracle import hierarchy_ref, swinv2_ref

    affinity = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else affinity
    torch.set_num_threads(threads)
    cfg = dict(img_size=224, embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24),
               window_size=7)
    tax = Taxonomy.synthetic()
    p = swinv2_ref.init_params_from_rng(swinv2_ref.state_shapes(num_classes=tax.num_leaves, **cfg), 0)
    for v in p.values():
        v.requires_grad_(True)
    geom = swinv2_ref.model_geometry(**cfg)
    lam = hierarchy_ref.hxe_level_weights("exponential", 0.1)
    rng = np.random.default_rng(0)

    def step(bs):
        x = torch.randn(bs, 3, 224, 224)
        paths = tax.leaf_paths[rng.integers(0, tax.num_leaves, bs)]
        t0 = time.perf_counter()
        logits = swinv2_ref.forward(p, x, geom)
        loss = hierarchy_ref.hxe_loss_torch(logits, paths, tax.perm, tax.node_start, tax.node_end,
                                            tax.tier_base, lam)
        loss.backward()
        for v in p.values():
            v.grad = None
        return time.perf_counter() - t0

    step(32)  # warm-up
    n, el = 0, 0.0
    while el < seconds and n < 50:
        el += step(32)
        n += 1
    t256 = step(256)
    return {"value": round(32 * n / el, 3), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"{n} train steps x 32 images (SwinV2-T 224 + HXE, f32, oracle/swinv2_ref.py); "
                      f"one step x 256 images: {256 / t256:.3f} images/sec",
            "bs256_images_per_sec": round(256 / t256, 3), "cpu_model": cpu_model(),
            "affinity_cpus": affinity}


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
    from hvamd import _lib, options
    for o in args.opt:
        name, _, val = o.partition("=")
        _lib.set_option(name, int(val))
    for o in args.host_opt:
        options.set(**options.parse(o))
    if args.stream_priority:
        # the whole run on a stream of this priority (negative = higher), the parameter-gradient
        # side stream staying at the default: the input-gradient chain dispatches first
        torch.cuda.set_stream(torch.cuda.Stream(device=device, priority=args.stream_priority))

    cfg, tax, model, trainer = build(args, device)
    if args.steps_in_flight >= 0:
        trainer.max_steps_in_flight = args.steps_in_flight or None
    img = model.module.patch_embed.img_size[0]
    batch = synthetic_batch(args, tax, rank, device, img)

    work = wmsa_work(model.module, args.batch)
    timing = not args.no_roofline
    timer, timed_steps, launches = None, args.steps, None
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
            launches = {k: ops.kernel_timer_launches(k) for k in (0, 1)}
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
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fallbacks = ops.library_fallbacks(reset=True)  # warm-up + timed steps
    # caching-allocator health over the warm-up + timed steps: a step that needs more than the
    # card holds makes the allocator free its cache and retry (a device-wide sync per retry)
    ms = torch.cuda.memory_stats(device)
    memory = {"peak_reserved_gib": round(torch.cuda.max_memory_reserved(device) / 2**30, 1),
              "peak_allocated_gib": round(torch.cuda.max_memory_allocated(device) / 2**30, 1),
              "alloc_retries": int(ms.get("num_alloc_retries", 0)), "device_allocs": int(ms.get("num_device_alloc", 0)),
              "device_frees": int(ms.get("num_device_free", 0))}
    comm = None
    if world > 1 and not args.graph and args.comm_steps > 0:
        # the exchange's exposed time and each bucket's overlap window, on extra steps after the
        # timed region (Trainer.comm_timing: marks at the backward's start / end, each all-reduce
        # enqueue, and after buckets.synchronize())
        from hvamd.trainer import comm_report
        trainer.comm_timing = []
        for _ in range(args.comm_steps):
            step()
        comm = comm_report(trainer.comm_timing)
        trainer.comm_timing = None
        t = torch.tensor([comm["exposed_ms"], comm["exposed_ms_max"]], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        comm["exposed_ms_max_over_ranks"] = round(t[0].item(), 3)
    gemm_timer, gemm_steps, gemm_shapes = None, 0, None
    if timing and not args.graph:
        # the kernel timers run over extra steps after the timed region, so `value` is a clean
        # wall time: W-MSA launches timed by their own dispatch packets, then the GEMMs (their
        # ~250 launches per step perturb the step by ~4 %)
        timed_steps = min(args.steps, 10)
        ops.kernel_timer_start(kinds=ops.TIMER_WMSA)
        # with the parameter-gradient side stream off, as the GEMM table below: a W-MSA backward
        # launch sharing its CUs with a side-stream weight gradient reads 10-20 % longer without
        # costing the step that much; this is the kernel's own time, as the serial rocprof summary
        with options.override(wgrad_stream=False):
            for _ in range(timed_steps):
                step()
        torch.cuda.synchronize()
        launches = {k: ops.kernel_timer_launches(k) for k in (0, 1)}
        timer = ops.kernel_timer_stop()
        gemm_steps = min(args.steps, 5)
        ops.kernel_timer_start(kinds=ops.TIMER_GEMM)
        # the per-shape GEMM table prices each launch against its own roof: these steps run the
        # parameter gradients on the main stream (options.wgrad_stream off), since a launch that
        # shares the CUs with the side stream's takes longer without costing the step that much
        with options.override(wgrad_stream=False):
            for _ in range(gemm_steps):
                step()
        torch.cuda.synchronize()
        gemm_shapes = ops.kernel_timer_shapes()
        gemm_timer = ops.kernel_timer_stop()
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_val = float(loss)
    if not np.isfinite(loss_val):
        raise RuntimeError(f"non-finite loss {loss_val}")
    images = world * args.batch * args.steps
    value = images / elapsed
    default_cfg = args.model == "swinv2_tiny_window7_224" and args.loss == "hxe"
    workload = {"swinv2_tiny_window7_224": "SwinV2-T 224 w7", "swinv2_base_window7_224": "SwinV2-B 224 w7",
                "swinv2_base_window24_384": "SwinV2-B 384 w24 (pretrained windows 12/12/12/6)"}.get(
                    args.model, args.model)
    workload += {"hxe": " + HXE (10000 leaves, 7 tiers)", "multitask": " + 7-tier multitask heads",
                 "ce": " + flat 1000-class CE"}[args.loss] + " train step"
    macs = model.module.flops()  # MACs per image, swinv2.py:847-867 accounting
    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (randn images resident in HBM, leaves uniform over a synthetic 10k-leaf "
                "7-tier tree); random-init weights",
        "config": {"workload": workload, "model": args.model, "loss": args.loss,
                   "global_batch": world * args.batch, "per_gpu_batch": args.batch, "image_size": img,
                   "parallelism": f"dp{world}",
                   "execution": "hip-graph replay" if args.graph else "eager"},
        "value_per_gpu": round(value / world, 2),
        "comm": ({"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                  "grad_buckets": len(trainer.buckets.buckets),
                  "grad_bytes_per_step": 4 * sum(b[0].numel() for b in trainer.buckets.buckets),
                  "bucket_mb": [round(b[0].numel() * 4 / 2**20, 1) for b in trainer.buckets.buckets],
                  "wgrad_side_stream": bool(options.OPTIONS.wgrad_stream and options.OPTIONS.wgrad_stream_multi_rank),
                  **(comm or {})}
                 if world > 1 else None),
        "final_loss": round(loss_val, 4),
        # launches that left libhvk for a torch / hipBLASLt op over the warm-up + timed steps
        "library_fallbacks": {"steps": args.warmup + args.steps, "sites": fallbacks},
        "memory": memory,
        # every routing switch the run used: host (hvamd.options) and library (hvk_set_option)
        "options": {"host": options.as_dict(), "lib": _lib.options()},
        # whole-step MFMA utilisation: 3 x 2 x MACs per image (forward + both backward GEMMs)
        "step_mfma": {"flops_per_step": 6 * macs * args.batch,
                      "achieved_tflops": round(6 * macs * args.batch * args.steps / elapsed / 1e12, 1),
                      "peak": MFMA_PEAK_TFS,
                      "frac": round(6 * macs * args.batch * args.steps / elapsed / 1e12 / MFMA_PEAK_TFS, 4)},
    }
    if timer:
        kf, kb = kernel_names(work["windows"])
        fw_ms, fw_n, _ = timer["wmsa_fwd"]
        bw_ms, bw_n, _ = timer["wmsa_bwd"]
        n_launch = fw_n // timed_steps
        traffic = measured_traffic("wmsa_fwd") if default_cfg else None
        large = max(work["windows"]) > 8
        r = roofline_block(f"{kf} (all {n_launch} launches per step)", work["fwd_bytes"],
                           work["fwd_flops"], fw_ms, fw_n, timed_steps, traffic,
                           work["fwd_exp"] if large else None)
        r["timing"] = ("dispatch-packet events (hipExtLaunchKernelGGL) over %d eager steps just "
                       "before the graph capture (replays carry no per-kernel events)" % timed_steps
                       if args.graph else
                       "dispatch-packet events (hipExtLaunchKernelGGL) over %d eager steps after the "
                       "timed region, parameter-gradient side stream off" % timed_steps)
        if traffic is not None:
            r["algorithmic_bytes_per_launch"] = work["fwd_bytes"] // n_launch
            r["traffic_fetch_x1_5"] = measured_traffic("wmsa_fwd", 1.5)
            r["traffic_source"] = TRAFFIC_SOURCE
        if launches:
            r["stages"] = stage_breakdown(model.module, args.batch, launches[0], 8, False)
        result["roofline"] = r
        result["roofline_bwd"] = roofline_block(
            kb, work["bwd_bytes"], work["bwd_flops"], bw_ms, bw_n, timed_steps,
            measured_traffic("wmsa_bwd") if default_cfg else None, work["bwd_exp"] if large else None)
        if launches:
            result["roofline_bwd"]["stages"] = stage_breakdown(model.module, args.batch, launches[1], 16, True)
        if default_cfg and measured_traffic("wmsa_bwd") is not None:
            result["roofline_bwd"]["traffic_fetch_x1_5"] = measured_traffic("wmsa_bwd", 1.5)
        if not large:
            # SURVEY.md §8(d) counts 16 T C backward bytes, an O read included; the w <= 8 backward
            # recomputes delta = rowsum(P dP) and never reads O, so the bytes it must move are
            # 14 T C (q, k, v, dO in; dq, dk, dv out): its rate against those, for the record
            rb = result["roofline_bwd"]
            moved = work["bwd_bytes"] * 14 // 16
            gbs = moved * timed_steps / (bw_ms / 1000) / 1e9
            rb["bytes_moved_per_step"] = moved
            rb["moved_gbs"] = round(gbs, 1)
            rb["moved_frac"] = round(gbs / HBM_PEAK_GBS, 4)
        # dense contractions on libhvk's MFMA GEMMs (every Linear but the classifier head):
        # their algorithmic flops (2 M N K per launch, summed by the library) over their
        # dispatch-packet-timed durations
        mf = {}
        gt, gsteps = (gemm_timer, gemm_steps) if gemm_timer else (timer, timed_steps)
        for kind, label in (("gemm", "linear_kernel + gemm_nt_kernel (forward, input grads)"),
                            ("wgrad", "dw_kernel (weight grads)")):
            ms, n, fl = gt[kind]
            if n:
                mf[kind] = {"kernels": label, "launches_per_step": n // gsteps,
                            "ms_per_step": round(ms / gsteps, 3),
                            "achieved_tflops": round(fl / (ms / 1000) / 1e12, 1),
                            "frac": round(fl / (ms / 1000) / 1e12 / MFMA_PEAK_TFS, 4)}
        tot_ms = sum(gt[k][0] for k in ("gemm", "wgrad"))
        tot_fl = sum(gt[k][2] for k in ("gemm", "wgrad"))
        if tot_ms > 0:
            mf.update({"bound": "mfma", "achieved": round(tot_fl / (tot_ms / 1000) / 1e12, 1),
                       "peak": MFMA_PEAK_TFS, "unit": "TFLOP/s",
                       "frac": round(tot_fl / (tot_ms / 1000) / 1e12 / MFMA_PEAK_TFS, 4),
                       "flops_per_step": tot_fl / gsteps,
                       "ms_per_step": round(tot_ms / gsteps, 3),
                       "timing": ("dispatch-packet events over %d eager steps after the timed region"
                                  % gsteps if gemm_timer else
                                  "dispatch-packet events over the pre-capture eager steps")})
        if gemm_shapes:
            mf["shapes"], mf["binding"] = shape_table(gemm_shapes, gemm_steps)
        result["mfma"] = mf
    if rank == 0 and world == 1 and args.cpu_baseline and default_cfg:
        result["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
