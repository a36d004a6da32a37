"""Which PyTorch ops still launch kernels inside the training step: torch.profiler over a few
steps of the bench configuration, aten ops grouped by call stack.
    python tools/torch_prof.py [--steps 3] [--pattern 'copy|fill|add|to|cat|zeros']"""
import argparse
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pattern", default=r"^aten::(copy_|fill_|add|cat|zero|_to_copy|mul|sum|mean|layer_norm|clone|exp|clamp|addmm|mm|matmul|to)")
    a = ap.parse_args()
    import bench
    device = torch.device("cuda", 0)
    ns = argparse.Namespace(model="swinv2_tiny_window7_224", loss="hxe", batch=256)
    cfg, tax, model, trainer = bench.build(ns, device)
    batch = bench.synthetic_batch(ns, tax, 0, device, 224)
    for _ in range(3):
        trainer.train_step(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(a.steps):
            trainer.train_step(batch)
        torch.cuda.synchronize()
    pat = re.compile(a.pattern)
    rows = prof.key_averages(group_by_input_shape=True)
    rows = [r for r in rows if pat.search(r.key) and r.device_time_total > 0]
    rows.sort(key=lambda r: -r.device_time_total)
    for r in rows[:40]:
        print(f"{r.device_time_total / a.steps:9.1f} us/step  {r.count / a.steps:5.1f}x  {r.key[:60]}  "
              f"{str(r.input_shapes)[:150]}")


if __name__ == "__main__":
    main()
