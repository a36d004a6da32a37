"""How long the host takes to enqueue one bench step (Python + autograd + ctypes launches), against
the step's GPU time: the GPU is first held busy by a long torch.cuda._sleep so that every launch
of the measured steps is enqueued without waiting for the device, then the enqueue time per step
is read off the host clock.  An enqueue time close to the step time means the eager step is
host-bound (the device idles between launches).

    python tools/host_overhead.py [--steps 2] [--host-opt NAME=VALUE ...]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--host-opt", action="append", default=[])
    a = ap.parse_args()
    import bench
    from hvamd import options
    for o in a.host_opt:
        options.set(**options.parse(o))

    class A:  # bench.build's argument surface
        model, loss, batch = "swinv2_tiny_window7_224", "hxe", 256
    dev = torch.device("cuda", 0)
    cfg, tax, model, trainer = bench.build(A, dev)
    batch = bench.synthetic_batch(A, tax, 0, dev)
    for _ in range(4):
        trainer.train_step(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        trainer.train_step(batch)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / 5 * 1000
    res = []
    for _ in range(3):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2.4e9))  # ~1 s of device time: the queue holds every launch below
        t0 = time.perf_counter()
        for _ in range(a.steps):
            trainer.train_step(batch)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        res.append((t1 - t0) / a.steps * 1000)
    print(f"step {step_ms:.2f} ms (device-bound wall); host enqueue per step {min(res):.2f} ms "
          f"(runs {', '.join(f'{r:.2f}' for r in res)})", flush=True)


if __name__ == "__main__":
    main()
