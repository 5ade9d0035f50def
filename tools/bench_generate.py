"""BASELINE config 5: generate_fromS.py video sweep at FFHQ-1024 (change_power 0 -> 50, 64 frames) on one GPU.

    python tools/bench_generate.py [--frames 64] [--batch 8] [--check 4]
Times render_sweep (the --from_video path of stylemc_amd/generate_fromS.py: S row + direction * power, batched
synthesis, uint8 HWC frames) with the frames resident in HBM (the JPEG/npy writing of the CLI is host I/O and not
timed), then checks `--check` evenly spaced frames against the CPU oracle (oracle/generate_fromS.py, pinned to the
reference's synthesis by tests/golden): |diff| <= 1 per pixel and >= 99.9 % exact (the GPU test's tolerance).
Synthetic seeded config-f weights (no checkpoint offline).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--check", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from stylemc_amd import build, generate_fromS, networks, synthetic, utils
    build.build(verbose=False)
    dev = "cuda"
    cfg = synthetic.generator_config(resolution=1024, channel_base=32768)
    sd = synthetic.generator_state_dict(cfg, seed=0)
    G = networks.build_generator(cfg, sd, device=dev)
    shapes = utils.get_temp_shapes(G)
    style_row = synthetic.synthetic_styles(1, seed=3)[0]
    direction = torch.zeros(1, 26, 512)
    direction[:, utils.S_TRAINABLE_SPACE_CHANNELS] = torch.randn(
        1, 8, 512, generator=torch.Generator().manual_seed(2)) * 0.1
    powers = np.linspace(0.0, 50.0, args.frames)
    sr, dr = style_row.to(dev), direction.to(dev)
    frames = generate_fromS.render_sweep(G, sr, dr, powers, shapes, batch=args.batch)  # warm-up
    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        frames = generate_fromS.render_sweep(G, sr, dr, powers, shapes, batch=args.batch)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    dt = min(times)
    # parity on a subset of the frames against the CPU oracle
    from oracle import generate_fromS as OG
    from oracle import networks as ON
    from oracle import synthesis as OS
    Go = ON.Generator(512, 0, 512, 1024, 3, channel_base=32768, conv_clamp=cfg["conv_clamp"])
    Go.load_state_dict(sd, strict=False)
    Go.eval().requires_grad_(False)
    idx = np.linspace(0, args.frames - 1, args.check).round().astype(int)
    ref = OG.render_sweep(Go, style_row, direction, powers[idx], OS.get_temp_shapes(Go))
    got = frames[torch.as_tensor(idx, device=dev)].cpu().numpy().astype(np.int16)
    diff = np.abs(got - ref.numpy().astype(np.int16))
    out = {"workload": "generate_fromS --from_video sweep, FFHQ-1024 (config-f, seeded weights), "
                       f"change_power 0 -> 50, {args.frames} frames, batch {args.batch}",
           "frames_per_s": round(args.frames / dt, 2), "seconds": round(dt, 4), "reps": args.reps,
           "parity": {"frames_checked": idx.tolist(), "max_abs_diff_u8": int(diff.max()),
                      "exact_fraction": round(float((diff == 0).mean()), 6),
                      "tolerance": "|diff| <= 1, >= 99.9 % exact (uint8 HWC, vs oracle/ CPU fp32)",
                      "pass": bool(diff.max() <= 1 and (diff == 0).mean() >= 0.999)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
