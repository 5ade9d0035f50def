#!/usr/bin/env python
"""find_direction throughput on MI355X (BASELINE.json metric), one JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

With no launcher in the environment (no WORLD_SIZE), ``--gpus N > 1`` starts the N rank processes itself
(spawn_ranks: fresh processes, before any GPU call here).  Under a launcher, a WORLD_SIZE that differs from
--gpus exits with status 2.  One-GPU rehearsal of the N-rank path: SMC_SHARE_GPU=1 SMC_DIST_BACKEND=gloo
(every rank on device 0; RCCL refuses two ranks on one GPU) -- the line then says ranks_share_gpu, and its
throughput is not a scaling number.

A step = one find_direction iteration (find_direction.py:292-347) on synthetic inputs that are
resident in HBM before timing: a config-f FFHQ-1024 generator with seeded weights, S codes
[129, 26, 512] ~ N(1, 0.5), seeded CLIP ViT-B/32 + IR-SE50, --clip_type small, landmarks 0.
Each GPU processes a batch of 4 seeds per step (weak scaling: global batch = 4 x N over 129 x N S codes,
so every GPU runs the single-GPU 129-seed batch schedule; one RCCL all_reduce of the direction gradient
per step).  value = images/s = 2 x seeds/s (edited + original
image per seed), seeds counted exactly (the batch picker can draw the short
last batch of the 129 seeds).

roofline: the dominant kernel family, the synthesis convs (every smc_conv3x3_wino_f32 / smc_conv_gemm_f32 launch
from modconv.py: ``wino4_kernel`` / ``wino_kernel`` for the 3x3 'same' convs, ``conv_gemm_lds_kernel`` / ``conv_row_kernel`` /
``convt_lds_kernel`` ... for the rest): the MFMA FLOPs of each launch's algorithm (dense MACs x 2 for the direct
kernels; 16 / 36 multiplies per 2x2 / 4x4 tile and channel pair for Winograd F(2x2) / F(4x4),
reported beside the
direct-equivalent rate) / its duration, timed with HIP events around every launch during --roofline-steps extra steps run right
after the timed region with the original-image branch serialised onto the main stream (in the timed
region that branch runs on a second stream, and a launch's event interval would include CU time
taken by the other stream's kernels), against the fp32 MFMA peak (157.3 TFLOP/s,
MI355X_MICROARCH.md).  traffic: HBM bytes per launch from the rocprofv3 PMC pass recorded in
profiles/pmc_traffic.json (null if absent).

cpu_baseline (rank 0, N=1): the test oracle (pure-torch fp32 CPU restatement of the reference loop,
oracle/, pinned to the reference by tests/golden) running the same step at FFHQ-1024, batch 4: 1 warm-up +
3 timed iterations on the host's CPU share (affinity set capped by the cgroup quota; os.cpu_count() and the
CPU model are reported beside it).  parity (same run): the GPU path repeats that exact oracle run and
reports the cosine similarity of the two final directions (the metric's "dir cosine-sim vs ref").  N > 1:
parity = the N-rank direction vs rank 0 re-running the same global batch in one process.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3
# the split-bf16 direct convs run every fp32 product as six bf16 MFMA products: their roof is the dense bf16 MFMA
# peak (256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz) / 6, in fp32-equivalent FLOP/s
BF16_MFMA_PEAK_TFLOPS = 2516.6
X3_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6


def kind_peak(kind):
    return X3_PEAK_TFLOPS if kind.endswith("_x3") else FP32_MFMA_PEAK_TFLOPS
METRIC = "find_direction images/sec @ FFHQ-1024 bs=4, 1/2/4/8 GPU; dir cosine-sim vs ref"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--resolution", type=int, default=1024)
    p.add_argument("--batch", type=int, default=4, help="seeds per GPU per step")
    p.add_argument("--n-seeds", type=int, default=None,
                   help="S codes in the run (default 129 per GPU: weak scaling keeps each GPU's batch schedule "
                        "identical to the single-GPU 129-seed run, short last batch included)")
    p.add_argument("--clip-type", default="small")
    p.add_argument("--clip-impl", default="hip", choices=["hip", "torch"],
                   help="hip: ViT on the gfx950 kernel library (config 4); torch: PyTorch-ROCm ops (config 2)")
    p.add_argument("--id-impl", default="hip", choices=["hip", "torch"],
                   help="hip: IR-SE50 on the gfx950 kernel library (config 4); torch: PyTorch-ROCm/MIOpen (config 2)")
    p.add_argument("--cpu-iters", type=int, default=4, help="CPU baseline / parity iterations (first = warm-up)")
    p.add_argument("--cpu-batch", type=int, default=4)
    p.add_argument("--cpu-threads", type=int, default=0, help="0: the host's CPU share (affinity, cgroup quota)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-timer", action="store_true", help="skip the roofline pass")
    p.add_argument("--roofline-steps", type=int, default=2, help="serialised steps timed per launch for the roofline")
    p.add_argument("--no-batch-losses", action="store_true",
                   help="run the original image's loss-network forwards separately (on the side stream)")
    p.add_argument("--conv-products", default="x3", choices=["x3", "fp32"],
                   help="direct implicit-GEMM convs: x3 = fp32 products as three-term bf16 splits (six bf16 MFMAs, "
                        "fp32-class error), fp32 = the exact-fp32 MFMA (modconv.X3)")
    p.add_argument("--vit-products", default="fp32", choices=["x3", "fp32"],
                   help="CLIP ViT projections: split-bf16 (x3) or exact-fp32 MFMA GEMMs (vit_hip.X3)")
    p.add_argument("--irse-products", default=None, choices=["x3", "fp32"],
                   help="IR-SE50 executor GEMMs: split-bf16 or exact-fp32 (irse_hip.X3; default: the library's)")
    p.add_argument("--prefetch-id", default=None, choices=["on", "off"],
                   help="the original image's IR-SE50 features on the prefetch stream (default: DirectionFinder's)")
    p.add_argument("--schedule", default="prefetch", choices=["pair", "prefetch"],
                   help="stream schedule: pair = original synthesis beside the edited one; prefetch = the next "
                        "iteration's original synthesis on a third stream (DESIGN.md section 6b)")
    return p.parse_args()


def host_cpus():
    """Threads the CPU baseline may use on this host, and how that was decided: the scheduler affinity set,
    capped by the cgroup CPU quota (a GPU box shares a large machine; os.cpu_count() reports all of it)."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    info["affinity"] = aff
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    info["cgroup_quota_cpus"] = quota
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    info["model"] = model
    threads = min(aff, quota) if quota else aff
    return max(1, threads), info


def _oracle_problem(resolution):
    from oracle import losses as OL
    from oracle import networks as ON
    from oracle import synthesis as OS
    from stylemc_amd import synthetic
    cfg = synthetic.generator_config(resolution=resolution)
    sd = synthetic.generator_state_dict(cfg, seed=0)
    G = torch.nn.Module()
    G.synthesis = ON.SynthesisNetwork(512, resolution, 3, channel_base=cfg["channel_base"], conv_clamp=256.0)
    G.synthesis.load_state_dict({k[10:]: v for k, v in sd.items() if k.startswith("synthesis.")}, strict=False)
    G.eval().requires_grad_(False)
    vis = OL.CLIPVisual().eval()
    vis.load_state_dict(synthetic.seeded_state_dict(vis, seed=4))
    vis.requires_grad_(False)
    clip = OL.CLIPLoss(vis, synthetic.text_direction(*TEXT))
    net = OL.IRSE50().eval()
    net.load_state_dict(synthetic.seeded_state_dict(net, seed=3))
    net.requires_grad_(False)
    return G, OS.get_temp_shapes(G), clip, OL.IDLoss(net)


# the CPU baseline / parity problem: PARITY_ITEMS S codes, batch 4, PARITY_ITERS iterations (the first is
# the CPU baseline's warm-up), 2 epochs so the cosine schedule covers them
PARITY_ITEMS, PARITY_EPOCHS = 8, 2
TEXT = ("a photo of a face of a feminine woman with no makeup", "a photo of a face of a masculine man")


def cpu_baseline(resolution, batch, iters, threads, cpu_info):
    """Oracle find_direction on the host (TEST ORACLE used as the baseline): `iters` iterations at `batch`,
    the first one untimed (warm-up)."""
    from oracle import find_direction as OF
    from stylemc_amd import synthetic
    from stylemc_amd.find_direction import initial_delta
    torch.set_num_threads(threads)
    G, shapes, clip, idl = _oracle_problem(resolution)
    styles = synthetic.synthetic_styles(PARITY_ITEMS, seed=0)
    log = []
    t0 = time.perf_counter()
    _, delta = OF.find_direction(G, styles, clip, idl, shapes, int(resolution).bit_length() - 3, batch_size=batch,
                                 n_epochs=PARITY_EPOCHS, max_iterations=iters, init_delta=initial_delta(0, 0.01),
                                 log=log)
    stamps = [t0] + [l["t"] for l in log]
    dt = stamps[-1] - stamps[1]
    seeds = sum(min(batch, PARITY_ITEMS - l["batch"] * batch) for l in log[1:])
    return {"value": 2 * seeds / dt, "unit": "images/s", "cores": threads, "kind": "port",
            "cpu": cpu_info,
            "sample": f"{iters - 1} timed find_direction iterations after 1 warm-up, batch {batch} "
                      f"({seeds} seed-steps, FFHQ-{resolution}, CLIP ViT-B/32 + IR-SE50) in {dt:.1f} s: oracle/ "
                      f"pure-torch fp32 CPU restatement of the reference loop, {threads} threads"}, delta.detach()


def direction_parity(G, clip, id_loss, resolution, batch, iters, delta_ref, dev, temp_shapes):
    """The metric's 'dir cosine-sim vs ref': the GPU DirectionFinder run on the cpu_baseline's exact
    problem (same seeded weights, S codes, batch, batch picks and start point); final directions compared."""
    from stylemc_amd import synthetic
    from stylemc_amd.find_direction import DirectionFinder, initial_delta
    styles = synthetic.synthetic_styles(PARITY_ITEMS, seed=0).to(dev)
    init = initial_delta(0, 0.01)
    f = DirectionFinder(G, styles, clip, id_loss, resolution=resolution, batch_size=batch, n_epochs=PARITY_EPOCHS,
                        seed=0, init_delta=init, temp_shapes=temp_shapes)
    for _ in range(iters):
        f.step()
    g = f.delta.detach().cpu().double().flatten()
    r = delta_ref.double().flatten()
    cos = torch.nn.functional.cosine_similarity(g, r, dim=0).item()
    i0 = init.double().flatten()
    ucos = torch.nn.functional.cosine_similarity(g - i0, r - i0, dim=0).item()
    err = ((g - r).abs().max() / r.abs().max()).item()
    return {"dir_cosine_vs_oracle": round(cos, 7), "update_cosine_vs_oracle": round(ucos, 7),
            "dir_max_rel_err": float(f"{err:.3e}"), "iters": iters, "batch": batch, "target": ">= 0.999",
            "what": f"final [1,8,512] direction after {iters} find_direction iterations at FFHQ-{resolution}, "
                    f"batch {batch}: HIP path vs oracle/ (fp32 CPU restatement of the reference loop, pinned to "
                    f"the reference by tests/golden) on identical inputs"}


def dist_selfcheck(G, clip, id_loss, world, dev, temp_shapes, resolution, batch, steps=2):
    """N > 1: the N-rank direction after `steps` steps on one global batch vs rank 0 re-running the same global
    batch in a single process.  Kernel plans are made for the global batch on every rank (plan_batch) and the
    per-image rows are summed in one fixed order, so the two are expected bit-equal (dir_equal_1rank) -- except where
    the single-process batch crosses a shape limit the shards do not (inputs >= 2 GiB take the register-staged
    kernels: batch 32 at r = 1024)."""
    from stylemc_amd import dist as sdist
    from stylemc_amd import synthetic
    from stylemc_amd.find_direction import DirectionFinder, initial_delta
    B = batch * world.world_size
    styles = synthetic.synthetic_styles(B, seed=17).to(dev)
    init = initial_delta(1, 0.01)
    kw = dict(resolution=resolution, batch_size=B, global_batch=B, n_epochs=4, seed=0, init_delta=init,
              temp_shapes=temp_shapes)
    f = DirectionFinder(G, styles, clip, id_loss, world=world, **kw)
    for _ in range(steps):
        f.step()
    d_n = f.delta.detach().cpu().double().flatten()
    out = None
    if world.rank == 0:
        f1 = DirectionFinder(G, styles, clip, id_loss, world=sdist.World(), **kw)
        for _ in range(steps):
            f1.step()
        d_1 = f1.delta.detach().cpu().double().flatten()
        i0 = init.double().flatten()
        out = {"dir_equal_1rank": bool(torch.equal(d_n, d_1)),
               "dir_max_abs_diff_vs_1rank": float((d_n - d_1).abs().max()),
               "dir_cosine_vs_1rank": round(torch.nn.functional.cosine_similarity(d_n, d_1, dim=0).item(), 7),
               "update_cosine_vs_1rank": round(torch.nn.functional.cosine_similarity(d_n - i0, d_1 - i0, dim=0).item(), 7),
               "steps": steps, "global_batch": B, "backend": world.backend,
               "world_size": torch.distributed.get_world_size()}
    world.barrier()
    return out


def pmc_traffic():
    """(bytes per conv-family launch, where the number comes from): PMC counters need their own rocprofv3 passes
    (tools/pmc_bench.sh), so the bench line carries the last recorded passes' figure and says which."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    src = (f"profiles/pmc_traffic.json ({d.get('recorded', 'r02 v13')}): {d.get('method', 'rocprofv3 PMC passes')}; "
           f"not measured in this run")
    return d.get("conv_gemm_bytes_per_launch"), src


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`python bench.py --gpus N` with no launcher in the environment: start N fresh rank processes of this same
    command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would) and return the first
    non-zero exit status, else 0.  Runs before this process makes any GPU call (torch.cuda.device_count() does
    not initialise the GPU on this image), so the children are started from a GPU-free parent.  A rank that
    fails ends the others (their exact PIDs), so a dead rank cannot leave its peers waiting in a collective."""
    import subprocess
    visible = torch.cuda.device_count()
    share = os.environ.get("SMC_SHARE_GPU") == "1"
    if visible < n and not share:
        print(f"bench.py: --gpus {n} but {visible} GPU(s) visible; set SMC_SHARE_GPU=1 SMC_DIST_BACKEND=gloo for a "
              f"one-GPU rehearsal", file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SMC_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return status


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus {args.gpus}",
                  file=sys.stderr)
            sys.exit(2)
    elif args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.launch_probe:   # launcher test (tests/test_bench_launcher_cpu.py): report the rank environment, no GPU
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "SMC_BENCH_LAUNCHER")
        print(json.dumps({k: os.environ.get(k) for k in keys}), flush=True)
        sys.exit(int(os.environ.get("SMC_PROBE_FAIL_RANK", "-1")) == int(os.environ.get("RANK", "0")) and 3 or 0)
    from stylemc_amd import _hip, build
    from stylemc_amd import dist as sdist
    world = sdist.init_from_env(use_cuda=True)
    dev = torch.device("cuda", world.device_index)
    torch.cuda.set_device(dev)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    if world.rank == 0:
        build.build(verbose=False)
    world.barrier()
    _hip.load()

    from stylemc_amd.find_direction import DirectionFinder, build_clip_losses, initial_delta, load_generator
    from stylemc_amd.id_loss import IDLoss
    from stylemc_amd import modconv, synthetic
    modconv.X3 = args.conv_products == "x3"
    from stylemc_amd import vit_hip
    vit_hip.X3 = args.vit_products == "x3"
    from stylemc_amd import irse_hip
    if args.irse_products is not None:
        irse_hip.X3 = args.irse_products == "x3"

    G = load_generator("synthetic", args.resolution, dev)
    # weak scaling: 129 seeds per GPU and a global batch of 4 per GPU give every N the single-GPU schedule
    # (33 batch indices, the last batch 1 seed per GPU); a fixed 129 seeds at N = 8 would make one draw in
    # five a 1-seed global batch that leaves 7 of 8 GPUs idle for that step
    n_seeds = args.n_seeds if args.n_seeds is not None else 129 * world.world_size
    styles = synthetic.synthetic_styles(n_seeds, seed=0).to(dev)
    clip = build_clip_losses(args.clip_type, dev, *TEXT, impl=args.clip_impl, synthetic_weights=True)
    finder = DirectionFinder(G, styles, clip, IDLoss("a", device=dev, weights=None, impl=args.id_impl), resolution=args.resolution,
                             batch_size=args.batch, global_batch=args.batch * world.world_size, seed=0, world=world,
                             init_delta=initial_delta(0, 0.01), n_epochs=1000,
                             batch_losses=not args.no_batch_losses, prefetch_orig=args.schedule != "pair",
                             **({} if args.prefetch_id is None else {"prefetch_id": args.prefetch_id == "on"}))
    for _ in range(args.warmup):
        finder.step()
    torch.cuda.synchronize()
    world.barrier()

    # timed region: throughput (no per-launch events in it)
    seeds = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = finder.step()
        lo = last["batch"] * finder.B
        seeds += min(lo + finder.B, finder.n_items) - lo
    torch.cuda.synchronize()
    world.barrier()
    dt = time.perf_counter() - t0
    dt = world.all_max(dt, dev)
    finite = bool(torch.isfinite(finder.delta).all().item())

    # roofline pass: the same step with the original-image branch serialised onto the main stream, so
    # each GEMM launch's HIP-event duration is its own execution time (with the side stream running
    # concurrently the events would also count CU time taken by the other stream's kernels; rocprofv3's
    # kernel trace, profiles/, measures the serialised duration too)
    roofline = None
    if not args.no_kernel_timer and args.roofline_steps > 0:
        timer = _hip.KernelTimer("conv_gemm")
        finder.overlap = False
        _hip.set_timer(timer)
        t1 = time.perf_counter()
        for _ in range(args.roofline_steps):
            finder.step()
        torch.cuda.synchronize()
        dt_r = time.perf_counter() - t1
        _hip.set_timer(None)
        finder.overlap = True
        s = timer.summary()
        achieved = s["flops"] / s["seconds"] / 1e12 if s["seconds"] > 0 else 0.0
        # the family's roof: every launch at its instruction's peak (fp32 MFMA, or bf16 MFMA / 6 for the split
        # products); frac = that ideal time / the measured time, peak = the FLOP-weighted blend of the roofs
        ideal = sum(d["flops"] / (kind_peak(k) * 1e12) for k, d in s["kinds"].items())
        peak_blend = s["flops"] / ideal / 1e12 if ideal > 0 else FP32_MFMA_PEAK_TFLOPS

        def part(d, what, kind):
            tf = d["flops"] / d["seconds"] / 1e12 if d["seconds"] > 0 else 0.0
            return {"what": what, "launches": d["launches"], "ms_per_step": round(1e3 * d["seconds"] / args.roofline_steps, 3),
                    "avg_launch_us": round(1e6 * d["seconds"] / max(d["launches"], 1), 2),
                    "achieved": round(tf, 3), "peak": round(kind_peak(kind), 1), "frac": round(tf / kind_peak(kind), 4),
                    "frac_of_fp32_peak": round(tf / FP32_MFMA_PEAK_TFLOPS, 4),
                    "direct_equiv_tflops": round(d["equiv_flops"] / d["seconds"] / 1e12, 3) if d["seconds"] > 0 else 0.0}

        kinds = {
            "wino": ("Winograd F(2x2,3x3) 3x3 'same' convs with a 32/64-channel input (conv1 fwd + data grad at "
                     "r = 32, 512, 1024); FLOPs = its 16 multiplies per 2x2 tile and channel pair (4/9 of the direct "
                     "conv's)"),
            "wino4": ("Winograd F(4x4,3x3) 3x3 'same' convs with >= 128 input channels (conv1 fwd + data grad at "
                      "r = 64..256); FLOPs = its 36 multiplies per 4x4 tile and channel pair (1/4 of the direct "
                      "conv's)"),
            "direct": ("direct implicit-GEMM kernels on the exact-fp32 MFMA (conv_gemm_lds / conv_row / convt_lds ...); "
                       "FLOPs = dense MACs x 2"),
            "direct_x3": ("direct implicit-GEMM kernels with split-bf16 products (conv_gemm_x3 / convt_x3: transposed "
                          "conv0, its stride-2 data grad, the < 32-px layers); FLOPs = dense MACs x 2 (fp32-equivalent), "
                          "roof = bf16 MFMA peak / 6"),
        }
        traffic, traffic_src = pmc_traffic()
        parts = {k: part(s["kinds"][k], kinds.get(k, k), k) for k in sorted(s["kinds"])}
        dom = max(parts, key=lambda k: parts[k]["ms_per_step"]) if parts else None
        equiv = s["equiv_flops"] / s["seconds"] / 1e12 if s["seconds"] > 0 else 0.0
        roofline = {"bound": "mfma", "achieved": round(achieved, 3), "peak": round(peak_blend, 2), "unit": "TFLOP/s",
                    "frac": round(ideal / s["seconds"], 4) if s["seconds"] > 0 else 0.0, "traffic": traffic,
                    "traffic_source": traffic_src,
                    "frac_basis": "executed fp32 products (Winograd: its 16 / 36 multiplies per 2x2 / 4x4 tile and "
                                  "channel pair; split-bf16 direct convs: dense MACs x 2) against each launch's "
                                  "instruction peak (fp32 MFMA 157.3; split-bf16 = bf16 MFMA 2516.6 / 6 = 419.4 "
                                  "fp32-equivalent TFLOP/s); peak = their FLOP-weighted blend",
                    "frac_of_fp32_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                    "dense_equiv_frac": round(equiv / FP32_MFMA_PEAK_TFLOPS, 4),
                    "dense_equiv_basis": "SURVEY 8(d) dense conv MACs x 2 per second / fp32 MFMA peak (above 1 is "
                                         "possible: Winograd executes 4/9 (F(2x2)) or 1/4 (F(4x4)) of the dense "
                                         "multiplies)",
                    "dominant_kernel": ({"part": dom, "frac": parts[dom]["frac"],
                                         "ms_per_step": parts[dom]["ms_per_step"]} if dom else None),
                    "kernel": "synthesis conv family (wino_kernel + wino4_kernel + the direct implicit-GEMM kernels)",
                    "launches": s["launches"],
                    "avg_launch_us": round(1e6 * s["seconds"] / max(s["launches"], 1), 2),
                    "alg_gflop_per_launch": round(s["flops"] / max(s["launches"], 1) / 1e9, 3),
                    "alg_bytes_per_launch": int(s["bytes"] / max(s["launches"], 1)),
                    "direct_equiv_tflops": round(equiv, 3),
                    "parts": parts,
                    "share_of_step_time": round(s["seconds"] / dt_r, 4),
                    "measured": f"HIP events around every launch, {args.roofline_steps} serialised steps after the "
                                f"timed region"}

    selfcheck = None
    if world.world_size > 1:
        selfcheck = dist_selfcheck(G, clip, finder.id_loss, world, dev, finder.temp_shapes, args.resolution,
                                   args.batch)
    if world.rank != 0:
        return
    out = {
        "metric": METRIC,
        "value": round(2 * seeds / dt, 3),
        "unit": "images/s",
        "n_gpus": world.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * dt / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded config-f weights, S ~ N(1, 0.5) for 129 seeds, seeded CLIP/IR-SE50)",
        "config": {"workload": "find_direction step: 2x StyleGAN2 S-space synthesis fwd + 1 bwd (HIP), "
                               f"CLIP ViT-B/32 fwd/bwd ({'HIP' if args.clip_impl == 'hip' else 'PyTorch-ROCm'}), "
                               f"IR-SE50 fwd/bwd ({'HIP' if args.id_impl == 'hip' else 'PyTorch-ROCm'}), SGD",
                   "resolution": args.resolution, "batch_per_gpu": args.batch,
                   "global_batch": args.batch * world.world_size, "seeds_per_sec": round(seeds / dt, 3),
                   "n_seeds": n_seeds, "seeds_per_gpu": n_seeds / world.world_size,
                   "parallelism": f"dp{world.world_size}", "clip_type": args.clip_type, "clip_impl": args.clip_impl, "id_impl": args.id_impl,
                   "batched_loss_pairs": finder.batch_losses, "landmarks_loss_coef": 0,
                   "conv_products": args.conv_products, "vit_products": args.vit_products,
                   "irse_products": "x3" if irse_hip.X3 else "fp32",
                   "direction_finite": finite, "world_size": world.world_size, "backend": world.backend,
                   "launcher": (os.environ.get("SMC_BENCH_LAUNCHER", "torch.distributed.run")
                                if world.world_size > 1 else None),
                   "ranks_share_gpu": world.world_size > 1 and os.environ.get("SMC_SHARE_GPU") == "1"},
        "roofline": roofline,
        "cpu_baseline": None,
        "parity": None,
    }
    if selfcheck is not None:
        out["parity"] = selfcheck
    if world.world_size == 1 and not args.no_cpu_baseline:
        threads, info = host_cpus()
        if args.cpu_threads > 0:
            threads = args.cpu_threads
        out["cpu_baseline"], delta_ref = cpu_baseline(args.resolution, args.cpu_batch, args.cpu_iters, threads, info)
        try:
            out["parity"] = direction_parity(G, clip, finder.id_loss, args.resolution, args.cpu_batch,
                                             args.cpu_iters, delta_ref, dev, finder.temp_shapes)
        except Exception as e:  # keep the bench line; the failure is reported in it
            out["parity"] = {"error": f"{type(e).__name__}: {e}"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
