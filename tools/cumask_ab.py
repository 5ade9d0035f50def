"""Does confining the prefetch stream (the next iteration's original-image synthesis) to a subset of the CUs
shorten the step?  The loss networks (latency-bound small kernels) run beside it; a CU-masked prefetch stream
(hipExtStreamCreateWithCUMask) leaves the rest of the chip to them.  Diagnostic only.

    python tools/cumask_ab.py --variants none,c75,i75,c50 [--rounds 2] [--steps 10]
c75 / c50: the first 75 / 50 % of the mask bits; i75: 3 of every 4 bits (interleaved).  Each variant in a fresh
process (a process's streams map onto hardware queues in creation order).
"""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def masked_stream_factory(kind, ncu):
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ncu + 31) // 32
    bits = [False] * (32 * words)
    if kind.startswith("c"):
        k = int(ncu * int(kind[1:]) / 100)
        for i in range(k):
            bits[i] = True
    else:  # interleaved: 3 of every 4 (i75) or 1 of every 2 (i50)
        num, den = (3, 4) if kind == "i75" else (1, 2)
        for i in range(ncu):
            bits[i] = (i % den) < num
    mask = (ctypes.c_uint32 * words)(*[sum(1 << b for b in range(32) if bits[32 * w + b]) for w in range(words)])
    keep = []

    def factory(dev):
        h = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask rc={rc}")
        keep.append(h)
        return torch.cuda.ExternalStream(h.value, device=dev)
    return factory


def main():
    import torch
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    name = sys.argv[sys.argv.index("--variant") + 1]
    from stylemc_amd import _hip, synthetic, utils
    from stylemc_amd import find_direction as FD
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    G = FD.load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    clip = FD.build_clip_losses("small", dev, "a", "b", synthetic_weights=True)
    idl = IDLoss("a", device=dev, weights=None)
    ts = utils.get_temp_shapes(G)
    f = FD.DirectionFinder(G, styles, clip, idl, resolution=1024, batch_size=4, seed=0, temp_shapes=ts,
                           init_delta=FD.initial_delta(0, 0.01), n_epochs=1000)
    if name != "none":
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        f._pre = masked_stream_factory(name, ncu)(dev)
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        f.step()
    e.record()
    torch.cuda.synchronize()
    print(f"{name:8s} {s.elapsed_time(e) / steps:7.2f} ms/step", flush=True)


def driver():
    steps = sys.argv[sys.argv.index("--steps") + 1] if "--steps" in sys.argv else "10"
    names = sys.argv[sys.argv.index("--variants") + 1].split(",")
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2
    for r in range(rounds):
        for n in names:
            out = subprocess.run([sys.executable, "-u", __file__, "--variant", n, "--steps", steps],
                                 capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if "ms/step" in l]
            print(f"round {r} {line[-1] if line else 'FAILED ' + out.stderr[-400:]}", flush=True)
            if out.returncode != 0:
                sys.exit(out.returncode)


if __name__ == "__main__":
    if "--variants" in sys.argv:
        driver()
    else:
        main()
