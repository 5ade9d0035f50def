"""Which PyTorch (aten) ops does a find_direction step launch besides the HIP library?  torch.profiler
over a few steps, aten ops ranked by self GPU time.   python tools/aten_ops.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stylemc_amd import _hip, synthetic
    from stylemc_amd import find_direction as FD
    from stylemc_amd.id_loss import IDLoss
    _hip.load()
    dev = torch.device("cuda", 0)
    G = FD.load_generator("synthetic", 1024, dev)
    styles = synthetic.synthetic_styles(129, seed=0).to(dev)
    f = FD.DirectionFinder(G, styles, FD.build_clip_losses("small", dev, "a", "b", synthetic_weights=True), IDLoss("a", device=dev, weights=None),
                           resolution=1024, batch_size=4, seed=0, init_delta=FD.initial_delta(0, 0.01), n_epochs=1000)
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                                record_shapes=True) as prof:
        for _ in range(3):
            f.step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=60, max_name_column_width=40,
                                                             max_shapes_column_width=60))


if __name__ == "__main__":
    main()
