"""Diagnose slow first GPU find_direction test: periodic stack dumps + phase timing."""
import faulthandler
import sys
import time

sys.path.insert(0, ".")
faulthandler.dump_traceback_later(30, repeat=True, file=sys.stderr)
t0 = time.time()
import torch  # noqa: E402
from tests import test_gpu_find_direction as T  # noqa: E402
print("import", time.time() - t0, flush=True)
for name, args in [("tiny", (32, 512, 5, 2, 4)), ("tiny-again", (32, 512, 5, 2, 4))]:
    t0 = time.time()
    o, g = T._run_pair(*args[:2], n_items=args[2], bs=args[3], iters=args[4])
    torch.cuda.synchronize()
    print(name, time.time() - t0, flush=True)
