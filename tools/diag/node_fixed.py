"""Fixed cost of the node kernels: launch floor (a one-block kernel), each node kernel with ONE block
(N = 16: one tile, no contention) and with 256 blocks of one tile each (N = 4096)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd"), str(ROOT / "tools")]
import torch
import node_breakdown as nb
from pdg.lib import lib, stream_handle
dev = torch.device("cuda:0")
s = stream_handle(dev)
cus = torch.cuda.get_device_properties(dev).multi_processor_count
flag = torch.ones(1, dtype=torch.int32, device=dev)
y = torch.zeros(16, device=dev)
print("launch floor (1-block kernel):", round(nb.time_launch(lambda: lib.pdg_zero_unless(flag.data_ptr(), y.data_ptr(), 1, s), 50), 2), "us")
big = torch.zeros(256 * 512 * 4, device=dev)
print("launch floor (256 x 256-thread kernel):", round(nb.time_launch(lambda: lib.pdg_zero_unless(flag.data_ptr(), big.data_ptr(), big.numel(), s), 50), 2), "us")
for N in (16, 32, 64, 16 * cus, 32 * cus):
    ks = nb.kernels(N, s, cus)
    print(N, {k: round(nb.time_launch(fn, 30), 1) for k, (fn, _) in ks.items()}, flush=True)
