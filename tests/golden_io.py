"""Load the reference-generated fixtures in tests/golden/*.npz."""
from pathlib import Path

import numpy as np
import torch

GOLDEN = Path(__file__).resolve().parent / "golden"
CASES = ("tiny_periodic", "batch3_div", "single_no_periodic", "batch2_div_s10")


def load(name: str) -> dict:
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    out = {k: z[k] for k in z.files}
    out["params"] = {k[6:]: torch.from_numpy(v) for k, v in out.items() if k.startswith("param.")}
    out["grads"] = {k[5:]: torch.from_numpy(v) for k, v in out.items() if k.startswith("grad.")}
    out["stats"] = {k[5:]: torch.from_numpy(v) for k, v in out.items() if k.startswith("stat.")}
    ptr = out["ptr"]
    ops = []
    for i in range(len(ptr) - 1):
        n = int(ptr[i + 1] - ptr[i])
        ops.append(torch.sparse_coo_tensor(torch.from_numpy(out[f"op_div_idx_{i}"]),
                                           torch.from_numpy(out[f"op_div_val_{i}"]), (n, 2 * n)).coalesce())
    out["op_divs"] = ops
    return out
