"""Per-tensor distance of the parameters after the resumed second Adam step (tests/test_gpu_checkpoint.py)
from the reference's, for the engine variants named on the command line (name=value, PDG_AB-style)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "p-div-gnn_amd")
from golden_io import GOLDEN  # noqa: E402
from gpu_common import golden_batch, rel  # noqa: E402
from test_gpu_checkpoint import _loaded_model  # noqa: E402


def run(over):
    from gnn_local_stress import models
    from pdg.trainer import Trainer
    case = np.load(GOLDEN / "ref_checkpoint_case.npz", allow_pickle=False)
    _, batch = golden_batch("batch3_div")
    m, _ = _loaded_model()
    for k, v in over.items():
        setattr(m._engine_for(batch.pos.device), k, v)
    tr = Trainer(m, lr=0.5, divergence=True, divergence_penalty=10.0)
    models.load_model_checkpoint(m, (GOLDEN / "ref_checkpoint.pth").as_posix(), optimizer=tr)
    tr.step(batch)
    torch.cuda.synchronize()
    d = {n: rel(p, case[f"param_after_step2.{n}"]) for n, p in m.state_dict().items()}
    return d


if __name__ == "__main__":
    over = {}
    for a in sys.argv[1:]:
        k, v = a.split("=")
        over[k] = bool(int(v))
    d = run(over)
    for n, v in sorted(d.items(), key=lambda kv: -kv[1])[:6]:
        print(f"{over} {n:40s} {v:.3e}")
