"""Diagnose the device-side zero-stress guard under HIP-graph replay (pdg/serve.py)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]
import numpy as np
import torch
import bench
from pdg import devgraph
from pdg.serve import CapturedForward
dev = torch.device("cuda:0")
for row in (bench.PUBLISHED_SWEEP[0], bench.PUBLISHED_SWEEP[-1]):
    sample, pts, faces, lab = bench.published_mesh(row[3], row[4])
    model = bench.published_model(dev, sample)
    g = devgraph.convert_mesh_to_graph(torch.from_numpy(pts).to(dev), torch.from_numpy(faces).to(dev),
                                       np.array([0.1, 0.2, 0.3], np.float32), torch.from_numpy(lab).to(dev))
    cap = CapturedForward(model, g)
    for ms in ([0.1, 0.2, 0.3], [0, 0, 0], [0.1, 0, 0], [0, 0, 0]):
        y = cap(np.array(ms, np.float32))
        torch.cuda.synchronize()
        print(row[0], ms, "flag", int(cap.flag.item()), "ms nonzero", int(torch.count_nonzero(cap.mean_stress)),
              "y nonzero", int(torch.count_nonzero(y)), flush=True)
    cap.mean_stress.zero_()
    y = cap._run()
    torch.cuda.synchronize()
    print(row[0], "eager zeros: flag", int(cap.flag.item()), "y nonzero", int(torch.count_nonzero(y)), flush=True)
