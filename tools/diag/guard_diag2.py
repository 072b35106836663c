"""Replays the test_gpu_published sequence with the guard flag printed at each stage."""
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
    strain = np.array([0.11, -0.07, 0.04], np.float32)
    g = devgraph.convert_mesh_to_graph(torch.from_numpy(pts).to(dev), torch.from_numpy(faces).to(dev), strain,
                                       torch.from_numpy(lab).to(dev))
    with torch.no_grad():
        y = model(g).local_stress.clone()
    cap = CapturedForward(model, g)
    y_r = cap(strain).clone()
    print(row[0], "equal", torch.equal(y, y_r), "flag", int(cap.flag.item()), flush=True)
    strain2 = np.array([-0.05, 0.12, -0.02], np.float32)
    g.mean_stress = torch.ones(sample.num_nodes, 3, device=dev) * torch.from_numpy(strain2).to(dev)
    with torch.no_grad():
        y2 = model(g).local_stress.clone()
    print(row[0], "equal2", torch.equal(cap(strain2), y2), "flag", int(cap.flag.item()), flush=True)
    yz = cap(np.zeros(3, np.float32))
    torch.cuda.synchronize()
    print(row[0], "zeros: flag", int(cap.flag.item()), "ms nz", int(torch.count_nonzero(cap.mean_stress)),
          "y nz", int(torch.count_nonzero(yz)), flush=True)
    yz = cap(np.zeros(3, np.float32))
    torch.cuda.synchronize()
    print(row[0], "zeros again: flag", int(cap.flag.item()), "y nz", int(torch.count_nonzero(yz)), flush=True)
