"""Which torch (non-HIP-library) ops run per training step (GPU box): torch.profiler over 3 steps of
the config-2 bench workload, aten ops grouped by Python call site."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd")]

import torch  # noqa: E402


def main():
    import bench
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg.trainer import Trainer
    cfg = bench.CONFIGS[2]
    batch, _ = bench.build_batch(cfg, seed=69, device=torch.device("cuda"), indices=list(range(cfg["graphs"])))
    stats = bench.dataset_stats(batch)
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).cuda()
    tr = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        for _ in range(3):
            tr.step(batch)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_stack_n=4).table(sort_by="count", row_limit=40, max_name_column_width=40))


if __name__ == "__main__":
    main()
