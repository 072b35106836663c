"""Per-step forward diagnostics of the HIP engine vs the golden latents (debug aid)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd"), str(ROOT / "tests")]
import torch  # noqa: E402

from gpu_common import golden_batch, rel  # noqa: E402
from gnn_local_stress.models import EncodeProcessDecode  # noqa: E402
from pdg.engine import PARAM_NAMES  # noqa: E402
from pdg.plan import plan_for  # noqa: E402

for case in sys.argv[1:] or ["tiny_periodic"]:
    g, batch = golden_batch(case)
    steps = int(g["steps"])
    torch.manual_seed(69)
    m = EncodeProcessDecode(1, steps, latent_size=128, input_nodes_features_size=6, output_nodes_features_size=3,
                            **{k: v.float() for k, v in g["stats"].items()})
    m.load_state_dict(g["params"])
    m = m.to("cuda")
    eng = m._engine_for(torch.device("cuda"))
    P = {n: m.get_parameter(n).detach() for n in PARAM_NAMES}
    plan = plan_for(batch)
    y, ctx = eng.forward(P, m.stats_tensor("cuda"), plan, batch.pos, batch.mean_stress,
                         batch.nodes_types.reshape(-1).contiguous(), batch.edge_attr, steps, True, True, True)
    torch.cuda.synchronize()
    perm = plan.perm.long()
    for t in range(steps):
        d = ctx.per_step[t]
        if f"latent_x_{t}" in g:
            # per_step[t]['x'] = x_t = input of step t = latent after step t-1 (latent_x_{t-1}); golden latents
            # are the processor outputs of step t, so compare x_{t+1} where available
            pass
        xt = d["x"].cpu()
        et = d["e"].cpu()
        if t >= 1 and f"latent_x_{t-1}" in g:
            print(case, "step", t, "x_t rel", rel(xt, g[f"latent_x_{t-1}"]),
                  "e_t rel", rel(et, torch.from_numpy(g[f"latent_e_{t-1}"])[perm.cpu()]))
    print(case, "out rel", rel(y, g["out_scaled"]))
