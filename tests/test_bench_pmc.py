"""bench.py takes PMC traffic only from a profiles/ file measured on its own tree:
a file whose "_meta" tree differs is ignored and the line says why, so frac_pmc never prices a
kernel's launches with another tree's bytes."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT)]

import bench  # noqa: E402

NAME = "void edge_fwd_coop_kernel<true, true, false>(int, ...)"


def _write(d: Path, name: str, tree: str, total: float) -> Path:
    (d / "profiles").mkdir(exist_ok=True)
    p = d / "profiles" / name
    p.write_text(json.dumps({"_meta": {"tree": tree}, NAME: {"total": total}}))
    return p


def test_pmc_file_of_another_tree_is_ignored(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    _write(tmp_path, "r07_pmc_traffic.json", "aaaa", 1.0e9)
    path, reason = bench.pmc_file("bbbb")
    assert path is None
    assert "bbbb" in reason and "aaaa" in reason
    assert bench.load_pmc(True, path) == {}


def test_pmc_file_of_this_tree_is_used(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    _write(tmp_path, "r08_pmc_traffic.json", "aaaa", 2.0e9)           # newer, but another tree
    good = _write(tmp_path, "r07_pmc_traffic.json", "bbbb", 1.5e9)
    path, reason = bench.pmc_file("bbbb")
    assert path == good and reason is None
    assert bench.load_pmc(True, path)["edge_fwd"] == 1_500_000_000


def test_no_pmc_file(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    path, reason = bench.pmc_file("bbbb")
    assert path is None and "no profiles" in reason


def test_roofline_without_traffic_has_no_pmc_fraction():
    work = {"edge_fwd": ([(1e9, bench.PEAK_FP32_MFMA)], 1.0e9)}
    r = bench.roofline("edge_fwd", work, {"edge_fwd": 2e-4}, {"edge_fwd": 2e-3}, 8e-3, {}, {"edge_fwd": 10}, None)
    assert r["traffic"] is None and r["frac_pmc"] is None and r["traffic_source"] is None


def test_sq_counters_only_from_this_tree(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    (tmp_path / "profiles").mkdir()
    rec = {"_meta": {"tree": "aaaa"}, "kernels": [{"kernel": NAME, "mfma_busy_at_2.4GHz": 0.42}]}
    (tmp_path / "profiles" / "r09_sq.json").write_text(json.dumps(rec))
    path, reason = bench.sq_file("bbbb")
    assert path is None and "bbbb" in reason
    path, reason = bench.sq_file("aaaa")
    assert reason is None and bench.load_sq(path) == {"edge_fwd": 0.42}


def test_edge_backward_bytes_follow_the_gz1e_variant():
    """The edge backward's algorithmic bytes drop one E-row stream (E x 512 B) when gz1e is formed by the
    P/Q gather backward from gC - gz1m instead of being stored (engine variant gz1e_from_gc)."""
    N, E, S, slab = 40328, 239744, 10, 256 * (128 * 128 + 128) * 4
    with_sum = bench.kernel_work(False, N, E, S, slab, True, e_sum=True)["edge_bwd"][1]
    stored = bench.kernel_work(False, N, E, S, slab, True, e_sum=False)["edge_bwd"][1]
    assert stored - with_sum == E * 128 * 4
    # the unfused edge backward does not depend on it
    assert (bench.kernel_work(False, N, E, S, slab, False, e_sum=True)["edge_bwd"]
            == bench.kernel_work(False, N, E, S, slab, False, e_sum=False)["edge_bwd"])


def test_compulsory_bytes_of_the_edge_forward_at_config_2():
    """frac_compulsory prices each gathered P / Q row once per node: at config 2 (N = 40,328,
    E = 239,744) the edge forward's 7 streamed rows per edge + 4 gathered rows per node + the int32
    src / dst come to 943.8 MB per launch (roofline table), against 1,352.2 MB with the
    gathers priced per edge."""
    N, E, S, slab = 40328, 239744, 10, 256 * (128 * 128 + 128) * 4
    work = bench.kernel_work(False, N, E, S, slab, True, e_sum=True)
    comp = bench.compulsory_bytes(work, N, E)
    assert round(work["edge_fwd"][1] / 1e6, 1) == 1352.2
    assert round(comp["edge_fwd"] / 1e6, 1) == 943.8
    assert comp["edge_bwd"] == work["edge_bwd"][1] - (E - N) * 512
    assert comp["node_net"] == work["node_net"][1]
    r = bench.roofline("edge_fwd", work, {"edge_fwd": 2e-4}, {"edge_fwd": 2e-3}, 8e-3, {}, {"edge_fwd": 10}, None, comp)
    assert r["frac_compulsory"] == round(comp["edge_fwd"] / 2e-4 / bench.PEAK_HBM, 4) < r["frac_gather_priced"]


def test_headline_frac_is_the_compulsory_fraction():
    """roofline.frac = bytes_compulsory_per_launch / avg_launch / 8 TB/s (0.61 at
    config 2's 192.5 us launches), the per-edge-priced figure only as frac_gather_priced (0.88) and
    SURVEY §8(d)'s reads-only formula (24 L E + 8 E = 740 MB) as frac_reads_only; with PMC bytes of the
    same tree, frac_pmc and their ratio to the compulsory bytes."""
    N, E, S, slab = 40328, 239744, 10, 256 * (128 * 128 + 128) * 4
    work = bench.kernel_work(False, N, E, S, slab, True, e_sum=True)
    comp = bench.compulsory_bytes(work, N, E)
    t = 192.5e-6
    ro = bench.reads_only_bytes("edge_fwd", E)
    assert round(ro / 1e6, 1) == 738.4
    assert bench.reads_only_bytes("segment_sum", E) is None
    pmc = {"edge_fwd": 905_200_000}
    r = bench.roofline("edge_fwd", work, {"edge_fwd": t}, {"edge_fwd": 8 * t}, 8e-3, pmc, {"edge_fwd": 24}, None,
                       comp, ro)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s"
    assert r["frac"] == round(comp["edge_fwd"] / t / 8e12, 4) == r["frac_compulsory"]
    assert abs(r["frac"] - 0.6129) < 2e-4
    assert r["bytes_per_launch"] == r["bytes_compulsory_per_launch"] == comp["edge_fwd"]
    assert r["achieved"] == round(comp["edge_fwd"] / t / 1e9, 2)
    assert r["frac_gather_priced"] == round(work["edge_fwd"][1] / t / 8e12, 4) > r["frac"]
    assert r["frac_reads_only"] == round(ro / t / 8e12, 4) < r["frac"]
    assert r["frac_pmc"] == round(905_200_000 / t / 8e12, 4)
    assert r["pmc_over_compulsory"] == round(905_200_000 / comp["edge_fwd"], 4)


def test_counter_files_are_per_config(tmp_path, monkeypatch):
    """Configs 3-5 take their counters from profiles/rNN_pmc_traffic_cC.json / rNN_sq_cC.json of the same
    tree; the main line's (config 2) file never prices another config's launches."""
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    main = _write(tmp_path, "r06_pmc_traffic.json", "aaaa", 1.0e9)
    c5 = _write(tmp_path, "r06_pmc_traffic_c5.json", "aaaa", 3.0e9)
    assert bench.pmc_file("aaaa", config=2) == (main, None)
    assert bench.pmc_file("aaaa", config=5) == (c5, None)
    path, reason = bench.pmc_file("aaaa", config=3)
    assert path is None and "_c3" in reason
    assert bench.load_pmc(True, c5)["edge_fwd"] == 3_000_000_000


def test_pmc_names_cover_the_shipped_instantiations(tmp_path):
    """The counter lookup finds the kernels the engine launches: the inference edge forward (config 5 runs no
    cooperative edge forward) and the Wc pass's <RES, LN> instantiation."""
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({
        "_meta": {"tree": "aaaa"},
        "void edge_fwd_infer_kernel<true, true, true>(int, ...)": {"total": 1.75e9},
        "void edge_gout_wc_kernel<true, true>(float const*, ...)": {"total": 6.5e8},
        "void edge_gout_wc_kernel<false, true>(float const*, ...)": {"total": 1.0},
        "void gemm_sum2_coop_kernel<true, true>(int, ...)": {"total": 1.06e8}}))
    pmc = bench.load_pmc(True, p)
    assert pmc["edge_fwd"] == 1_750_000_000
    assert pmc["edge_gout"] == 650_000_000
    assert pmc["gemm_sum2"] == 106_000_000
